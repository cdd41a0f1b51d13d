// renderer.cpp — Renderer of the reference (render.cpp) for the compute path:
// OnInit creates the HIP context (InitDevice, render.cpp:49-147) and the scene
// and camera (the commented-out render.cpp:135-139); OnRender updates the camera,
// launches the path tracer over the whole frame through the C-ABI, reads back
// rgba8 and writes "NNN.png" (render.cpp:451-511); OnCompute loops frames with
// the same wall-clock logging (render.cpp:430-449).
#include "../../../include/wgt/renderer.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <iomanip>
#include <iostream>
#include <sstream>
#include <thread>
#include <vector>

#include "procedural.h"

namespace wgt {

bool Renderer::OnInit(bool hasWindow) {
  if (hasWindow) {
    std::cerr << "[GLFW] Could not open window! (the MI355X renderer is headless)" << std::endl;
    return false;
  }
  if (wgt_create(cfg_.device, &ctx_) != WGT_OK) {
    std::cerr << "[WebGPUTracer] Could not initialize HIP device: " << wgt_last_error(nullptr)
              << std::endl;
    return false;
  }
  std::cout << "[WebGPUTracer] HIP device " << cfg_.device << " ready" << std::endl;
  camera_ = Camera(ctx_, cfg_.spp);
  if (cfg_.fixed_seed) camera_.SetSeed(0);
  scene_ = Scene(ctx_, false);
  if (cfg_.scene != "cornell") {
    // mesh configs: light + Cornell walls + mesh (the two inner boxes removed)
    scene_.quads_.resize(5);
    if (cfg_.scene == "bunny" || cfg_.scene == "sponza") {
      std::vector<Triangle> tris;
      if (cfg_.scene == "bunny") procedural::Bunny(69451, 1, tris);
      else procedural::Sponza(262267, 1, tris);
      scene_.AddTriangles(tris);
    } else if (cfg_.scene.rfind("obj:", 0) == 0) {
      if (!scene_.LoadObj(cfg_.scene.c_str() + 4, COL_WHITE)) return false;
    } else {
      std::cerr << "[WebGPUTracer] unknown scene " << cfg_.scene << std::endl;
      return false;
    }
  }
  return scene_.InitBuffers(ctx_);
}

bool Renderer::OnCompute(uint32_t start_frame, uint32_t end_frame) {
  std::cout << "[WebGPUTracer] Running compute pass ..." << std::endl;
  auto start = std::chrono::system_clock::now();
  bool success = false;
  if (cfg_.batch <= 1) {
    for (uint32_t i = start_frame - 1; i < end_frame; ++i) success = OnRender(i);
  } else {
    for (uint32_t i = start_frame - 1; i < end_frame; i += cfg_.batch)
      success = OnRenderBatch(i, std::min(cfg_.batch, end_frame - i));
  }
  auto end = std::chrono::system_clock::now();
  double elapsed = (double)std::chrono::duration_cast<std::chrono::milliseconds>(end - start).count();
  std::cout << "[WebGPUTracer] Finished: " << elapsed * 0.001 << "(sec)s" << std::endl;
  return success;
}

bool Renderer::OnRender(uint32_t frame) {
  auto start = std::chrono::system_clock::now();
  float t = (float)frame / (float)cfg_.max_frame;
  float aspect = (float)cfg_.width / (float)cfg_.height;
  if (cfg_.fixed_seed) camera_.SetSeed(frame);
  camera_.Update(t, aspect);
  image_.assign((size_t)cfg_.width * cfg_.height * 4, 0);
  int rc = wgt_render_tile(ctx_, &camera_.GetParam(), cfg_.width, cfg_.height, 0, 0, cfg_.width,
                           cfg_.height, image_.data(), nullptr, nullptr, nullptr);
  if (rc != WGT_OK) {
    std::cerr << "[WebGPUTracer] render failed: " << wgt_last_error(ctx_) << std::endl;
    return false;
  }
  std::ostringstream sout;
  sout << std::setw(3) << std::setfill('0') << frame;
  if (cfg_.write_png) {
    std::string output_file = cfg_.out_dir + "/" + sout.str() + ".png";
    if (wgt_write_png(output_file.c_str(), image_.data(), cfg_.width, cfg_.height) != WGT_OK) {
      std::cerr << "[WebGPUTracer] Image output failed." << std::endl;
      return false;
    }
  }
  auto end = std::chrono::system_clock::now();
  double elapsed = (double)std::chrono::duration_cast<std::chrono::milliseconds>(end - start).count();
  std::cout << "[" << sout.str() << "]: " << elapsed * 0.001 << "(sec)s" << std::endl;
  return true;
}

bool Renderer::OnRenderBatch(uint32_t first, uint32_t n) {
  auto start = std::chrono::system_clock::now();
  float aspect = (float)cfg_.width / (float)cfg_.height;
  std::vector<uint32_t> seeds(n);
  for (uint32_t j = 0; j < n; ++j) {  // the seed OnRender would use for frame first + j
    if (cfg_.fixed_seed) camera_.SetSeed(first + j);
    camera_.Update((float)(first + j) / (float)cfg_.max_frame, aspect);
    seeds[j] = camera_.GetParam().seed;
  }
  const size_t frame_bytes = (size_t)cfg_.width * cfg_.height * 4;
  std::vector<uint8_t> images(frame_bytes * n);
  if (wgt_render_frames(ctx_, &camera_.GetParam(), cfg_.width, cfg_.height, seeds.data(), n, images.data(),
                        nullptr) != WGT_OK) {
    std::cerr << "[WebGPUTracer] render failed: " << wgt_last_error(ctx_) << std::endl;
    return false;
  }
  if (cfg_.write_png) {
    // the batch's PNGs are encoded concurrently by at most hardware_concurrency (and 16)
    // writers, each taking the next frame of the batch
    std::vector<int> rc(n, WGT_OK);
    std::atomic<uint32_t> next{0};
    const uint32_t hw = std::max(1u, std::thread::hardware_concurrency());
    const uint32_t n_writers = std::min({n, hw, 16u});
    std::vector<std::thread> writers;
    for (uint32_t k = 0; k < n_writers; ++k) {
      writers.emplace_back([&] {
        for (uint32_t j = next++; j < n; j = next++) {
          std::ostringstream sout;
          sout << std::setw(3) << std::setfill('0') << first + j;
          const std::string output_file = cfg_.out_dir + "/" + sout.str() + ".png";
          rc[j] = wgt_write_png(output_file.c_str(), images.data() + frame_bytes * j, cfg_.width, cfg_.height);
        }
      });
    }
    for (auto& t : writers) t.join();
    if (std::any_of(rc.begin(), rc.end(), [](int r) { return r != WGT_OK; })) {
      std::cerr << "[WebGPUTracer] Image output failed." << std::endl;
      return false;
    }
  }
  image_.assign(images.end() - frame_bytes, images.end());
  auto end = std::chrono::system_clock::now();
  double elapsed = (double)std::chrono::duration_cast<std::chrono::milliseconds>(end - start).count();
  std::cout << "[" << first << "-" << first + n - 1 << "]: " << elapsed * 0.001 << "(sec)s" << std::endl;
  return true;
}

void Renderer::OnFinish() {
  scene_.Release();
  camera_.Release();
  if (ctx_) {
    wgt_destroy(ctx_);
    ctx_ = nullptr;
  }
}

}  // namespace wgt
