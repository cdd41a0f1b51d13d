// renderer.h — Renderer mirroring src/include/renderer.h of the reference for the
// compute (path-tracing) path: OnInit / OnCompute / OnRender / OnFinish with the
// same meaning and bool returns.  The WebGPU device/queue/pipeline become a
// wgt_ctx (HIP device + stream); the windowed raster demo (OnFrame, swap chain,
// depth buffer, GUI) is out of scope.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../wgt_api.h"
#include "camera.h"
#include "scene.h"

namespace wgt {

struct RendererConfig {
  uint32_t width = 512;     // renderer.h:53
  uint32_t height = 512;    // renderer.h:54
  uint32_t max_frame = 1;   // renderer.h:55
  uint32_t spp = 1000;      // renderer.h:56
  int device = 0;
  std::string scene = "cornell";  // cornell | bunny | sponza | obj:<path>
  std::string out_dir = ".";
  bool fixed_seed = false;        // seed = frame index instead of RandSeed()
  bool write_png = true;
  uint32_t batch = 1;             // frames per launch in OnCompute (wgt_render_frames); 1 = reference loop
};

class Renderer {
 public:
  Renderer() = default;
  explicit Renderer(const RendererConfig& cfg) : cfg_(cfg) {}
  ~Renderer() { OnFinish(); }

  bool OnInit(bool hasWindow);                              // render.cpp:12-45
  bool OnCompute(uint32_t start_frame, uint32_t end_frame); // render.cpp:430-449
  bool OnRender(uint32_t frame);                            // render.cpp:451-511
  // OnRender for frames [first, first + n) in one launch (frame f -> "fff.png")
  bool OnRenderBatch(uint32_t first, uint32_t n);
  void OnFinish();                                          // render.cpp:599-650
  bool IsRunning() { return false; }  // no window on the GPU box

  const std::vector<uint8_t>& LastImage() const { return image_; }
  const wgt_stats& LastStats() const { return stats_; }
  wgt_ctx* Context() { return ctx_; }

 private:
  RendererConfig cfg_;
  wgt_ctx* ctx_ = nullptr;
  Camera camera_{};
  Scene scene_{};
  std::vector<uint8_t> image_;
  wgt_stats stats_{};
};

}  // namespace wgt
