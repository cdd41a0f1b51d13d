// main.cpp — CLI mirroring src/main.cpp of the reference:
//   wgt_tracer [--frame start end] [--width W] [--height H] [--spp N]
//              [--scene cornell|bunny|sponza|obj:<path>] [--device D] [--out DIR]
//              [--fixed-seed] [--no-png] [--batch B]
// The reference parses only `--frame s e` (main.cpp:21-26) with W=H=512,
// SPP=1000 compiled in (renderer.h:53-56); those stay the defaults.
#include <cstdlib>
#include <cstring>
#include <iostream>

#include "../../include/wgt/renderer.h"

int main(int argc, char* argv[]) {
  std::cout << "[WebGPUTracer] Starting WebGPUTracer (_)=---=(_)" << std::endl;
  wgt::RendererConfig cfg;
  uint32_t start_frame = 1, end_frame = 1;
  for (int i = 1; i < argc; ++i) {
    auto need = [&](int k) {
      if (i + k >= argc) {
        std::cerr << "[WebGPUTracer] missing value for " << argv[i] << std::endl;
        std::exit(2);
      }
    };
    if (!std::strcmp(argv[i], "--frame")) { need(2); start_frame = (uint32_t)atoi(argv[i + 1]); end_frame = (uint32_t)atoi(argv[i + 2]); i += 2; }
    else if (!std::strcmp(argv[i], "--width")) { need(1); cfg.width = (uint32_t)atoi(argv[++i]); }
    else if (!std::strcmp(argv[i], "--height")) { need(1); cfg.height = (uint32_t)atoi(argv[++i]); }
    else if (!std::strcmp(argv[i], "--spp")) { need(1); cfg.spp = (uint32_t)atoi(argv[++i]); }
    else if (!std::strcmp(argv[i], "--scene")) { need(1); cfg.scene = argv[++i]; }
    else if (!std::strcmp(argv[i], "--device")) { need(1); cfg.device = atoi(argv[++i]); }
    else if (!std::strcmp(argv[i], "--out")) { need(1); cfg.out_dir = argv[++i]; }
    else if (!std::strcmp(argv[i], "--fixed-seed")) { cfg.fixed_seed = true; }
    else if (!std::strcmp(argv[i], "--no-png")) { cfg.write_png = false; }
    else if (!std::strcmp(argv[i], "--batch")) { need(1); cfg.batch = (uint32_t)atoi(argv[++i]); }
    else { std::cerr << "[WebGPUTracer] unknown option " << argv[i] << std::endl; return 2; }
  }
  if (start_frame < 1 || end_frame < start_frame) {
    std::cerr << "[WebGPUTracer] bad frame range" << std::endl;
    return 2;
  }
  wgt::Renderer renderer(cfg);
  if (!renderer.OnInit(false)) {
    std::cerr << "[WebGPUTracer] (_)=--.. Something went wrong" << std::endl;
    return 1;
  }
  if (!renderer.OnCompute(start_frame, end_frame)) {
    std::cerr << "[WebGPUTracer] (_)=--.. Something went wrong" << std::endl;
    return 1;
  }
  renderer.OnFinish();
  std::cout << "[WebGPUTracer] (_)=---=(_) WebGPUTracer Finished" << std::endl;
  return 0;
}
