// camera.h — Camera mirroring src/include/camera.h of the reference.  The uniform
// buffer + bind group (camera.h:8-49) become a host-side 48-B CameraParam that is
// passed to the C-ABI launcher by value.
#pragma once

#include <cstdint>
#include <random>

#include "../wgt_api.h"
#include "vec.h"

namespace wgt {

// util.h:43-47 RandSeed(): std::random_device
inline uint32_t RandSeed() {
  std::random_device rnd;
  return rnd();
}

class Camera {
 public:
  Camera() = default;
  explicit Camera(wgt_ctx* ctx, uint32_t spp) : ctx_(ctx), spp_(spp) {}  // camera.cpp:5-14
  wgt_ctx* Context() const { return ctx_; }

  // camera.h:19-31 — byte-identical to wgt_camera_param
  struct CameraParam {
    Point3 origin;
    float dummy{};
    Point3 target;
    float dummy1{};
    float aspect;
    float fovy;
    uint32_t spp;
    uint32_t seed;
    CameraParam(vec3 o, vec3 t, float a, float f, uint32_t s, uint32_t sd)
        : origin(o), target(t), aspect(a), fovy(f), spp(s), seed(sd) {}
  };

  // camera.cpp:64-70.  The reference seeds every frame from std::random_device;
  // a fixed seed (SetSeed) makes frames reproducible (parity tests, benchmarks).
  void Update(float t, float aspect);
  void SetSeed(uint32_t seed) { fixed_seed_ = true; seed_ = seed; }
  void UseRandomSeed() { fixed_seed_ = false; }
  const wgt_camera_param& GetParam() const { return param_; }
  uint32_t spp() const { return spp_; }
  void Release() {}  // camera.cpp:16-21: nothing on the device to free

 private:
  wgt_ctx* ctx_ = nullptr;
  uint32_t spp_ = 1;
  bool fixed_seed_ = false;
  uint32_t seed_ = 0;
  wgt_camera_param param_{};
};

static_assert(sizeof(Camera::CameraParam) == 48, "CameraParam must stay 48 bytes");
static_assert(sizeof(wgt_camera_param) == 48, "wgt_camera_param must stay 48 bytes");

}  // namespace wgt
