// camera.cpp — Camera::Update of the reference (camera.cpp:64-70): fixed pose
// origin (278,278,-800), target (278,278,0), fovy 40; `t` is ignored exactly as
// in the reference.  The seed is RandSeed() (std::random_device, util.h:43-47)
// unless a fixed seed was set.
#include "../../../include/wgt/camera.h"

#include <cstring>

namespace wgt {

void Camera::Update(float t, float aspect) {
  (void)t;
  Point3 origin = vec3(278, 278, -800);
  Point3 target = vec3(278, 278, 0);
  float fovy = 40.0f;
  CameraParam param(origin, target, aspect, fovy, spp_, fixed_seed_ ? seed_ : RandSeed());
  std::memcpy(&param_, &param, sizeof(param_));
}

}  // namespace wgt
