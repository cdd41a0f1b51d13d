// scene.h — Scene mirroring src/include/scene.h of the reference.  The WebGPU
// buffers/bind groups (scene.h:10-51) become one upload through the C-ABI
// (wgt_upload_scene), which also builds the BVH over triangles.
#pragma once

#include <string>
#include <vector>

#include "../wgt_api.h"
#include "objects.h"

namespace wgt {

class Scene {
 public:
  Scene() = default;
  // scene.cpp:14-36: the Cornell box.  With upload=true the buffers go straight
  // to the device like Scene::InitBuffers (scene.cpp:161-165).
  explicit Scene(wgt_ctx* ctx, bool upload = true);

  // scene.cpp:56-65 (private and unused in the reference; public here so the
  // mesh configs can use it).  Returns false with Error(...) on parse failure
  // instead of exit(1) (scene.cpp:78) — no process exit inside a library.
  bool LoadObj(const char* file_path, Color3 color, vec3 translation = vec3(0, 0, 0),
               bool emissive = false);
  // Append already-built triangles (procedural stand-ins).
  void AddTriangles(const std::vector<Triangle>& tris);

  // Scene::InitBuffers (scene.cpp:161-165): pack + upload (+ BVH).
  bool InitBuffers(wgt_ctx* ctx);
  void Release();  // scene.cpp:41-50 (idempotent)

  // CreateQuadBuffer / CreateSphereBuffer / CreateTriangleBuffer packing
  // (scene.cpp:223-271, 276-306, 170-218) into the reference byte layouts.
  std::vector<wgt_quad> PackQuads(const std::vector<Quad>& quads) const;
  std::vector<wgt_sphere> PackSpheres() const;
  std::vector<wgt_triangle> PackTriangles() const;

  std::vector<Triangle> tris_;
  std::vector<Quad> lights_;
  std::vector<Quad> quads_;
  std::vector<Sphere> spheres_;
  uint32_t tri_stride_ = 20 * 4;   // scene.h:45
  uint32_t quad_stride_ = 24 * 4;  // scene.h:46
  uint32_t sphere_stride_ = 8 * 4; // scene.h:47

 private:
  bool LoadVertices(const char* file_path, std::vector<Vertex>& vertices);
  wgt_ctx* ctx_ = nullptr;
  bool uploaded_ = false;
};

}  // namespace wgt
