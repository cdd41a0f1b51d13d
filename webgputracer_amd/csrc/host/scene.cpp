// scene.cpp — Scene of the reference (src/scene.cpp) on top of the C-ABI:
// Cornell-box construction, OBJ loading, packing into the reference GPU byte
// layouts, and the upload that replaces Scene::InitBuffers.
#include "../../../include/wgt/scene.h"

#include <cstdio>
#include <cstring>
#include <iostream>

#include "obj_loader.h"

namespace wgt {

// scene.cpp:14-36
Scene::Scene(wgt_ctx* ctx, bool upload) : ctx_(ctx) {
  lights_.emplace_back(Point3(213, 554, 227), vec3(130, 0, 0), vec3(0, 0, 105), COL_LIGHT, true);
  auto cb = CornellBox();
  cb.PushToQuads(quads_);
  auto box1 = Box(Point3(0, 0, 0), Point3(165, 330, 165), COL_WHITE);
  box1.RotateY(15);
  box1.Translate(vec3(265, 0, 295));
  auto box2 = Box(Point3(0, 0, 0), Point3(165, 165, 165), COL_WHITE);
  box2.RotateY(-18);
  box2.Translate(vec3(130, 0, 65));
  box1.PushQuads(quads_);
  box2.PushQuads(quads_);
  spheres_.emplace_back(Point3(0, 0, 0), 0, COL_ZERO);  // dummy sphere, scene.cpp:31
  if (upload && ctx_) InitBuffers(ctx_);
}

// scene.cpp:56-65
bool Scene::LoadObj(const char* file_path, Color3 color, vec3 translation, bool emissive) {
  std::vector<Vertex> vertices;
  if (!LoadVertices(file_path, vertices)) return false;
  for (size_t i = 0; i < vertices.size() / 3; ++i) {
    auto v0 = vertices[i * 3].Translate(translation);
    auto v1 = vertices[i * 3 + 1].Translate(translation);
    auto v2 = vertices[i * 3 + 2].Translate(translation);
    tris_.emplace_back(v0, v1, v2, color, emissive);
  }
  return true;
}

// scene.cpp:70-131 (tinyobjloader replaced by the own loader, obj_loader.cpp)
bool Scene::LoadVertices(const char* file_path, std::vector<Vertex>& vertices) {
  std::string err, warn;
  if (!obj::LoadTriangulated(file_path, vertices, err, warn)) {
    std::cerr << "[WebGPUTracer] ObjReader: " << err << std::endl;
    return false;
  }
  if (!warn.empty()) std::cout << "[WebGPUTracer] ObjReader: " << warn << std::endl;
  return true;
}

void Scene::AddTriangles(const std::vector<Triangle>& tris) {
  tris_.insert(tris_.end(), tris.begin(), tris.end());
}

// scene.cpp:223-271
std::vector<wgt_quad> Scene::PackQuads(const std::vector<Quad>& quads) const {
  std::vector<wgt_quad> out(quads.size());
  const float dummy = 1.0f;
  for (size_t i = 0; i < quads.size(); ++i) {
    const Quad& q = quads[i];
    wgt_quad& o = out[i];
    o.pos[0] = q.q_[0]; o.pos[1] = q.q_[1]; o.pos[2] = q.q_[2]; o.pos[3] = dummy;
    o.right[0] = q.right_[0]; o.right[1] = q.right_[1]; o.right[2] = q.right_[2]; o.right[3] = dummy;
    o.up[0] = q.up_[0]; o.up[1] = q.up_[1]; o.up[2] = q.up_[2]; o.up[3] = dummy;
    o.norm[0] = q.norm_[0]; o.norm[1] = q.norm_[1]; o.norm[2] = q.norm_[2]; o.norm[3] = dummy;
    o.w[0] = q.w_[0]; o.w[1] = q.w_[1]; o.w[2] = q.w_[2];
    o.d = q.d_;
    o.col[0] = q.color_[0]; o.col[1] = q.color_[1]; o.col[2] = q.color_[2];
    o.emissive = q.emissive_ ? 1.0f : 0.0f;
  }
  return out;
}

// scene.cpp:276-306
std::vector<wgt_sphere> Scene::PackSpheres() const {
  std::vector<wgt_sphere> out(spheres_.size());
  for (size_t i = 0; i < spheres_.size(); ++i) {
    const Sphere& s = spheres_[i];
    out[i].center[0] = s.center_[0]; out[i].center[1] = s.center_[1]; out[i].center[2] = s.center_[2];
    out[i].radius = s.radius_;
    out[i].col[0] = s.color_[0]; out[i].col[1] = s.color_[1]; out[i].col[2] = s.color_[2];
    out[i].emissive = s.emissive_;
  }
  return out;
}

// scene.cpp:170-218
std::vector<wgt_triangle> Scene::PackTriangles() const {
  std::vector<wgt_triangle> out(tris_.size());
  const float dummy = 1.0f;
  for (size_t i = 0; i < tris_.size(); ++i) {
    const Triangle& t = tris_[i];
    wgt_triangle& o = out[i];
    const Point3 v = t.vertex_[0].point_;
    o.v0[0] = v[0]; o.v0[1] = v[1]; o.v0[2] = v[2]; o.v0[3] = dummy;
    o.e1[0] = t.e1_[0]; o.e1[1] = t.e1_[1]; o.e1[2] = t.e1_[2]; o.e1[3] = dummy;
    o.e2[0] = t.e2_[0]; o.e2[1] = t.e2_[1]; o.e2[2] = t.e2_[2]; o.e2[3] = dummy;
    o.face_norm[0] = t.face_norm_[0]; o.face_norm[1] = t.face_norm_[1];
    o.face_norm[2] = t.face_norm_[2]; o.face_norm[3] = dummy;
    o.col[0] = t.color_[0]; o.col[1] = t.color_[1]; o.col[2] = t.color_[2];
    o.emissive = t.emissive_ ? 1.0f : 0.0f;
  }
  return out;
}

// scene.cpp:161-165
bool Scene::InitBuffers(wgt_ctx* ctx) {
  ctx_ = ctx;
  auto l = PackQuads(lights_);
  auto q = PackQuads(quads_);
  auto s = PackSpheres();
  auto t = PackTriangles();
  int rc = wgt_upload_scene(ctx, l.data(), (uint32_t)l.size(), q.data(), (uint32_t)q.size(), s.data(),
                            (uint32_t)s.size(), t.empty() ? nullptr : t.data(), (uint32_t)t.size());
  if (rc != WGT_OK) {
    std::cerr << "[WebGPUTracer] scene upload failed: " << wgt_last_error(ctx) << std::endl;
    return false;
  }
  uploaded_ = true;
  return true;
}

// scene.cpp:41-50: the device buffers are owned by the context; dropping them is
// a re-upload or wgt_destroy.  Idempotent.
void Scene::Release() { uploaded_ = false; }

}  // namespace wgt
