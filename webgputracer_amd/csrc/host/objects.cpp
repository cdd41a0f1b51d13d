// objects.cpp — host geometry of the reference: src/objects/{triangle,quad,box,
// cornell_box}.cpp with glm's arithmetic (include/wgt/vec.h).  Compiled with
// -ffp-contract=off so the scene bytes equal the reference's fp32 evaluation.
#include <cmath>

#include "../../../include/wgt/objects.h"

namespace wgt {

// triangle.cpp:3-16
Triangle::Triangle(Vertex v0, Vertex v1, Vertex v2, Color3 color, bool emissive) {
  vertex_[0] = v0;
  vertex_[1] = v1;
  vertex_[2] = v2;
  e1_ = vertex_[1].point_ - vertex_[0].point_;
  e2_ = vertex_[2].point_ - vertex_[0].point_;
  face_norm_ = glm::normalize(glm::cross(e1_, e2_));
  color_ = color;
  emissive_ = emissive;
}

// quad.cpp:3-13
Quad::Quad(vec3 q, vec3 right, vec3 up, Color3 color, bool emissive) {
  q_ = q;
  right_ = right;
  up_ = up;
  Recalculate();
  color_ = color;
  emissive_ = emissive;
}

void Quad::Recalculate() {
  vec3 n = glm::cross(right_, up_);
  norm_ = glm::normalize(n);
  d_ = glm::dot(norm_, q_);
  w_ = n / glm::dot(n, n);
}

// quad.cpp:15-25 (right_/up_ are transformed as points, w = 1, like the reference)
void Quad::RotateY(float angle) {
  mat4 R = glm::rotate(mat4(1.0f), glm::radians(angle), vec3(0, 1, 0));
  q_ = xyz(R * vec4(q_, 1.0f));
  right_ = xyz(R * vec4(right_, 1.0f));
  up_ = xyz(R * vec4(up_, 1.0f));
  Recalculate();
}

// quad.cpp:27-35
void Quad::Translate(vec3 direction) {
  mat4 T = glm::translate(mat4(1.0f), direction);
  q_ = xyz(T * vec4(q_, 1.0f));
  Recalculate();
}

// box.cpp:3-20
Box::Box(vec3 aabb_min, vec3 aabb_max, Color3 color, bool emissive) {
  aabb_min_ = aabb_min;
  aabb_max_ = aabb_max;
  center_ = (aabb_max_ + aabb_min_) / 2.0f;
  color_ = color;
  emissive_ = emissive;
  Point3 mn(std::fmin(aabb_min_.x, aabb_max_.x), std::fmin(aabb_min_.y, aabb_max_.y),
            std::fmin(aabb_min_.z, aabb_max_.z));
  Point3 mx(std::fmax(aabb_min_.x, aabb_max_.x), std::fmax(aabb_min_.y, aabb_max_.y),
            std::fmax(aabb_min_.z, aabb_max_.z));
  vec3 dx(mx.x - mn.x, 0, 0);
  vec3 dy(0, mx.y - mn.y, 0);
  vec3 dz(0, 0, mx.z - mn.z);
  quads_.emplace_back(Point3(mn.x, mn.y, mx.z), dx, dy, color);
  quads_.emplace_back(Point3(mx.x, mn.y, mx.z), -dz, dy, color);
  quads_.emplace_back(Point3(mx.x, mn.y, mn.z), -dx, dy, color);
  quads_.emplace_back(Point3(mn.x, mn.y, mn.z), dz, dy, color);
  quads_.emplace_back(Point3(mn.x, mx.y, mx.z), dx, -dz, color);
  quads_.emplace_back(Point3(mn.x, mn.y, mn.z), dx, dz, color);
}

void Box::RotateY(float angle) {  // box.cpp:24-28
  for (auto& quad : quads_) quad.RotateY(angle);
}
void Box::Translate(vec3 direction) {  // box.cpp:31-35
  for (auto& quad : quads_) quad.Translate(direction);
}
void Box::PushQuads(std::vector<Quad>& quads) {  // box.cpp:38-40
  quads.insert(quads.end(), quads_.begin(), quads_.end());
}

// cornell_box.cpp:4-11
CornellBox::CornellBox() {
  quads_.emplace_back(Point3(555, 0, 0), vec3(0, 0, 555), vec3(0, 555, 0), COL_GREEN);
  quads_.emplace_back(Point3(0, 0, 555), vec3(0, 0, -555), vec3(0, 555, 0), COL_RED);
  quads_.emplace_back(Point3(0, 555, 0), vec3(555, 0, 0), vec3(0, 0, 555), COL_WHITE);
  quads_.emplace_back(Point3(0, 0, 555), vec3(555, 0, 0), vec3(0, 0, -555), COL_WHITE);
  quads_.emplace_back(Point3(555, 0, 555), vec3(-555, 0, 0), vec3(0, 555, 0), COL_WHITE);
}
void CornellBox::PushToQuads(std::vector<Quad>& quads) {  // cornell_box.cpp:13-15
  quads.insert(quads.end(), quads_.begin(), quads_.end());
}

}  // namespace wgt
