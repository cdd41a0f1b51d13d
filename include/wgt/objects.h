// objects.h — host geometry mirroring src/include/objects/*.h of the reference
// (Vertex, Triangle, Quad, Box, CornellBox, Sphere) and the colours of
// src/include/utils/color_util.h:5-10.  Same member names and semantics.
#pragma once

#include <vector>

#include "vec.h"

namespace wgt {

// color_util.h:5-10 (double literals narrowed to float, as glm::vec3(double...) does)
inline const Color3 COL_RED = Color3((float).65, (float).05, (float).05);
inline const Color3 COL_GREEN = Color3((float).12, (float).45, (float).15);
inline const Color3 COL_BLUE = Color3((float).1, (float).2, (float).5);
inline const Color3 COL_WHITE = Color3((float).73, (float).73, (float).73);
inline const Color3 COL_LIGHT = Color3(15, 15, 15);
inline const Color3 COL_ZERO = Color3(0, 0, 0);

// vertex.h / vertex.cpp
class Vertex {
 public:
  Vertex() = default;
  Vertex(vec3 point, vec3 normal, float u, float v) : point_(point), normal_(normal), u_(u), v_(v) {}
  Vertex Translate(vec3 translation) {  // vertex.cpp:3-6
    point_ += translation;
    return *this;
  }
  vec3 point_;
  vec3 normal_;
  float u_ = 0.0f, v_ = 0.0f;
};

// triangle.h / triangle.cpp:3-16
class Triangle {
 public:
  Triangle() = default;
  Triangle(Vertex v0, Vertex v1, Vertex v2, Color3 color, bool emissive = false);
  Vertex vertex_[3];
  vec3 face_norm_, e1_, e2_;
  Color3 color_;
  bool emissive_ = false;
};

// quad.h / quad.cpp
class Quad {
 public:
  Quad() = default;
  Quad(vec3 q, vec3 right, vec3 up, Color3 color, bool emissive = false);
  void RotateY(float angle);
  void Translate(vec3 direction);
  vec3 q_, right_, up_, norm_, w_;
  float d_ = 0.0f;
  Color3 color_;
  bool emissive_ = false;

 private:
  void Recalculate();
};

// box.h / box.cpp
class Box {
 public:
  Box() = default;
  Box(vec3 aabb_min, vec3 aabb_max, Color3 color, bool emissive = false);
  void RotateY(float angle);
  void Translate(vec3 direction);
  void PushQuads(std::vector<Quad>& quads);

 private:
  vec3 aabb_min_, aabb_max_, center_;
  Color3 color_;
  bool emissive_ = false;
  std::vector<Quad> quads_;
};

// cornell_box.h / cornell_box.cpp
class CornellBox {
 public:
  CornellBox();
  void PushToQuads(std::vector<Quad>& quads);
  std::vector<Quad> quads_;
};

// sphere.h
class Sphere {
 public:
  Sphere() = default;
  Sphere(Point3 center, float radius, Color3 color, float emissive = 0.0f)
      : center_(center), radius_(radius), color_(color), emissive_(emissive) {}
  Point3 center_;
  float radius_ = 0.0f;
  Color3 color_;
  float emissive_ = 0.0f;
};

}  // namespace wgt
