// vec.h — the slice of glm the reference host code uses (src/include/utils/util.h:13-24,
// glm::vec3/vec4/mat4x4, cross, dot, normalize, rotate, translate, radians), restated
// with glm 0.9.9's operation order so that scene bytes are reproduced exactly.
// glm itself is not vendored by the reference (gitignored, .gitignore:179-184), so its
// version is unpinned; the arithmetic below is its published algorithm.
#pragma once

#include <cmath>
#include <cstdint>

namespace wgt {

struct vec3 {
  float x = 0.0f, y = 0.0f, z = 0.0f;
  vec3() = default;
  vec3(float a, float b, float c) : x(a), y(b), z(c) {}
  float& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
  float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
struct vec4 {
  float x = 0.0f, y = 0.0f, z = 0.0f, w = 0.0f;
  vec4() = default;
  vec4(float a, float b, float c, float d) : x(a), y(b), z(c), w(d) {}
  vec4(vec3 v, float d) : x(v.x), y(v.y), z(v.z), w(d) {}
};
using Point3 = vec3;  // util.h:93
using Color3 = vec3;  // util.h:94

inline vec3 operator+(vec3 a, vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline vec3 operator-(vec3 a, vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline vec3 operator-(vec3 a) { return {-a.x, -a.y, -a.z}; }
inline vec3 operator*(vec3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline vec3 operator*(float s, vec3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline vec3 operator/(vec3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline vec3& operator+=(vec3& a, vec3 b) { a = a + b; return a; }
inline vec4 operator*(vec4 a, float s) { return {a.x * s, a.y * s, a.z * s, a.w * s}; }
inline vec4 operator+(vec4 a, vec4 b) { return {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }

namespace glm {
// func_geometric.inl: dot(vec3) = (a.x*b.x + a.y*b.y) + a.z*b.z
inline float dot(vec3 a, vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline vec3 cross(vec3 x, vec3 y) {
  return {x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y};
}
// normalize(x) = x * inversesqrt(dot(x, x)), inversesqrt(v) = 1 / sqrt(v)
inline vec3 normalize(vec3 v) {
  float inv = 1.0f / std::sqrt(dot(v, v));
  return v * inv;
}
inline float radians(float deg) { return deg * static_cast<float>(0.01745329251994329576923690768489); }
}  // namespace glm

// column-major 4x4, c[col] like glm::mat4x4
struct mat4 {
  vec4 c[4];
  explicit mat4(float diag = 1.0f) {
    c[0] = {diag, 0, 0, 0};
    c[1] = {0, diag, 0, 0};
    c[2] = {0, 0, diag, 0};
    c[3] = {0, 0, 0, diag};
  }
  vec4& operator[](int i) { return c[i]; }
  const vec4& operator[](int i) const { return c[i]; }
};
// type_mat4x4.inl operator*(mat4, vec4): (m0*v0 + m1*v1) + (m2*v2 + m3*v3)
inline vec4 operator*(const mat4& m, vec4 v) {
  vec4 add0 = m[0] * v.x + m[1] * v.y;
  vec4 add1 = m[2] * v.z + m[3] * v.w;
  return add0 + add1;
}

namespace glm {
// matrix_transform.inl rotate()
inline mat4 rotate(const mat4& m, float angle, vec3 v) {
  const float a = angle;
  const float c = std::cos(a);
  const float s = std::sin(a);
  vec3 axis = normalize(v);
  vec3 temp = (1.0f - c) * axis;
  float R[3][3];
  R[0][0] = c + temp[0] * axis[0];
  R[0][1] = temp[0] * axis[1] + s * axis[2];
  R[0][2] = temp[0] * axis[2] - s * axis[1];
  R[1][0] = temp[1] * axis[0] - s * axis[2];
  R[1][1] = c + temp[1] * axis[1];
  R[1][2] = temp[1] * axis[2] + s * axis[0];
  R[2][0] = temp[2] * axis[0] + s * axis[1];
  R[2][1] = temp[2] * axis[1] - s * axis[0];
  R[2][2] = c + temp[2] * axis[2];
  mat4 out;
  out[0] = m[0] * R[0][0] + m[1] * R[0][1] + m[2] * R[0][2];
  out[1] = m[0] * R[1][0] + m[1] * R[1][1] + m[2] * R[1][2];
  out[2] = m[0] * R[2][0] + m[1] * R[2][1] + m[2] * R[2][2];
  out[3] = m[3];
  return out;
}
// matrix_transform.inl translate(): Result[3] = m[0]*v[0] + m[1]*v[1] + m[2]*v[2] + m[3]
inline mat4 translate(const mat4& m, vec3 v) {
  mat4 out = m;
  out[3] = m[0] * v[0] + m[1] * v[1] + m[2] * v[2] + m[3];
  return out;
}
}  // namespace glm

inline vec3 xyz(vec4 v) { return {v.x, v.y, v.z}; }

}  // namespace wgt
