// wgt_math.h — fp32 vector math + the numerics contract of the product path.
//
// Used by the HIP kernels (device) and by the host scene/camera code, so that a
// value computed on either side has the same bits.  Everything here is plain
// IEEE fp32 +,-,*,/,sqrt with NO contraction (the library is built with
// -ffp-contract=off) and a fixed left-to-right evaluation order that restates
// the WGSL expressions of resources/shader/path_tracer.wgsl (reference).
//
// WGSL leaves transcendental precision to the implementation; the product fixes
// it here: Cody-Waite reduction by pi/2 with a 17+24-bit split
// and degree-9/8 minimax polynomials, built from +,-,*,floor only.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define WGT_HD __host__ __device__ __forceinline__

namespace wgt {

// path_tracer.wgsl:1-10
constexpr float kPI = 3.14159265359f;
constexpr float k_1_PI = 0.318309886184f;
constexpr uint32_t kNoHit = 0xffffffffu;
constexpr int kRayDepth = 50;
constexpr float kRayMin = 0.001f;
constexpr float kRayMax = 1e20f;

struct f3 {
  float x, y, z;
};

WGT_HD f3 mk(float x, float y, float z) { return f3{x, y, z}; }
WGT_HD f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
WGT_HD f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
WGT_HD f3 operator-(f3 a) { return f3{-a.x, -a.y, -a.z}; }
WGT_HD f3 operator*(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
WGT_HD f3 operator*(float s, f3 a) { return f3{s * a.x, s * a.y, s * a.z}; }
WGT_HD f3 operator/(f3 a, float s) { return f3{a.x / s, a.y / s, a.z / s}; }
// WGSL dot: (x*x + y*y) + z*z
WGT_HD float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
WGT_HD f3 cross(f3 a, f3 b) {
  return f3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// Correctly rounded sqrt and division (device: shorter sequences than the
// compiler's general lowerings; DESIGN.md §3.2 states where each form is used and
// why it is exact there; tests/test_gpu_numerics.py checks them exhaustively).
//
// The compiler lowers llvm.sqrt.f32 as hardware v_sqrt_f32 (<= 1 ulp; it flushes
// a denormal input), then the neighbour whose residual x - s*s brackets x, with an
// input scaling by 2^32 for x < 2^-96 and a class fix-up for +-0 / +inf.  The
// fix-up is an identity for this sequence (+-0 and +inf come out unchanged, NaN
// and negative normals give NaN).
namespace detail {
WGT_HD float sqrt_seq(float x) {
#ifdef __HIP_DEVICE_COMPILE__
  const float s = __builtin_amdgcn_sqrtf(x);
  const float dn = __uint_as_float(__float_as_uint(s) - 1u);
  const float up = __uint_as_float(__float_as_uint(s) + 1u);
  const float rdn = __builtin_fmaf(-dn, s, x), rup = __builtin_fmaf(-up, s, x);
  const float r = rdn <= 0.0f ? dn : s;
  return rup > 0.0f ? up : r;
#else
  return __builtin_sqrtf(x);
#endif
}
}  // namespace detail
// sqrt_fast: the sequence alone.  Exact for x = +-0, x >= 2^-96, +inf, NaN and
// negative normals, i.e. every input except 0 < |x| < 2^-96 (and -denormals).
// Used only where the input is in that set by construction: rand() values and
// 1 - rand() (0 or >= 2^-33 in magnitude; 1 - rand() < 0 is a normal >= 2^-24)
// and squared lengths of vectors within 2^-22 of unit length or NaN.
WGT_HD float sqrt_fast(float x) { return detail::sqrt_seq(x); }
// sqrt_rn: exact for every input: the compiler's 2^32 input scaling, selected
// (not branched: a branch costs more than the 4 VALU in the persistent kernel).
// Used wherever the input depends on differences of points (hit distances, the
// light vector, sphere discriminants) or on scene-supplied normals.
WGT_HD float sqrt_rn(float x) {
#ifdef __HIP_DEVICE_COMPILE__
  const bool small = x < 0x1p-96f;
  const float s = detail::sqrt_seq(small ? x * 0x1p32f : x);
  return small ? s * 0x1p-16f : s;  // exact scalings
#else
  return __builtin_sqrtf(x);
#endif
}
// div_rn: the compiler's IEEE division sequence (reciprocal refined by one Newton
// step, two residual corrections) without v_div_scale / v_div_fixup, which are
// identities when |n|, |d| and the quotient lie in [2^-100, 2^100] (the residuals
// n - d*q stay normal, so the FMAs compute them exactly).  Its one use, the quad
// plane distance t = n / denom (isect_quad), is exact wherever the result decides
// anything: |denom| >= kRayMin is tested first, and the scene and frame limits
// checked at upload and per render (wgt_runtime.cpp) bound
// |denom| <= |qn| |d| <= 2*sqrt(3) * 2^32 < 2^35 (normal components within 2, primary
// directions within 2^32) and |n| <= 2^44, so a quotient in the accepted [kRayMin, kRayMax]
// is in the domain, and one outside it comes out outside it too (|q| < 2^-80 or
// > 2^100 cannot turn into [kRayMin, kRayMax]).
WGT_HD float div_rn(float n, float d) {
#ifdef __HIP_DEVICE_COMPILE__
  float r = __builtin_amdgcn_rcpf(d);
  r = __builtin_fmaf(__builtin_fmaf(-d, r, 1.0f), r, r);
  float q = n * r;
  q = __builtin_fmaf(__builtin_fmaf(-d, q, n), r, q);
  return __builtin_fmaf(__builtin_fmaf(-d, q, n), r, q);
#else
  return n / d;
#endif
}
// Division as the compiler's IEEE sequence without v_div_scale: the reciprocal refined once
// (rcp_of), then div_rn's two residual corrections and v_div_fixup (div_by), which sets the
// sign, zeros, infinities and NaNs as the IEEE sequence does.  The result is the IEEE quotient
// when v_div_scale would not scale (normal operands and quotient well inside the exponent
// range); its one use, the traversal's 1/d (wgt_geom.h safe_inv_short), is checked on every
// input it can take (wgt_selftest_math).
struct RcpF {
  float d, r;
};
WGT_HD RcpF rcp_of(float d) {
#ifdef __HIP_DEVICE_COMPILE__
  float r = __builtin_amdgcn_rcpf(d);
  r = __builtin_fmaf(__builtin_fmaf(-d, r, 1.0f), r, r);
  return RcpF{d, r};
#else
  return RcpF{d, 0.0f};
#endif
}
WGT_HD float div_by(float n, RcpF R) {
#ifdef __HIP_DEVICE_COMPILE__
  float q = n * R.r;
  q = __builtin_fmaf(__builtin_fmaf(-R.d, q, n), R.r, q);
  q = __builtin_fmaf(__builtin_fmaf(-R.d, q, n), R.r, q);
  return __builtin_amdgcn_div_fixupf(q, R.d, n);
#else
  return n / R.d;
#endif
}
WGT_HD float length(f3 a) { return sqrt_rn(dot(a, a)); }
// WGSL normalize(v) = v / length(v)   (zero vector -> NaN, as the reference relies on)
WGT_HD f3 normalize(f3 a) { return a / length(a); }
// normalize for a vector within 2^-22 of unit length (or NaN / inf / 0): sqrt_fast
WGT_HD f3 normalize_unit(f3 a) { return a / sqrt_fast(dot(a, a)); }
WGT_HD float distance(f3 a, f3 b) { return length(a - b); }
WGT_HD bool has_nan(f3 a) { return (a.x != a.x) | (a.y != a.y) | (a.z != a.z); }

// path_tracer.wgsl:68-70
WGT_HD float fabs_w(float x) { return x < 0.0f ? -x : x; }
// WGSL sign()
WGT_HD float sign_w(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }
// WGSL max(x, 0.0) with max(NaN, 0) = 0
WGT_HD float max0(float x) { return x > 0.0f ? x : 0.0f; }

// ---------------------------------------------------------------- transcendental
namespace detail {
constexpr float k2OverPi = 0.636619772367581343f;
constexpr float kPio2Hi = 1.5707855225e+00f;  // 0x3fc90f80 (17 significant bits)
constexpr float kPio2Lo = 1.0804334124e-05f;  // 0x37354443
WGT_HD float reduce(float x, float& q) {
  float k = __builtin_floorf(x * k2OverPi + 0.5f);
  q = k - 4.0f * __builtin_floorf(k * 0.25f);
  return (x - k * kPio2Hi) - k * kPio2Lo;
}
WGT_HD float ksin(float r) {
  float z = r * r;
  return r + (r * z) * (-1.6666667163e-01f +
                        z * (8.3333337680e-03f + z * (-1.9841270114e-04f + z * 2.7557314297e-06f)));
}
WGT_HD float kcos(float r) {
  float z = r * r;
  return (1.0f - 0.5f * z) +
         (z * z) * (4.1666667908e-02f +
                    z * (-1.3888889225e-03f + z * (2.4801587642e-05f + z * -2.7557314297e-07f)));
}
}  // namespace detail

WGT_HD float sin_w(float x) {
  float q;
  float r = detail::reduce(x, q);
  if (q == 0.0f) return detail::ksin(r);
  if (q == 1.0f) return detail::kcos(r);
  if (q == 2.0f) return -detail::ksin(r);
  return -detail::kcos(r);
}
WGT_HD float cos_w(float x) {
  float q;
  float r = detail::reduce(x, q);
  if (q == 0.0f) return detail::kcos(r);
  if (q == 1.0f) return -detail::ksin(r);
  if (q == 2.0f) return -detail::kcos(r);
  return detail::ksin(r);
}
// sin and cos of the same angle with one reduction (bit-identical to sin_w/cos_w)
WGT_HD void sincos_w(float x, float& s, float& c) {
  float q;
  float r = detail::reduce(x, q);
  float ks = detail::ksin(r), kc = detail::kcos(r);
  if (q == 0.0f) { s = ks; c = kc; }
  else if (q == 1.0f) { s = kc; c = -ks; }
  else if (q == 2.0f) { s = -ks; c = -kc; }
  else { s = -kc; c = ks; }
}
WGT_HD float tan_w(float x) { return sin_w(x) / cos_w(x); }
WGT_HD float radians_w(float deg) { return deg * 0.017453292519943295f; }

// ------------------------------------------------------------------- rand()
// path_tracer.wgsl:88-95.  bitcast<f32>(0x2f800004u) = 2.3283075e-10 (> 2^-32).
constexpr float kRandScale = __builtin_bit_cast(float, 0x2f800004u);
WGT_HD float rand_next(uint32_t& seed) {
  uint32_t s = seed * 747796405u + 2891336453u;
  seed = s;
  uint32_t word = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
  return (float)((word >> 22u) ^ word) * kRandScale;
}
// Advance the LCG state by n steps (n < 256) in 8 affine compositions; used to
// skip the remaining bounces of a NaN-absorbed path bit-exactly.
struct Affine {
  uint32_t a, c;
};
struct AffinePow2 {
  Affine f[8];
  constexpr AffinePow2() : f{} {
    Affine g{747796405u, 2891336453u};
    for (int j = 0; j < 8; ++j) {
      f[j] = g;
      g = Affine{g.a * g.a, g.a * g.c + g.c};
    }
  }
};
WGT_HD uint32_t lcg_jump(uint32_t s, uint32_t n) {
  constexpr AffinePow2 P{};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if ((n >> j) & 1u) s = P.f[j].a * s + P.f[j].c;
  }
  return s;
}

}  // namespace wgt
