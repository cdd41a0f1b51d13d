// wgt_geom.h — triangle / BVH geometry spec shared by the HIP kernels and the
// host BVH builder.  The reference shader has no triangles or
// BVH; its host code prepares exactly the Moller-Trumbore inputs
// v0, e1 = v1 - v0, e2 = v2 - v0 (src/objects/triangle.cpp:9-11), which are
// what the kernel consumes.
//
// Spec: a triangle is hit at t iff Moller-Trumbore passes with t in
// [kRayMin, kRayMax] AND t lies inside the slab interval of the triangle's own
// padded box (tri_box).  The closest triangle is the minimum (t, index).  Node
// boxes are unions of tri boxes and use the same slab formula, so node tests
// are conservative bit-for-bit (rounding is monotone) and BVH traversal returns
// exactly the brute-force answer.
#pragma once

#include "wgt_math.h"

namespace wgt {

// Padded box of one triangle: bounds of v0, v0+e1, v0+e2, then
// pad = ((hi-lo)*1e-4 + (|lo|+|hi|)*1e-5) + 1e-6 per axis.
WGT_HD void tri_box(f3 v0, f3 e1, f3 e2, f3& lo, f3& hi) {
  float l[3], h[3];
  const float a3[3] = {v0.x, v0.y, v0.z};
  const float b3[3] = {e1.x, e1.y, e1.z};
  const float d3[3] = {e2.x, e2.y, e2.z};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float a = a3[c];
    float b = a + b3[c];
    float d = a + d3[c];
    float mn = a < b ? a : b;
    mn = mn < d ? mn : d;
    float mx = a > b ? a : b;
    mx = mx > d ? mx : d;
    float pad = ((mx - mn) * 1e-4f + (fabs_w(mn) + fabs_w(mx)) * 1e-5f) + 1e-6f;
    l[c] = mn - pad;
    h[c] = mx + pad;
  }
  lo = f3{l[0], l[1], l[2]};
  hi = f3{h[0], h[1], h[2]};
}

// 1/d with |d| < 1e-30 replaced by copysign(1e-30, d): finite, so slab values are never NaN.
WGT_HD float safe_inv(float x) {
  if (fabs_w(x) < 1e-30f) x = __builtin_copysignf(1e-30f, x);
  return 1.0f / x;
}

// safe_inv by the short reciprocal (wgt_math.h div_by): the IEEE quotient for every 1e-30 <= |x| <=
// 2^34 (wgt_selftest_math tests each such bit pattern), which holds render rays' directions
// (primary components within 2^32, scattered ones unit; the clamp gives |x| >= 1e-30)
WGT_HD float safe_inv_short(float x) {
  if (fabs_w(x) < 1e-30f) x = __builtin_copysignf(1e-30f, x);
  return div_by(1.0f, rcp_of(x));
}

// Slab interval of box [lo, hi] for a ray given as inv = 1/d and ot = -(o * inv):
// t = fma(b, inv, ot) per plane.  The formula is monotone in the plane coordinate
// b (exact fma, monotone rounding), which is all the nesting argument needs.  No
// operand is NaN (inv finite, boxes finite), so min/max need no NaN rules.
WGT_HD void slab(f3 ot, f3 inv, f3 lo, f3 hi, float& tnear, float& tfar) {
  const float t0x = __builtin_fmaf(lo.x, inv.x, ot.x), t1x = __builtin_fmaf(hi.x, inv.x, ot.x);
  const float t0y = __builtin_fmaf(lo.y, inv.y, ot.y), t1y = __builtin_fmaf(hi.y, inv.y, ot.y);
  const float t0z = __builtin_fmaf(lo.z, inv.z, ot.z), t1z = __builtin_fmaf(hi.z, inv.z, ot.z);
  tnear = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(t0x, t1x), __builtin_fminf(t0y, t1y)),
                          __builtin_fminf(t0z, t1z));
  tfar = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(t0x, t1x), __builtin_fmaxf(t0y, t1y)),
                         __builtin_fmaxf(t0z, t1z));
}
WGT_HD f3 slab_offset(f3 o, f3 inv) { return f3{-(o.x * inv.x), -(o.y * inv.y), -(o.z * inv.z)}; }

// Two-sided Moller-Trumbore (fixed op order).  The early-outs
// stay (a branch-free form, one combined predicate, measured slower on sponza),
// except the determinant test, which joins the u test: without a branch between
// them the compiler issues the v0 load with the other two instead of after the
// determinant (one memory round trip per test instead of two).  Same result: a
// rejected determinant rejects either way (NaN: not rejected, as before).
// SHORT: 1/det by the short division div_rn (wgt_math.h), exact for 2^-100 <= |det| <=
// 2^100.  A |det| < 1e-12 is rejected whatever inv_det is, and for render rays |det| <=
// |e1| |e2| |d| <= 3 sqrt(3) 2^92 < 2^95 (triangle edge components within 2^30, wgt_runtime.cpp
// check_scene_limits; primary-direction components within 2^32, scattered ones unit), so the
// result is the IEEE one; caller-supplied rays (k_trace) use IEEE.
template <bool SHORT = false>
WGT_HD bool mt_test(f3 o, f3 d, f3 v0, f3 e1, f3 e2, float& tout) {
  f3 pvec = cross(d, e2);
  float det = dot(e1, pvec);
  const bool det_ok = !(fabs_w(det) < 1e-12f);
  float inv_det = SHORT ? div_rn(1.0f, det) : 1.0f / det;
  f3 tvec = o - v0;
  float u = dot(tvec, pvec) * inv_det;
  if (!det_ok || u < 0.0f || u > 1.0f) return false;
  f3 qvec = cross(tvec, e1);
  float v = dot(d, qvec) * inv_det;
  if (v < 0.0f || u + v > 1.0f) return false;
  float t = dot(e2, qvec) * inv_det;
  if (t < kRayMin || kRayMax < t) return false;
  tout = t;
  return true;
}

// Leaf-ordered triangle record, 64 B (4 x float4), one cache-line half:
//   A = (v0.xyz, original index bits)   B = (e1.xyz, box.lo.x)
//   C = (e2.xyz, box.lo.y)              D = (box.lo.z, box.hi.xyz)
// A-C feed Moller-Trumbore; D (same 128-B line, loaded with A-C) is used only for a
// candidate closest hit, to check t against the triangle's own padded box (tri_box,
// computed by the host builder with the same fp32 operations).
constexpr int kTriRecordFloats = 16;  // the host / exported record (wgt_bvh_build)
// The device record the kernels walk (by byte offsets) is the 64-B record above.  Records
// without the padded box (40 B, round 3; 48 B with 16-B aligned loads, round 6) load one
// float4 fewer per test but recompute the box (tri_box) for a candidate: slower on both
// scenes, removed.
constexpr uint32_t kTriRecordBytes = 64;
// triangles tested per triangle step of the phase-split kernel (wgt_device.h tri_step): two
// measured -1.6% on sponza, -1.3% on bunny at 1080p/256 spp; three and four +6%/+13% on sponza
// (profiles/sweeps/r03_ab_tri_per_step.log)
#ifndef WGT_TRI_PER_STEP
#define WGT_TRI_PER_STEP 2
#endif
static_assert(WGT_TRI_PER_STEP >= 1 && WGT_TRI_PER_STEP <= 4, "1 to 4 triangles per step");

// BVH4 node, 128 B (8 x float4, one L2 cache line), children in SoA order:
//   N[0] = lo.x of children 0..3   N[1] = hi.x   N[2] = lo.y   N[3] = hi.y
//   N[4] = lo.z                    N[5] = hi.z   N[6] = child refs (int bits)
//   N[7] = 0
// An empty slot holds the point box at kEmptySlotCoord on every axis and a copy
// of a live child's ref.  Its slab distances are beyond kRayMax (or negative) for
// every ray with |d| < 1e18, so it is never entered; were it entered, the visit
// would only repeat a live child: the closest hit never depends on culling beyond
// its being conservative.
// child ref >= 0: internal node index; < 0: leaf, ~ref = first*8 + (count-1)
// into the leaf-ordered triangle array (count <= 8).
constexpr int kBvhWidth = 4;
constexpr float kEmptySlotCoord = 3e38f;
constexpr int kNode4Floats = 32;
constexpr int kLeafMax = 8;
// Compact BVH4 node: an 80-B record (5 x float4) = a 64-B node + its 16-B child
// refs; the same tree as the 128-B nodes with every child plane stored as a
// binary16 code h >= 0, decoded as qdec(h, s, org_a) = fma(h, s, org_a) (one
// rounding of an exact product, monotone in h) with one scene-wide power-of-two
// step s:
//   C[0] = (org.x, org.y, org.z, 0)      org = lower bounds of the children's
//          union
//   an empty slot has the code +inf (0x7c00) for every plane: whatever the sign
//   of 1/d (finite and nonzero, safe_inv), its entry distance is +inf or its
//   exit distance -inf, so the slab test rejects it and it is never entered
//   C[1] = lo.x of children (0|1, 2|3 as half pairs), hi.x (0|1, 2|3)
//   C[2] = lo.y, hi.y                     C[3] = lo.z, hi.z
//   C[4] = child refs (int bits), as N[6]
// The builder picks each lo code as the largest whose plane decodes <= the exact
// bound and each hi code as the smallest whose plane decodes >= it, so a decoded
// box contains its 128-B box and, through it, every triangle box below: the
// nesting argument of DESIGN.md §3.4 holds unchanged.  Kernels read this form when
// the 128-B tree exceeds kCompactNodeBytes (one XCD's L2).  The
// record is not line-aligned (80 of 128 B): half the records span two lines, yet
// measured faster than refs in a separate array (two lines per visit) or 128-B
// records (the full footprint).
constexpr int kCNodeFloats = 16;     // the node part, as exported by wgt_bvh_build_compact
constexpr int kCRecordFloat4s = 5;  // node + refs, the device record
constexpr size_t kCompactNodeBytes = (size_t)4 << 20;
WGT_HD float qdec(float code, float step, float org) { return __builtin_fmaf(code, step, org); }
WGT_HD float half_bits_to_float(uint32_t b) {
  const uint32_t e = (b >> 10) & 0x1fu, m = b & 0x3ffu;
  const float v = e ? __builtin_bit_cast(float, ((e + 112u) << 23) | (m << 13)) : (float)m * 5.9604645e-8f;
  return (b & 0x8000u) ? -v : v;
}

WGT_HD int leaf_ref(uint32_t first, uint32_t count) { return ~(int)(first * 8u + (count - 1u)); }
WGT_HD uint32_t leaf_first(int ref) { return ((uint32_t)~ref) >> 3; }
WGT_HD uint32_t leaf_count(int ref) { return (((uint32_t)~ref) & 7u) + 1u; }

}  // namespace wgt
