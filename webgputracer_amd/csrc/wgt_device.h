// wgt_device.h — device building blocks of the path tracer kernels (wgt_kernels.hip).
// Each function restates one piece of resources/shader/path_tracer.wgsl (cited
// per function); both kernel families therefore compute bit-identical results.
#pragma once

#include <type_traits>

#include "wgt_geom.h"
#include "wgt_internal.h"

namespace wgt {

struct Hit {
  float dist;
  uint32_t prim;
  bool emissive;
  bool front_face;
  f3 pos, norm, col;
};

__device__ __forceinline__ f3 xyz(float4 v) { return f3{v.x, v.y, v.z}; }

__device__ __forceinline__ void hit_init(Hit& h) {
  // HitInfo() zero-initialised, then path_tracer.wgsl:292-296
  h.dist = kRayMax;
  h.prim = kNoHit;
  h.emissive = false;
  h.front_face = false;
  h.pos = f3{0.0f, 0.0f, 0.0f};
  h.norm = f3{0.0f, 0.0f, 0.0f};
  h.col = f3{0.0f, 0.0f, 0.0f};
}

// Accept quad q at parameter t with distance ray_dist (tail of intersect_quad).
__device__ __forceinline__ void quad_accept(f3 o, f3 d, const float4* __restrict__ q, uint32_t id,
                                            float t, float ray_dist, Hit& h) {
  const f3 qn = xyz(q[3]);
  const bool ff = dot(d, qn) < 0.0f;
  const float4 c = q[5];
  h.dist = ray_dist;
  h.prim = id;
  h.emissive = c.w > 0.0f;
  h.front_face = ff;
  h.pos = o + t * d;
  h.norm = ff ? qn : -qn;
  h.col = xyz(c);
}

// path_tracer.wgsl:314-338.  `qt` receives t of the accepted quad: the triangle
// search bound, and what finalize needs to rebuild the quad hit bit for bit.
// EXACT: the compiler's IEEE division for t, for rays outside the render limits
// that make div_rn exact here (k_trace's caller-supplied rays, wgt_math.h).
template <bool EXACT = false>
__device__ __forceinline__ void isect_quad(f3 o, f3 d, const float4* __restrict__ q, uint32_t id,
                                           Hit& h, float& qt) {
  const f3 qn = xyz(q[3]);
  const float denom = dot(qn, d);
  if (fabs_w(denom) < kRayMin) return;
  const float4 wd = q[4];
  const float num = wd.w - dot(qn, o);
  const float t = EXACT ? num / denom : div_rn(num, denom);
  if (t < kRayMin || kRayMax < t) return;
  // ray_dist is monotone non-decreasing in t >= 0 (each rounded step is), so t >=
  // qt (the accepted quad's t) implies ray_dist >= h.dist: the `>=` rejection
  // below, decided before the square root.  qt is +inf until a quad is accepted.
  if (t >= qt) return;
  const f3 pos = o + t * d;
  const float ray_dist = distance(pos, o);
  if (ray_dist >= h.dist) return;
  const f3 hit_vec = pos - xyz(q[0]);
  const f3 w = xyz(wd);
  const float a = dot(w, cross(hit_vec, xyz(q[2])));
  const float b = dot(w, cross(xyz(q[1]), hit_vec));
  // (a < 0) || (1 < a) || (b < 0) || (1 < b), NaN included: IEEE minNum/maxNum
  // return the non-NaN operand, and with both NaN every compare is false
  if ((__builtin_fminf(a, b) < 0.0f) || (1.0f < __builtin_fmaxf(a, b))) return;
  quad_accept(o, d, q, id, t, ray_dist, h);
  qt = t;
}

// path_tracer.wgsl:340-369 (sphere_uv is dead downstream: not computed)
__device__ __forceinline__ void isect_sphere(f3 o, f3 d, const float4* __restrict__ s, uint32_t id,
                                             Hit& h) {
  const float4 cr = s[0];
  const f3 center = xyz(cr);
  const f3 oc = o - center;
  const float a = dot(d, d);
  const float half_b = dot(oc, d);
  const float c = dot(oc, oc) - cr.w * cr.w;
  const float disc = half_b * half_b - a * c;
  if (disc < 0.0f) return;
  const float sqrt_d = sqrt_rn(disc);
  float root = (-half_b - sqrt_d) / a;
  if (root < kRayMin || kRayMax < root) {
    root = (-half_b + sqrt_d) / a;
    if (root < kRayMin || kRayMax < root) return;
  }
  const f3 pos = o + root * d;
  const float ray_dist = distance(pos, o);
  if (ray_dist >= h.dist) return;
  const f3 sn = (pos - center) / cr.w;
  const bool ff = dot(d, sn) < 0.0f;
  const float4 col = s[1];
  h.dist = ray_dist;
  h.prim = id;
  h.emissive = col.w > 0.0f;
  h.front_face = ff;
  h.pos = pos;
  h.norm = ff ? sn : -sn;
  h.col = xyz(col);
}

template <bool EXACT = false>
__device__ __forceinline__ void quad_scan(const DevScene& sc, f3 o, f3 d, Hit& h, float& qt) {
  hit_init(h);
  qt = __builtin_inff();
  const uint32_t nlq = sc.n_lights + sc.n_quads;
  for (uint32_t k = 0; k < nlq; ++k) {
    isect_quad<EXACT>(o, d, sc.quads + 6 * k, k, h, qt);
  }
}

// The quad scan of the persistent kernel: quad_scan's result (the accepted quad and its t) without
// the per-quad distance and its square root ("quad distance").
//
// quad_scan accepts quad k when it is valid (t in range, inside the quad) and its rounded distance
// f(t_k) = distance(o + t_k d, o) is below the best so far (kRayMax at first), so it returns the FIRST
// quad (scan order) whose f equals the minimum of f over the valid quads, provided that minimum is
// below kRayMax.  f is non-decreasing in t (every rounded step is), so the valid quad of smallest t
// (first on equal t) attains the minimum; this scan tracks that quad (t < qt, no distance) and the
// t of the best it replaced, `prev`: the smallest t of the valid quads before it in scan order.  Its
// answer is quad_scan's unless f(prev) == f(t) (an earlier quad ties in distance) or f(t) >= kRayMax.
// Both are excluded by a test on the max norms D = max|d_i|, L = max|o_i| (|.| <= ||.|| <= sqrt(3) |.|):
//   * f(t) < kRayMax when t D < 2^64: f(t) <= (sqrt(3) t D (1 + 3 eps) + eps sqrt(3) L)(1 + 2.6 eps)
//     + 2^-74 < 1e20 (eps = 2^-24, L < 2^41 under the scene limits);
//   * f(t) < f(prev) when g = (prev - t) - 2^-19 (prev + t) > 0, g D > 2^-18 L and prev D >= 2^-49: each
//     component of pos - o is t d_i within eps (3 |t d_i| + |o_i|), so ||pos - o|| is t ||d|| within
//     eps (3 t ||d|| + ||o||); the test (computed in fp32, whose roundings its factor-2 margins absorb)
//     gives (prev - t) ||d|| - 2^-20 (prev + t) ||d|| > 2^-19 ||o||, so the two exact norms differ by
//     >= 2^-21 prev ||d||, more than the dot product's and square root's roundings (2.6 eps relative,
//     2^-74 absolute from denormal squares) can close when prev ||d|| >= 2^-50.
// A lane that fails the test (an almost-tie: rays near the line where two quads meet) takes the
// reference scan, quad_scan; returns false for such a lane.  EXACT: as quad_scan<EXACT>.
template <bool EXACT = false>
__device__ __forceinline__ bool quad_scan_fast(const DevScene& sc, f3 o, f3 d, uint32_t& prim, float& qt) {
  prim = kNoHit;
  qt = __builtin_inff();
  float prev = __builtin_inff();
  const uint32_t nlq = sc.n_lights + sc.n_quads;
  for (uint32_t k = 0; k < nlq; ++k) {
    const float4* __restrict__ q = sc.quads + 6 * k;
    const f3 qn = xyz(q[3]);
    const float denom = dot(qn, d);
    if (fabs_w(denom) < kRayMin) continue;
    const float4 wd = q[4];
    const float num = wd.w - dot(qn, o);
    const float t = EXACT ? num / denom : div_rn(num, denom);
    if (t < kRayMin || kRayMax < t) continue;
    if (t >= qt) continue;
    const f3 pos = o + t * d;
    const f3 hit_vec = pos - xyz(q[0]);
    const f3 w = xyz(wd);
    const float a = dot(w, cross(hit_vec, xyz(q[2])));
    const float b = dot(w, cross(xyz(q[1]), hit_vec));
    if ((__builtin_fminf(a, b) < 0.0f) || (1.0f < __builtin_fmaxf(a, b))) continue;
    prev = qt;
    qt = t;
    prim = k;
  }
  bool exact = true;
  if (prim != kNoHit) {
    const float D = __builtin_fmaxf(__builtin_fmaxf(fabs_w(d.x), fabs_w(d.y)), fabs_w(d.z));
    const float L = __builtin_fmaxf(__builtin_fmaxf(fabs_w(o.x), fabs_w(o.y)), fabs_w(o.z));
    exact = qt * D < 0x1p64f;
    if (prev != __builtin_inff()) {
      const float g = (prev - qt) - 0x1p-19f * (prev + qt);
      exact = exact && g * D > 0x1p-18f * L && prev * D >= 0x1p-49f;
    }
  }
  if (!exact) {
    Hit h;
    quad_scan<EXACT>(sc, o, d, h, qt);
    prim = h.prim;
  }
  return exact;
}

// The quad part of a hit rebuilt from (prim, t): the same operations as isect_quad.
__device__ __forceinline__ void quad_rebuild(const DevScene& sc, f3 o, f3 d, uint32_t prim, float t,
                                             Hit& h) {
  hit_init(h);
  if (prim == kNoHit) return;
  const f3 pos = o + t * d;
  quad_accept(o, d, sc.quads + 6 * prim, prim, t, distance(pos, o), h);
}

__device__ __forceinline__ uint32_t last_prim(const DevScene& sc) {
  return sc.n_lights + sc.n_quads + sc.n_tris + sc.n_spheres - 1u;
}

// A NaN ray's hit: the last sphere (every rejection test is false for NaN).
__device__ __forceinline__ void nan_hit(const DevScene& sc, f3 o, f3 d, Hit& h) {
  hit_init(h);
  const uint32_t k = sc.n_spheres - 1;
  isect_sphere(o, d, sc.spheres + 2 * k, sc.n_lights + sc.n_quads + sc.n_tris + k, h);
}

struct TravStats {
  uint32_t nodes, tris, wave_steps, lane_steps;
  uint32_t spills, refills;  // parked k_render_ps: global-stack moves (park_fix)
  uint32_t overflows;        // parked k_render_ps: park_fix's overflow exit (never taken: tests assert 0)
};

// Counts one per wave (first active lane) and one per active lane.
__device__ __forceinline__ void simt_count(uint32_t& wave, uint32_t& lane) {
  const unsigned long long b = __ballot(1);
  if (__lane_id() == (unsigned)(__ffsll((long long)b) - 1)) ++wave;
  ++lane;
}

// One triangle test of a 64-B record (wgt_geom.h kTriRecordBytes) held in registers:
// Moller-Trumbore, then for a candidate that beats (bt, bi) the slab check against the
// triangle's own padded box.  inv: 1/d.  Returns true with (tt, idx)
// when the triangle becomes the closest hit.
// SHORT: mt_test's short reciprocal (render rays only, wgt_geom.h).
template <bool SHORT>
__device__ __forceinline__ bool tri_test_rec(float4 A, float4 B, float4 C, float4 D, f3 o, f3 d, f3 ot, f3 inv,
                                             float bt, uint32_t bi, float& tt, uint32_t& idx) {
  const f3 v0 = xyz(A), e1 = xyz(B), e2 = xyz(C);
  idx = __float_as_uint(A.w);
  const f3 blo = f3{B.w, C.w, D.x}, bhi = f3{D.y, D.z, D.w};
  if (!mt_test<SHORT>(o, d, v0, e1, e2, tt)) return false;
  if (!(tt < bt || (tt == bt && idx < bi))) return false;
  float bn, bf;
  slab(ot, inv, blo, bhi, bn, bf);
  return bn <= tt && tt <= bf;
}
// The same for the record at byte offset lf: all four float4 loaded at once (the padded box D,
// for a candidate closest hit, used to be loaded in the branch, a second dependent round trip).
template <bool SHORT>
__device__ __forceinline__ bool tri_test(const float4* __restrict__ tris, uint32_t lf, f3 o, f3 d, f3 ot, f3 inv,
                                         float bt, uint32_t bi, float& tt, uint32_t& idx) {
  const float4* __restrict__ p = (const float4*)((const char*)tris + lf);
  return tri_test_rec<SHORT>(p[0], p[1], p[2], p[3], o, d, ot, inv, bt, bi, tt, idx);
}

// Resumable BVH4 traversal: closest triangle = min (t, index) with t < bound (or
// t <= bound and index < bi when bi = kNoHit).  Per-lane stack: DevScene::stack
// entries in LDS (stride kBlock, conflict-free).
struct Trav {
  f3 inv, ot;
  float bt;
  uint32_t bi;
  int ref;          // current internal node (when no leaf is open)
  uint32_t lf, le;  // open leaf: byte offsets of the next triangle record and of the leaf's end
  int sp;
};
// A triangle was accepted (bi starts at kNoHit, see trav_init).
__device__ __forceinline__ bool trav_found(const Trav& t) { return t.bi != kNoHit; }

// The node form CN: 0 = 128-B nodes, 1 = 80-B compact records.

// CN (compact nodes): t.inv holds s/d (s = the form's step, a power of two: exact), the
// factor of the fused slab step (cchild_key); the triangle box check multiplies
// it back by 1/s.
// EXACT: the IEEE 1/d (k_trace's caller-supplied rays); else the short reciprocal (render rays).
template <int CN = 0, bool EXACT = false>
__device__ __forceinline__ void trav_init(const DevScene& sc, f3 o, f3 d, bool quad_hit, float qt, Trav& t) {
  t.inv = EXACT ? f3{safe_inv(d.x), safe_inv(d.y), safe_inv(d.z)}
                : f3{safe_inv_short(d.x), safe_inv_short(d.y), safe_inv_short(d.z)};
  t.ot = slab_offset(o, t.inv);
  if (CN) t.inv = sc.cstep * t.inv;
  // a triangle must satisfy t < t_quad to beat a quad hit (ray_dist is monotone in
  // t): with bi = kNoHit the rule "t < bt, or t == bt and index < bi" accepts
  // exactly t <= bt, so bt = the float below t_quad (t_quad > 0).  A box entered
  // at t_quad could only hold triangles with t >= t_quad, so culling it is exact.
  t.bt = quad_hit ? __uint_as_float(__float_as_uint(qt) - 1u) : kRayMax;
  t.bi = kNoHit;
  t.ref = 0;
  t.lf = t.le = 0;
  t.sp = 0;
}


// Sort key of one BVH4 child: the bits of the clamped entry distance max(near,
// kRayMin) (positive and not NaN, so its bits order as unsigned and never equal
// kMissKey); kMissKey if the ray misses the box or the box lies beyond the current
// closest hit.  Equal keys sort in either order (the ref moves with its key).  hit = max(near, kRayMin) <= min(far, bt) is the node test
// near <= far && near <= bt && far >= kRayMin, because bt >= kRayMin always
// (bt is kRayMax, a quad t or a triangle t, all >= kRayMin).
constexpr uint32_t kMissKey = 0xFFFFFFFFu;
// min(f, bt) for bt > 0 and f not NaN (no NaN ray traverses: wgt_kernels.hip resolves
// them without tracing, and a NaN k_trace ray tests no triangle either way): the signed
// minimum of the bits orders every negative f below bt and positive floats as fminf
// does.  An integer minimum needs no canonicalised operand, where fminf of the
// loop-carried bt costs a v_max_f32 bt, bt per node step (IEEE mode).  Compact nodes only:
// the 128-B form's step measured 0.9 % slower with it (profiles/r06/ab_r06q.txt).
__device__ __forceinline__ float min_bt(float f, float bt) {
  return __int_as_float(__builtin_elementwise_min(__float_as_int(f), __float_as_int(bt)));
}
__device__ __forceinline__ uint32_t child_key(const Trav& t, float lx, float hx, float ly, float hy,
                                              float lz, float hz, uint32_t slot) {
  const float t0x = __builtin_fmaf(lx, t.inv.x, t.ot.x), t1x = __builtin_fmaf(hx, t.inv.x, t.ot.x);
  const float t0y = __builtin_fmaf(ly, t.inv.y, t.ot.y), t1y = __builtin_fmaf(hy, t.inv.y, t.ot.y);
  const float t0z = __builtin_fmaf(lz, t.inv.z, t.ot.z), t1z = __builtin_fmaf(hz, t.inv.z, t.ot.z);
  const float n = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(t0x, t1x), __builtin_fminf(t0y, t1y)),
                                  __builtin_fmaxf(__builtin_fminf(t0z, t1z), kRayMin));
  const float f = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(t0x, t1x), __builtin_fmaxf(t0y, t1y)),
                                  __builtin_fminf(__builtin_fmaxf(t0z, t1z), t.bt));
  return n <= f ? __float_as_uint(n) : kMissKey;
}
// Sort keys and refs of the 4 children of node `ref`, read from the 128-B nodes
// (CN = false) or from the compact nodes (CN = true, wgt_geom.h).
__device__ __forceinline__ float hcode(uint32_t w, uint32_t slot) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)((slot & 1u) ? (w >> 16) : (w & 0xffffu)));
}
// Compact node: per axis the ray's entry plane is the lo code for inv >= 0 and the
// hi code for inv < 0 (one select per two children), which equals the min / max
// form of child_key because the slab formula is monotone in the plane.  The slab
// distance of the plane org' + h*s is one fused step fma(h, s/d, c) with h taken
// from a half word (v_fma_mix_f32) and c = fma(org/s, s/d, ot) per node and axis;
// the builder's code margin makes the interval contain the exact one (wgt_geom.h,
// DESIGN.md §3.4).  An empty slot's +inf codes give n = +inf or f = -inf: a miss
// without a mask.
__device__ __forceinline__ uint32_t cchild_key(const Trav& t, const uint32_t* nw, const uint32_t* fw, f3 c,
                                               uint32_t slot) {
  const uint32_t k = slot >> 1;
  const float tnx = __builtin_fmaf(hcode(nw[0 + k], slot), t.inv.x, c.x);
  const float tfx = __builtin_fmaf(hcode(fw[0 + k], slot), t.inv.x, c.x);
  const float tny = __builtin_fmaf(hcode(nw[2 + k], slot), t.inv.y, c.y);
  const float tfy = __builtin_fmaf(hcode(fw[2 + k], slot), t.inv.y, c.y);
  const float tnz = __builtin_fmaf(hcode(nw[4 + k], slot), t.inv.z, c.z);
  const float tfz = __builtin_fmaf(hcode(fw[4 + k], slot), t.inv.z, c.z);
  const float n = __builtin_fmaxf(__builtin_fmaxf(tnx, tny), __builtin_fmaxf(tnz, kRayMin));
  const float f = min_bt(__builtin_fminf(__builtin_fminf(tfx, tfy), tfz), t.bt);
  return n <= f ? __float_as_uint(n) : kMissKey;
}
template <int CN>
__device__ __forceinline__ void node_keys(const DevScene& sc, const Trav& t, int ref, uint32_t& k0, uint32_t& k1,
                                          uint32_t& k2, uint32_t& k3, int& r0, int& r1, int& r2, int& r3) {
  if (CN) {
    // 80-B record: origin, codes, refs
    const float4* __restrict__ n = (const float4*)((const char*)sc.cnodes + (uint32_t)ref);  // byte offset
    const int4 rf = __builtin_bit_cast(int4, n[4]);
    const float4 a = n[0];
    const uint4 x = __builtin_bit_cast(uint4, n[1]), y = __builtin_bit_cast(uint4, n[2]),
                z = __builtin_bit_cast(uint4, n[3]);
    // c = the slab distance of the node origin org' = (org/s) * s: fma(org/s, s/d, ot)
    const f3 c = f3{__builtin_fmaf(a.x, t.inv.x, t.ot.x), __builtin_fmaf(a.y, t.inv.y, t.ot.y),
                    __builtin_fmaf(a.z, t.inv.z, t.ot.z)};
    const bool sx = t.inv.x < 0.0f, sy = t.inv.y < 0.0f, sz = t.inv.z < 0.0f;
    const uint32_t nw[6] = {sx ? x.z : x.x, sx ? x.w : x.y, sy ? y.z : y.x,
                            sy ? y.w : y.y, sz ? z.z : z.x, sz ? z.w : z.y};
    const uint32_t fw[6] = {sx ? x.x : x.z, sx ? x.y : x.w, sy ? y.x : y.z,
                            sy ? y.y : y.w, sz ? z.x : z.z, sz ? z.y : z.w};
    r0 = rf.x, r1 = rf.y, r2 = rf.z, r3 = rf.w;
    k0 = cchild_key(t, nw, fw, c, 0u);
    k1 = cchild_key(t, nw, fw, c, 1u);
    k2 = cchild_key(t, nw, fw, c, 2u);
    k3 = cchild_key(t, nw, fw, c, 3u);
  } else {
    const float4* __restrict__ n = (const float4*)((const char*)sc.nodes + (uint32_t)ref);  // ref: byte offset
    const float4 lx = n[0], hx = n[1], ly = n[2], hy = n[3], lz = n[4], hz = n[5];
    const float4 rf = n[6];
    r0 = __float_as_int(rf.x), r1 = __float_as_int(rf.y), r2 = __float_as_int(rf.z), r3 = __float_as_int(rf.w);
    k0 = child_key(t, lx.x, hx.x, ly.x, hy.x, lz.x, hz.x, 0u);
    k1 = child_key(t, lx.y, hx.y, ly.y, hy.y, lz.y, hz.y, 1u);
    k2 = child_key(t, lx.z, hx.z, ly.z, hy.z, lz.z, hz.z, 2u);
    k3 = child_key(t, lx.w, hx.w, ly.w, hy.w, lz.w, hz.w, 3u);
  }
}

// Compare-exchange of (key, ref) pairs: the smaller key (and its ref) to a.
__device__ __forceinline__ void cas(uint32_t& ka, int& ra, uint32_t& kb, int& rb) {
  const bool sw = kb < ka;
  const uint32_t k = sw ? kb : ka;
  kb = sw ? ka : kb;
  ka = k;
  const int r = sw ? rb : ra;
  rb = sw ? ra : rb;
  ra = r;
}

// One BVH4 node OR one triangle per call (a leaf is opened as a range and its
// triangles are tested one per step), so every lane's step costs about the same
// and a wave never pays for an 8-triangle leaf loop at every step.  A node step
// sorts its hit children by entry distance (5 compare-exchanges of (key, ref)), descends into
// the nearest and pushes the others farthest first.  The stack lives in LDS
// only, sized to the builder's exact worst case, so it cannot overflow.  Push /
// pop / descend are selects around one leaf-or-node branch to keep the
// exec-mask bookkeeping small.  Returns true when the traversal has finished.
template <bool STATS>
__device__ __forceinline__ bool trav_step(const DevScene& sc, f3 o, f3 d, Trav& t,
                                          int* __restrict__ lds, TravStats& st) {
  if (STATS) simt_count(st.wave_steps, st.lane_steps);
  bool pop;
  int next = 0;
  if (t.lf < t.le) {
    if (STATS) st.tris++;
    float tt;
    uint32_t idx;
    if (tri_test<false>(sc.tris, t.lf, o, d, t.ot, t.inv, t.bt, t.bi, tt, idx)) {  // IEEE: k_trace's rays
      t.bt = tt;
      t.bi = idx;
    }
    t.lf += kTriRecordBytes;
    if (t.lf < t.le) return false;
    pop = true;
  } else {
    if (STATS) st.nodes++;
    uint32_t k0, k1, k2, k3;
    int r0, r1, r2, r3;
    node_keys<false>(sc, t, t.ref, k0, k1, k2, k3, r0, r1, r2, r3);
    cas(k0, r0, k1, r1);
    cas(k2, r2, k3, r3);
    cas(k0, r0, k2, r2);
    cas(k1, r1, k3, r3);
    cas(k1, r1, k2, r2);
    // push the hit children other than the nearest, farthest first; a write for a
    // missed child lands above the top and is overwritten or never read
    lds[t.sp * kBlock] = r3;
    t.sp += k3 != kMissKey ? 1 : 0;
    lds[t.sp * kBlock] = r2;
    t.sp += k2 != kMissKey ? 1 : 0;
    lds[t.sp * kBlock] = r1;
    t.sp += k1 != kMissKey ? 1 : 0;
    next = r0;
    pop = k0 == kMissKey;
  }
  if (pop) {
    if (t.sp == 0) return true;
    --t.sp;
    next = lds[t.sp * kBlock];
  }
  const bool leaf = next < 0;
  const uint32_t lfirst = leaf_first(next) * kTriRecordBytes;
  t.lf = leaf ? lfirst : t.lf;
  t.le = leaf ? lfirst + leaf_count(next) * kTriRecordBytes : t.le;
  t.ref = leaf ? t.ref : next;
  return false;
}

// ---------------------------------------------------------------------------
// Speculative two-mode traversal (k_render_ps).  A wave step is uniformly a
// NODE step (lanes with an internal node to visit) or a TRIANGLE step (lanes
// with a pending leaf), so a step issues one of the two code paths instead of
// both.  A lane that reaches a leaf parks it as its pending leaf and keeps
// descending (speculation, after Aila & Laine's speculative while-while); a
// second leaf found meanwhile waits on the stack (one entry beyond the
// builder's bound: DevScene::stack includes it).  Culling with a not yet
// updated best t is only less tight, never wrong: the closest hit is a minimum
// over (t, index) of every triangle whose boxes the ray enters.
//
// Lane state after every step: an internal node in t.ref, or kNoRef with a
// pending leaf (lf < le), or done (kNoRef, no pending leaf, empty stack).
constexpr int kNoRef = 0x7fffffff;

// The per-lane LDS traversal stack of k_render_ps, entry i of a lane at stride
// kBlock (conflict-free).  Stack32: one int per entry.  Stack24: a 16-bit and an
// 8-bit array (3 B per entry, the high byte sign-extending), which fits every ref
// of a tree with fewer than 2^16 nodes and 2^20 triangles (byte offsets < 2^23,
// leaf refs >= -2^23; DevScene::ps_waves) and lets LDS hold the full 31-entry
// bound of 24 waves per CU: 6 waves per SIMD without a narrower tree.
// S: the stride in entries (kBlock: one wave per block).
template <int S = kBlock>
struct Stack32S {
  int* __restrict__ p;
  __device__ __forceinline__ int ld(int i) const { return p[i * S]; }
  __device__ __forceinline__ void st(int i, int v) const { p[i * S] = v; }
};
template <int S = kBlock>
struct Stack24S {
  uint16_t* __restrict__ lo;
  int8_t* __restrict__ hi;
  __device__ __forceinline__ int ld(int i) const { return ((int)hi[i * S] << 16) | (int)lo[i * S]; }
  __device__ __forceinline__ void st(int i, int v) const {
    lo[i * S] = (uint16_t)v;
    hi[i * S] = (int8_t)(v >> 16);
  }
};
using Stack32 = Stack32S<>;
using Stack24 = Stack24S<>;
// Parked traversal state of k_render_ps (DevScene::ps_park): the
// lane's Trav lives in LDS words (stride kBlock, conflict-free) while its wave runs a
// service pass, so the service code does not hold the traversing lanes' 11 registers and
// needs no scratch.  Word 9 holds the LDS stack top in its low half and the depth of the
// lane's global stack (entries moved out of LDS, DevFrame::ps_spill) in its high half:
// the traversal phase reads and writes only the low half.  The open leaf is one word:
// the record offset (a multiple of kTriRecordBytes) plus the records left (<= 8).
struct Park {
  uint32_t* __restrict__ p;
  __device__ __forceinline__ uint32_t ld(int j) const { return p[j * kBlock]; }
  __device__ __forceinline__ void st(int j, uint32_t v) const { p[j * kBlock] = v; }
  __device__ __forceinline__ uint32_t sp() const { return ((const uint16_t*)(p + 9 * kBlock))[0]; }
  __device__ __forceinline__ void set_sp(uint32_t v) const { ((uint16_t*)(p + 9 * kBlock))[0] = (uint16_t)v; }
};
// the record offset's zero low bits (6 for 64-B records) hold the count (<= kLeafMax)
constexpr uint32_t kParkLeafMask = kTriRecordBytes - 1u;
static_assert((kTriRecordBytes & kParkLeafMask) == 0u && kParkLeafMask >= (uint32_t)kLeafMax,
              "the parked open leaf packs its count into the offset's low bits");
__device__ __forceinline__ uint32_t park_leaf(const Trav& t) { return t.lf | ((t.le - t.lf) / kTriRecordBytes); }
__device__ __forceinline__ void unpark_leaf(uint32_t w, Trav& t) {
  t.lf = w & ~kParkLeafMask;
  t.le = t.lf + (w & kParkLeafMask) * kTriRecordBytes;
}
// the whole state; the global depth (word 9's high half) is left as it is
__device__ __forceinline__ void park_put(const Park& P, const Trav& t) {
  P.st(0, __float_as_uint(t.inv.x)); P.st(1, __float_as_uint(t.inv.y)); P.st(2, __float_as_uint(t.inv.z));
  P.st(3, __float_as_uint(t.ot.x)); P.st(4, __float_as_uint(t.ot.y)); P.st(5, __float_as_uint(t.ot.z));
  P.st(6, __float_as_uint(t.bt)); P.st(7, t.bi); P.st(8, (uint32_t)t.ref);
  P.set_sp((uint32_t)t.sp);
  P.st(10, park_leaf(t));
}
__device__ __forceinline__ void park_get(const Park& P, Trav& t) {
  t.inv = f3{__uint_as_float(P.ld(0)), __uint_as_float(P.ld(1)), __uint_as_float(P.ld(2))};
  t.ot = f3{__uint_as_float(P.ld(3)), __uint_as_float(P.ld(4)), __uint_as_float(P.ld(5))};
  t.bt = __uint_as_float(P.ld(6));
  t.bi = P.ld(7);
  t.ref = (int)P.ld(8);
  t.sp = (int)P.sp();
  unpark_leaf(P.ld(10), t);
}

// Place `cand` (a child ref, or kNoRef = take the next stack entry).
template <class STK>
__device__ __forceinline__ void trav_resolve(const DevScene& sc, Trav& t, int cand, const STK& lds) {
#pragma unroll
  for (int it = 0; it < 3; ++it) {
    if (cand == kNoRef) {
      if (t.sp == 0) break;
      --t.sp;
      cand = lds.ld(t.sp);
    }
    if (cand >= 0) {
      t.ref = cand;
      return;
    }
    if (t.lf >= t.le) {  // no pending leaf: this one becomes it; keep looking for a node
      t.lf = leaf_first(cand) * kTriRecordBytes;
      t.le = t.lf + leaf_count(cand) * kTriRecordBytes;
      cand = kNoRef;
      continue;
    }
    lds.st(t.sp, cand);  // a second leaf waits on the stack
    ++t.sp;
    break;
  }
  t.ref = kNoRef;
}

__device__ __forceinline__ bool trav_done(const Trav& t) { return t.ref == kNoRef && t.lf >= t.le && t.sp == 0; }

// Parked k_render_ps: a lane leaves its traversal phase when a node step leaves fewer than
// 4 free LDS entries above its stack top (the next step's 3 pushes and a parked leaf), or
// when its LDS stack runs empty with entries still on its global stack.  Its service pass
// then moves stack entries between LDS and the lane's global stack (gs, stride `stride`)
// and the traversal resumes: the stack keeps its order, split over the two, so the
// traversal visits what the whole-LDS stack would (it only stops early when the LDS part
// runs empty, which any order of the exact min (t, index) search allows).
// Returns 1 for a spill, 2 for a refill.
template <class STK>
__device__ __forceinline__ uint32_t park_fix(const DevScene& sc, const Park& P, const STK& lds, uint32_t cap,
                                             int* __restrict__ gs, uint32_t stride) {
  const uint32_t w9 = P.ld(9);
  const uint32_t sp = w9 & 0xffffu, g = w9 >> 16;
  if (sp + 4u > cap) {  // overflow: all but the top `keep` entries move to the global stack
    const uint32_t keep = (cap - 3u) / 2u;  // 1 <= keep <= cap - 4 for cap >= kMinPsCap
    const uint32_t m = sp - keep;
    if (g + m > sc.stack) {
      // g + sp never exceeds the builder's bound sc.stack (the global stack's size); were
      // it to, the traversal ends here (a wrong image the parity tests catch) rather than
      // writing out of bounds or spilling forever
      P.st(8, (uint32_t)kNoRef);
      P.st(10, 0u);
      P.st(9, 0u);
      return 3u;
    }
    for (uint32_t i = 0; i < m; ++i) gs[(size_t)(g + i) * stride] = lds.ld((int)i);
    for (uint32_t i = 0; i < keep; ++i) lds.st((int)i, lds.ld((int)(i + m)));
    P.st(9, keep | (g + m) << 16);
    return 1u;
  }
  // the LDS part ran empty (nothing open, g > 0): the top m global entries come back, then
  // the pop the traversal stopped at; m - 1 <= cap - 4 leaves room for the next node step
  const uint32_t half = (cap - 3u) / 2u + 1u;
  const uint32_t m = g < half ? g : half;
  for (uint32_t i = 0; i < m; ++i) lds.st((int)i, gs[(size_t)(g - m + i) * stride]);
  Trav t;
  t.ref = kNoRef;
  unpark_leaf(P.ld(10), t);
  t.sp = (int)m;
  trav_resolve(sc, t, kNoRef, lds);
  P.st(8, (uint32_t)t.ref);
  P.st(10, park_leaf(t));
  P.st(9, (uint32_t)t.sp | (g - m) << 16);
  return 2u;
}

// Visit t.ref: bring the nearest hit child to slot 0 (three compare-exchanges: the
// pairs, then their minima), push the other three unordered, place the nearest.
// The full 5-exchange network cost 10 more VALU per node step for 0.6% fewer node
// visits.  Any order is exact (the closest hit is a minimum
// over (t, index)), and a missed child's kMissKey keeps it off the stack wherever it
// sits: each push advances the top only for a hit.
// ROOT: the step of a ray that has just started (t.ref = 0 for every lane): the node's
// address is uniform, so its loads are scalar (SMEM) loads shared by the wave.
template <bool STATS, int CN, class STK, bool ROOT = false>
__device__ __forceinline__ void node_step(const DevScene& sc, Trav& t, const STK& lds, TravStats& st) {
  if (STATS) st.nodes++;
  uint32_t k0, k1, k2, k3;
  int r0, r1, r2, r3;
  node_keys<CN>(sc, t, ROOT ? 0 : t.ref, k0, k1, k2, k3, r0, r1, r2, r3);
  cas(k0, r0, k1, r1);
  cas(k2, r2, k3, r3);
  cas(k0, r0, k2, r2);
  lds.st(t.sp, r3);
  t.sp += k3 != kMissKey ? 1 : 0;
  lds.st(t.sp, r2);
  t.sp += k2 != kMissKey ? 1 : 0;
  lds.st(t.sp, r1);
  t.sp += k1 != kMissKey ? 1 : 0;
  trav_resolve(sc, t, k0 != kMissKey ? r0 : kNoRef, lds);
}

template <bool STATS, int CN, class STK>
__device__ __forceinline__ void root_step(const DevScene& sc, Trav& t, const STK& lds, TravStats& st) {
  node_step<STATS, CN, STK, true>(sc, t, lds, st);
}

// Test the next triangle of the pending leaf; a lane without a node to visit
// takes the next stack entry once its leaf is done.
template <bool STATS, int CN = 0, class STK>
__device__ __forceinline__ void tri_step(const DevScene& sc, f3 o, f3 d, Trav& t, const STK& lds,
                                         TravStats& st) {
  // 1/d: under CN t.inv holds s/d, and (s/d) * (1/s) is 1/d exactly
  const f3 inv = CN ? sc.rcstep * t.inv : t.inv;
#if WGT_TRI_PER_STEP > 1
  // up to WGT_TRI_PER_STEP triangles of the open leaf per step (a slot past the leaf's end
  // re-reads the first record and is ignored): the closest hit is a minimum over (t, index), so
  // testing them against the same bound and merging is exact.  Every slot's record is loaded
  // before any test: loaded inside tri_test, the second record's loads sat behind the first
  // test's early-out branches, two dependent round trips per step (round 6: sponza +1.5 %,
  // bunny +0.9 %)
  constexpr int K = WGT_TRI_PER_STEP;
  float tt[K];
  uint32_t idx[K];
  bool hit[K];
  uint32_t n = 1;
  float4 R[K][4];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint32_t a = t.lf + uint32_t(j) * kTriRecordBytes;
    const bool live = j == 0 || a < t.le;
    const float4* __restrict__ q = (const float4*)((const char*)sc.tris + (live ? a : t.lf));
    R[j][0] = q[0], R[j][1] = q[1], R[j][2] = q[2], R[j][3] = q[3];
  }
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const bool live = j == 0 || t.lf + uint32_t(j) * kTriRecordBytes < t.le;
    hit[j] = tri_test_rec<true>(R[j][0], R[j][1], R[j][2], R[j][3], o, d, t.ot, inv, t.bt, t.bi, tt[j], idx[j]);
    if (j > 0) {
      hit[j] = hit[j] && live;
      n += live ? 1u : 0u;
    }
  }
  if (hit[0]) {  // passed tri_test's own (t, index) filter against the same bound
    t.bt = tt[0];
    t.bi = idx[0];
  }
#pragma unroll
  for (int j = 1; j < K; ++j)
    if (hit[j] && (tt[j] < t.bt || (tt[j] == t.bt && idx[j] < t.bi))) {
      t.bt = tt[j];
      t.bi = idx[j];
    }
  if (STATS) st.tris += n;
  t.lf += n * kTriRecordBytes;
#else
  if (STATS) st.tris++;
  float tt;
  uint32_t idx;
  if (tri_test<true>(sc.tris, t.lf, o, d, t.ot, inv, t.bt, t.bi, tt, idx)) {
    t.bt = tt;
    t.bi = idx;
  }
  t.lf += kTriRecordBytes;
#endif
  if (t.lf >= t.le && t.ref == kNoRef) trav_resolve(sc, t, kNoRef, lds);
}

// Merge the triangle result into the quad hit, then scan the spheres: the end of
// sample_hit (path_tracer.wgsl:305-309) with triangles between quads and spheres.
// PRELOAD: the triangle's shading record is read before the quad hit is rebuilt (the
// caller issues both loads together, preload_tshade) instead of after the distance
// comparison that needs it: one memory round trip per finalise instead of two.
// The triangle result of a finished traversal: (bt, bi), bi = kNoHit when no
// triangle was accepted (trav_found).
__device__ __forceinline__ void preload_tshade(const DevScene& sc, uint32_t bi, float4& s0, float4& s1) {
  const uint32_t i = bi != kNoHit ? bi : 0u;  // record 0 for a ray without a triangle hit: unused
  s0 = sc.tshade[2 * i];
  s1 = sc.tshade[2 * i + 1];
}
__device__ __forceinline__ void preload_tshade(const DevScene& sc, const Trav& t, float4& s0, float4& s1) {
  preload_tshade(sc, t.bi, s0, s1);
}
__device__ __forceinline__ void finish_hit(const DevScene& sc, f3 o, f3 d, float bt, uint32_t bi, Hit& h,
                                           const float4* pre = nullptr) {
  const uint32_t nlq = sc.n_lights + sc.n_quads;
  if (bi != kNoHit) {
    const f3 pos = o + bt * d;
    const float ray_dist = distance(pos, o);
    if (!(ray_dist >= h.dist)) {
      const float4 s0 = pre ? pre[0] : sc.tshade[2 * bi], s1 = pre ? pre[1] : sc.tshade[2 * bi + 1];
      const f3 fn = xyz(s0);
      const bool ff = dot(d, fn) < 0.0f;
      h.dist = ray_dist;
      h.prim = nlq + bi;
      h.emissive = s0.w > 0.0f;
      h.front_face = ff;
      h.pos = pos;
      h.norm = ff ? fn : -fn;
      h.col = xyz(s1);
    }
  }
  for (uint32_t k = 0; k < sc.n_spheres; ++k)
    isect_sphere(o, d, sc.spheres + 2 * k, nlq + sc.n_tris + k, h);
}
__device__ __forceinline__ void finish_hit(const DevScene& sc, f3 o, f3 d, const Trav& t, Hit& h,
                                           const float4* pre = nullptr) {
  finish_hit(sc, o, d, t.bt, t.bi, h, pre);
}

// Full sample_hit for one ray (k_trace with EXACT, k_render).
template <bool TRIS, bool STATS, bool EXACT = false>
__device__ __forceinline__ void sample_hit(const DevScene& sc, f3 o, f3 d, int* __restrict__ lds,
                                           Hit& h, TravStats& st) {
  if (has_nan(o) || has_nan(d)) {
    nan_hit(sc, o, d, h);
    return;
  }
  float qt;
  uint32_t qprim;
  quad_scan_fast<EXACT>(sc, o, d, qprim, qt);
  quad_rebuild(sc, o, d, qprim, qt, h);
  Trav t;
  trav_init<0, EXACT>(sc, o, d, h.prim != kNoHit, qt, t);
  if (TRIS) {
    while (!trav_step<STATS>(sc, o, d, t, lds, st)) {
    }
  }
  finish_hit(sc, o, d, t, h);
}

struct Light {
  f3 pos, right, up;
};

// raytrace() after sample_hit (path_tracer.wgsl:267-287).  Returns path.end.
__device__ __forceinline__ bool shade(const DevScene& sc, const Light& L, const Hit& h, int depth,
                                      uint32_t& seed, f3& ro, f3& rd, f3& pc) {
  if (h.emissive) {
    if (depth != 0) {
      const float ff = h.front_face ? 1.0f : 0.0f;
      pc = (ff * h.col) * pc;
    } else {
      pc = h.col;
    }
    return true;
  }
  // sample_direction (path_tracer.wgsl:146-154).  The shading divisions stay IEEE: short forms
  // behind per-lane range tests measured slower
  const f3 w = normalize(h.norm);  // onb.w of build_onb_from_w(hit.norm)
  f3 sdir;
  // both branches draw two more rand() (r1 then r2) right away: drawn once here, the
  // same values in the same order
  const bool cosine = rand_next(seed) > 0.5f;
  const float r1 = rand_next(seed);
  const float r2 = rand_next(seed);
  if (cosine) {
    // sample_from_cosine: build_onb_from_w (:133-140) + rand_cos_dir (:123-131)
    const f3 a = (sign_w(w.x) * w.x) > 0.9f ? f3{0.0f, 1.0f, 0.0f} : f3{1.0f, 0.0f, 0.0f};
    // |w| = 1 +- 2^-22 and a is the axis w is furthest from: |w x a|^2 >= 0.19
    const f3 v = normalize_unit(cross(w, a));
    const f3 u = cross(w, v);
    const float z = sqrt_fast(1.0f - r2);
    const float phi = 2.0f * kPI * r1;
    float sphi, cphi;
    sincos_w(phi, sphi, cphi);
    const float sr2 = sqrt_fast(r2);
    const float lx2 = cphi * sr2;
    const float ly2 = sphi * sr2;
    sdir = (lx2 * u + ly2 * v) + z * w;
  } else {
    // sample_from_light (:163-168), not normalised
    sdir = ((L.pos + r1 * L.right) + r2 * L.up) - h.pos;
  }
  // mixture_pdf (:191-193) = 0.5*cosine_pdf + 0.5*light_area_pdf
  const float len = length(sdir);
  const f3 nd = sdir / len;  // normalize(dir): shared by cosine_pdf, the light cosine and :282
  const float cs = dot(nd, w);
  const float cpdf = cs <= 0.0f ? 0.0f : cs * k_1_PI;
  const float dist2 = len * len;
  const float light_cosine = fabs_w(nd.y) + kRayMin;
  const float lpdf = dist2 / (light_cosine * sc.light_area);
  const float pdf_val = 0.5f * cpdf + 0.5f * lpdf;
  // scattering_pdf (:217-220) normalises the already normalised direction again
  const f3 nd2 = normalize_unit(nd);  // nd = sdir / exact length: unit, NaN or 0
  const float cs2 = dot(h.norm, nd2);
  const float spdf = cs2 < 0.0f ? 0.0f : cs2 * k_1_PI;
  pc = (spdf * (pc * h.col)) / pdf_val;
  ro = h.pos;
  rd = nd;
  return false;
}

__device__ __forceinline__ uint8_t unorm8(float x) {
  float c = max0(x);
  c = c < 1.0f ? c : 1.0f;
  return (uint8_t)__builtin_floorf(c * 255.0f + 0.5f);
}

// Per-pixel state shared by both kernels.
struct Pixel {
  uint32_t xy;  // x | y << 16 (frames are at most 65535 x 65535, check_render_args): one register
  uint32_t seed;
  uint32_t sij;  // the sample's s_i | s_j << 16 (sqrt_spp < 2^16); index = s_i + s_j * sqrt_spp
  f3 col;
};
// all sqrt_spp^2 samples done (sj reaches sqrt_spp; at once when spp = 0)
__device__ __forceinline__ uint32_t px_si(const Pixel& px) { return px.sij & 0xffffu; }
__device__ __forceinline__ uint32_t px_sj(const Pixel& px) { return px.sij >> 16; }
__device__ __forceinline__ bool px_done(const DevFrame& fr, const Pixel& px) { return px_sj(px) >= fr.sqrt_spp; }
// next (s_i, s_j) in the reference's loop order (path_tracer.wgsl:381-382)
__device__ __forceinline__ void px_next(const DevFrame& fr, Pixel& px) {
  px.sij = px_si(px) + 1u == fr.sqrt_spp ? (px.sij & 0xffff0000u) + 0x10000u : px.sij + 1u;
}
// sample 0 (the one whose first hit is the pixel's hit ID)
__device__ __forceinline__ bool px_first(const Pixel& px) { return px.sij == 0u; }

struct Counters {
  uint32_t q, tr, nan, lw, ll;
  uint32_t qref;  // rays whose quad scan took the reference path (quad_scan_fast's almost-ties)
  uint32_t px;  // pixels finished by this lane
};

// x / d for d >= 1 with m = (2^32 - 1) / d (host): mulhi(x, m) is x / d or up to two less
// (x m / 2^32 > x / d - x / 2^32 - x / (d 2^32) - 1 > x / d - 3 for x < 2^32), fixed by two steps.
__device__ __forceinline__ uint32_t udiv_by(uint32_t x, uint32_t d, uint32_t m) {
  uint32_t q = __umulhi(x, m);
  uint32_t r = x - q * d;
  if (r >= d) { ++q; r -= d; }
  if (r >= d) ++q;
  return q;
}

// Pixel of pixel slot (block, lane) = (slot >> 6, slot & 63): block b covers an
// 8x8 sub-block of tile b / (sub-blocks per tile).  false if the slot is outside
// its tile or the frame.  po = the pixel's offset in the tile-major output
// ((tile * th + ly) * tw + lx; the host keeps tiles * tw * th < 2^31).
__device__ __forceinline__ bool slot_setup(const DevFrame& fr, const wgt_tile* __restrict__ tiles,
                                           uint32_t block, uint32_t lane, uint32_t& po, Pixel& px) {
  const uint32_t bx = (fr.tw + 7u) >> 3, by = (fr.th + 7u) >> 3;
  const uint32_t bpt = bx * by;
  // divisions by the host's multipliers (DevFrame::div_bx, div_bpt): no per-lane reciprocal kept
  // live through the kernel, where the compiler's division by a runtime value would hoist one
  const uint32_t tile = udiv_by(block, bpt, fr.div_bpt);
  const uint32_t rem = block - tile * bpt;
  const uint32_t ry = udiv_by(rem, bx, fr.div_bx);
  const uint32_t lx = (rem - ry * bx) * 8u + (lane & 7u);
  const uint32_t ly = ry * 8u + (lane >> 3);
  if (tile >= fr.n_tiles || lx >= fr.tw || ly >= fr.th) return false;
  const wgt_tile td = tiles[tile];
  const uint32_t x = td.x0 + lx, y = td.y0 + ly;
  if (x >= fr.W || y >= fr.H) return false;  // path_tracer.wgsl:377
  px.xy = x | y << 16;
  px.seed = x + y * fr.W + td.seed * fr.W * fr.H;  // path_tracer.wgsl:378
  px.sij = 0u;
  px.col = f3{0.0f, 0.0f, 0.0f};
  po = (tile * fr.th + ly) * fr.tw + lx;
  return true;
}

// Pixel of this lane in a one-pixel-per-lane launch, or false if the lane has none.
__device__ __forceinline__ bool pixel_setup(const DevFrame& fr, const wgt_tile* __restrict__ tiles,
                                            uint32_t& po, Pixel& px) {
  return slot_setup(fr, tiles, blockIdx.x, threadIdx.x, po, px);
}

// setup_camera_ray + pixel_sample_square (path_tracer.wgsl:232-262) for the sample (s_i, s_j) of px.sij
__device__ __forceinline__ void camera_ray(const DevFrame& fr, Pixel& px, f3& ro, f3& rd) {
  const f3 origin = f3{fr.ox, fr.oy, fr.oz};
  const f3 du = f3{fr.dux, fr.duy, fr.duz};
  const f3 dv = f3{fr.dvx, fr.dvy, fr.dvz};
  const f3 pixel_center = (f3{fr.pox, fr.poy, fr.poz} + (float)(px.xy & 0xffffu) * du) + (float)(px.xy >> 16) * dv;
  const float sx = -0.5f + fr.recip_sqrt_spp * ((float)px_si(px) + rand_next(px.seed));
  const float sy = -0.5f + fr.recip_sqrt_spp * ((float)px_sj(px) + rand_next(px.seed));
  const f3 pixel_sample = pixel_center + (sx * du + sy * dv);
  ro = origin;
  rd = pixel_sample - origin;
}

// col += max(path.col, 0) / f32(spp) (path_tracer.wgsl:393) and advance to the next sample
__device__ __forceinline__ void end_sample(const DevFrame& fr, Pixel& px, f3 pc) {
  // x / 2^k == x * 2^-k exactly (one rounding of the same real value), so a
  // power-of-two spp multiplies
  const f3 m{max0(pc.x), max0(pc.y), max0(pc.z)};
  px.col = px.col + (fr.inv_fspp != 0.0f ? fr.inv_fspp * m : m / fr.fspp);
  px_next(fr, px);
}

// The pixel's hit ID (path_tracer.wgsl:384-386): the primitive of sample 0's camera ray.
__device__ __forceinline__ void first_hit(const Pixel& px, int depth, uint32_t prim, uint32_t po,
                                          uint32_t* __restrict__ outhit) {
  if (outhit && depth == 0 && px_first(px)) outhit[po] = prim;
}

// NaN-absorbed for the rest of the path: 3 rand() per remaining bounce, colour NaN.
template <bool STATS>
__device__ __forceinline__ void skip_nan_path(const DevScene& sc, const DevFrame& fr, Pixel& px,
                                              int depth, Counters& c) {
  px.seed = lcg_jump(px.seed, 3u * (uint32_t)(kRayDepth - depth));
  if (STATS) {
    c.q += (uint32_t)(kRayDepth - depth);
    c.nan += (uint32_t)(kRayDepth - depth);
  }
  // col += max(NaN, 0) / spp == col + 0
  px_next(fr, px);
}

__device__ __forceinline__ void write_pixel(const DevFrame& fr, uint32_t po, const Pixel& px, uchar4* out8,
                                            float4* out32, uint32_t* outhit) {
  if (out32) out32[po] = make_float4(px.col.x, px.col.y, px.col.z, 1.0f);
  if (out8) out8[po] = make_uchar4(unorm8(px.col.x), unorm8(px.col.y), unorm8(px.col.z), 255);
  // the hit ID is written when sample 0's first hit is known (first_hit); a
  // pixel without samples has none
  if (outhit && fr.sqrt_spp == 0u) outhit[po] = kNoHit;
}

__device__ __forceinline__ void flush_counters(unsigned long long* __restrict__ counters,
                                               const Counters& c, const TravStats& st,
                                               uint32_t nsamp) {
  // c.px pixels, nsamp samples each
  atomicAdd(&counters[CNT_QUERIES], (unsigned long long)c.q);
  atomicAdd(&counters[CNT_TRACED], (unsigned long long)c.tr);
  atomicAdd(&counters[CNT_SAMPLES], (unsigned long long)nsamp * c.px);
  atomicAdd(&counters[CNT_NAN], (unsigned long long)c.nan);
  atomicAdd(&counters[CNT_NODES], (unsigned long long)st.nodes);
  atomicAdd(&counters[CNT_TRIS], (unsigned long long)st.tris);
  atomicAdd(&counters[CNT_PIXELS], (unsigned long long)c.px);
  if (c.qref) atomicAdd(&counters[CNT_QUAD_REF], (unsigned long long)c.qref);
  atomicAdd(&counters[CNT_LOOP_WAVE], (unsigned long long)c.lw);
  atomicAdd(&counters[CNT_LOOP_LANE], (unsigned long long)c.ll);
  atomicAdd(&counters[CNT_TRAV_WAVE], (unsigned long long)st.wave_steps);
  atomicAdd(&counters[CNT_TRAV_LANE], (unsigned long long)st.lane_steps);
  if (st.spills) atomicAdd(&counters[CNT_STACK_SPILLS], (unsigned long long)st.spills);
  if (st.refills) atomicAdd(&counters[CNT_STACK_REFILLS], (unsigned long long)st.refills);
  if (st.overflows) atomicAdd(&counters[CNT_STACK_OVERFLOWS], (unsigned long long)st.overflows);
}


}  // namespace wgt
