// wgt_kernels.hip — the MI355X (gfx950) path-tracing kernels.
//
// k_render: one lane per pixel, one wave (64 lanes = 8x8 pixels) per block.  Each
// lane runs its pixel's whole compute_sample (path_tracer.wgsl:374-398) as a flat
// state machine — one closest-hit query + one shading step per loop iteration — so
// the 64 lanes of a wave stay converged on the trace even when their paths are at
// different samples/bounces.  The per-pixel RNG stream is serial across samples
// (path_tracer.wgsl:378, 381-395), so there is no sample-level parallelism.
//
// sample_hit (path_tracer.wgsl:290-310) = linear scan of lights and quads (scalar
// loads: the scene is wave-uniform), BVH2 traversal over triangles (per-lane
// LDS stack, Moller-Trumbore in fp32, wgt_geom.h), then the sphere scan.
//
// NaN rays (any NaN in start/dir) are resolved without tracing: every rejection
// test of the reference is false for NaN, so the last primitive of the scan — the
// last sphere — wins.  When that sphere is not emissive the path can only
// continue NaN-absorbed to depth 50 with exactly 3 rand() per bounce and a NaN
// colour (contributing max(NaN, 0) = 0), so the LCG is advanced by 3*(50-depth)
// steps in O(8) and the sample ends: bit-identical output, ~2/3 fewer queries on
// the Cornell box.
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

// path_tracer.wgsl:314-338.  `qt` receives t of the accepted quad (used only as
// a conservative bound for the triangle search).
__device__ __forceinline__ void isect_quad(f3 o, f3 d, const float4* __restrict__ q, uint32_t id,
                                           Hit& h, float& qt) {
  const f3 qn = xyz(q[3]);
  const float denom = dot(qn, d);
  if (fabs_w(denom) < kRayMin) return;
  const float4 wd = q[4];
  const float t = (wd.w - dot(qn, o)) / denom;
  if (t < kRayMin || kRayMax < t) return;
  const f3 pos = o + t * d;
  const float ray_dist = distance(pos, o);
  if (ray_dist >= h.dist) return;
  const f3 hit_vec = pos - xyz(q[0]);
  const f3 w = xyz(wd);
  const float a = dot(w, cross(hit_vec, xyz(q[2])));
  const float b = dot(w, cross(xyz(q[1]), hit_vec));
  if ((a < 0.0f) || (1.0f < a) || (b < 0.0f) || (1.0f < b)) return;
  const bool ff = dot(d, qn) < 0.0f;
  const float4 c = q[5];
  h.dist = ray_dist;
  h.prim = id;
  h.emissive = c.w > 0.0f;
  h.front_face = ff;
  h.pos = pos;
  h.norm = ff ? qn : -qn;
  h.col = xyz(c);
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
  const float sqrt_d = __builtin_sqrtf(disc);
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

struct TravStats {
  uint32_t nodes, tris;
};

// Closest triangle = min (t, index) with t < bound (or t <= bound and index < bi
// when bi = kNoHit).  Per-lane stack: kStackLds entries in LDS (stride kBlock,
// conflict-free), overflow in private memory.
template <bool STATS>
__device__ __forceinline__ bool bvh_closest(const DevScene& sc, f3 o, f3 d, float& best_t,
                                            uint32_t& best_i, int* __restrict__ lds,
                                            TravStats& st) {
  const f3 inv = f3{safe_inv(d.x), safe_inv(d.y), safe_inv(d.z)};
  int priv[kStackScratch];
  int sp = 0;
  int ref = 0;
  bool found = false;
  uint32_t iters = 0;
  for (;;) {
    if (ref >= 0) {
      const float4* __restrict__ n = sc.nodes + 4 * ref;
      const float4 a = n[0], b = n[1], c = n[2], e = n[3];
      if (STATS) st.nodes++;
      float n0, f0, n1, f1;
      slab(o, inv, f3{a.x, a.z, c.x}, f3{a.y, a.w, c.y}, n0, f0);
      slab(o, inv, f3{b.x, b.z, c.z}, f3{b.y, b.w, c.w}, n1, f1);
      const bool h0 = (n0 <= f0) & (n0 <= best_t) & (f0 >= kRayMin);
      const bool h1 = (n1 <= f1) & (n1 <= best_t) & (f1 >= kRayMin);
      const int r0 = __float_as_int(e.x), r1 = __float_as_int(e.y);
      if (h0 && h1) {
        const bool swap = n1 < n0;
        const int nearr = swap ? r1 : r0;
        const int farr = swap ? r0 : r1;
        if (sp < kStackLds) lds[sp * kBlock] = farr;
        else if (sp < kStackLds + kStackScratch) priv[sp - kStackLds] = farr;
        ++sp;
        ref = nearr;
        continue;
      }
      if (h0) { ref = r0; continue; }
      if (h1) { ref = r1; continue; }
    } else {
      const uint32_t first = leaf_first(ref), cnt = leaf_count(ref);
      for (uint32_t k = 0; k < cnt; ++k) {
        const float4* __restrict__ tp = sc.tris + 3 * (first + k);
        const float4 A = tp[0], B = tp[1], C = tp[2];
        if (STATS) st.tris++;
        const f3 v0 = xyz(A), e1 = xyz(B), e2 = xyz(C);
        float t;
        if (mt_test(o, d, v0, e1, e2, t)) {
          const uint32_t idx = __float_as_uint(A.w);
          if (t < best_t || (t == best_t && idx < best_i)) {
            f3 lo, hi;
            tri_box(v0, e1, e2, lo, hi);
            float bn, bf;
            slab(o, inv, lo, hi, bn, bf);
            if (bn <= t && t <= bf) {
              best_t = t;
              best_i = idx;
              found = true;
            }
          }
        }
      }
    }
    if (sp == 0 || ++iters > sc.max_iters) break;
    --sp;
    ref = sp < kStackLds ? lds[sp * kBlock] : priv[sp - kStackLds];
  }
  return found;
}

// sample_hit (path_tracer.wgsl:290-310) + triangles between quads and spheres.
template <bool TRIS, bool STATS>
__device__ __forceinline__ void sample_hit(const DevScene& sc, f3 o, f3 d, int* __restrict__ lds,
                                           Hit& h, TravStats& st) {
  hit_init(h);
  const uint32_t nlq = sc.n_lights + sc.n_quads;
  if (has_nan(o) || has_nan(d)) {
    // every rejection is false for NaN: the last primitive scanned wins
    const uint32_t k = sc.n_spheres - 1;
    isect_sphere(o, d, sc.spheres + 2 * k, nlq + sc.n_tris + k, h);
    return;
  }
  float qt = kRayMax;
  for (uint32_t k = 0; k < nlq; ++k) isect_quad(o, d, sc.quads + 6 * k, k, h, qt);
  if (TRIS) {
    float bt = kRayMax;
    uint32_t bi = kNoHit;
    if (h.prim != kNoHit) {  // a triangle must satisfy t < t_quad to win (ray_dist is monotone in t)
      bt = qt;
      bi = 0u;
    }
    if (bvh_closest<STATS>(sc, o, d, bt, bi, lds, st)) {
      const f3 pos = o + bt * d;
      const float ray_dist = distance(pos, o);
      if (!(ray_dist >= h.dist)) {
        const float4 s0 = sc.tshade[2 * bi], s1 = sc.tshade[2 * bi + 1];
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
  }
  for (uint32_t k = 0; k < sc.n_spheres; ++k)
    isect_sphere(o, d, sc.spheres + 2 * k, nlq + sc.n_tris + k, h);
}

__device__ __forceinline__ uint8_t unorm8(float x) {
  float c = max0(x);
  c = c < 1.0f ? c : 1.0f;
  return (uint8_t)__builtin_floorf(c * 255.0f + 0.5f);
}

template <bool TRIS, bool STATS>
__global__ void __launch_bounds__(kBlock)
k_render(DevScene sc, DevFrame fr, const wgt_tile* __restrict__ tiles, uchar4* __restrict__ out8,
         float4* __restrict__ out32, uint32_t* __restrict__ outhit,
         unsigned long long* __restrict__ counters) {
  __shared__ int s_stack[kStackLds * kBlock];
  const uint32_t bx = (fr.tw + 7u) >> 3, by = (fr.th + 7u) >> 3;
  const uint32_t bpt = bx * by;
  const uint32_t tile = blockIdx.x / bpt;
  const uint32_t rem = blockIdx.x - tile * bpt;
  const uint32_t lx = (rem % bx) * 8u + (threadIdx.x & 7u);
  const uint32_t ly = (rem / bx) * 8u + (threadIdx.x >> 3);
  if (tile >= fr.n_tiles || lx >= fr.tw || ly >= fr.th) return;
  const wgt_tile td = tiles[tile];
  const uint32_t x = td.x0 + lx, y = td.y0 + ly;
  if (x >= fr.W || y >= fr.H) return;  // path_tracer.wgsl:377
  int* lds = s_stack + threadIdx.x;

  // path_tracer.wgsl:378
  uint32_t seed = x + y * fr.W + td.seed * fr.W * fr.H;
  const f3 origin = f3{fr.ox, fr.oy, fr.oz};
  const f3 du = f3{fr.dux, fr.duy, fr.duz};
  const f3 dv = f3{fr.dvx, fr.dvy, fr.dvz};
  // pixel_center (path_tracer.wgsl:258), frame-invariant per pixel
  const f3 pixel_center = (f3{fr.pox, fr.poy, fr.poz} + (float)x * du) + (float)y * dv;
  const float4 L0 = sc.quads[0], L1 = sc.quads[1], L2 = sc.quads[2];
  const f3 lpos = xyz(L0), lright = xyz(L1), lup = xyz(L2);

  f3 col = f3{0.0f, 0.0f, 0.0f};
  f3 ro = origin, rd = origin, pc = f3{1.0f, 1.0f, 1.0f};
  const uint32_t nsamp = fr.sqrt_spp * fr.sqrt_spp;
  uint32_t k = 0, si = 0, sj = 0;
  int depth = 0;
  uint32_t hit0 = kNoHit;
  TravStats st{0u, 0u};
  uint32_t c_q = 0, c_tr = 0, c_nan = 0;

  while (k < nsamp) {
    if (depth == 0) {
      // setup_camera_ray + pixel_sample_square (path_tracer.wgsl:232-262)
      const float px = -0.5f + fr.recip_sqrt_spp * ((float)si + rand_next(seed));
      const float py = -0.5f + fr.recip_sqrt_spp * ((float)sj + rand_next(seed));
      const f3 pixel_sample = pixel_center + (px * du + py * dv);
      ro = origin;
      rd = pixel_sample - origin;
      pc = f3{1.0f, 1.0f, 1.0f};
    }
    Hit h;
    const bool nanray = has_nan(ro) || has_nan(rd);
    if (nanray && !sc.last_sphere_emissive) {
      // NaN-absorbed for the rest of the path: 3 rand() per remaining bounce.
      seed = lcg_jump(seed, 3u * (uint32_t)(kRayDepth - depth));
      if (STATS) {
        c_q += (uint32_t)(kRayDepth - depth);
        c_nan += (uint32_t)(kRayDepth - depth);
      }
      if (k == 0 && depth == 0) hit0 = sc.n_lights + sc.n_quads + sc.n_tris + sc.n_spheres - 1u;
      // col += max(NaN, 0) / spp == col + 0
      depth = 0;
      ++k;
      if (++si == fr.sqrt_spp) { si = 0; ++sj; }
      continue;
    }
    sample_hit<TRIS, STATS>(sc, ro, rd, lds, h, st);
    if (STATS) {
      ++c_q;
      if (nanray) ++c_nan; else ++c_tr;
    }
    if (k == 0 && depth == 0) hit0 = h.prim;

    // raytrace (path_tracer.wgsl:264-288)
    bool end;
    if (h.emissive) {
      end = true;
      if (depth != 0) {
        const float ff = h.front_face ? 1.0f : 0.0f;
        pc = (ff * h.col) * pc;
      } else {
        pc = h.col;
      }
    } else {
      end = false;
      // sample_direction (path_tracer.wgsl:146-154)
      const f3 w = normalize(h.norm);  // onb.w of build_onb_from_w(hit.norm)
      f3 sdir;
      if (rand_next(seed) > 0.5f) {
        // sample_from_cosine: build_onb_from_w (:133-140) + rand_cos_dir (:123-131)
        const f3 a = (sign_w(w.x) * w.x) > 0.9f ? f3{0.0f, 1.0f, 0.0f} : f3{1.0f, 0.0f, 0.0f};
        const f3 v = normalize(cross(w, a));
        const f3 u = cross(w, v);
        const float r1 = rand_next(seed);
        const float r2 = rand_next(seed);
        const float z = __builtin_sqrtf(1.0f - r2);
        const float phi = 2.0f * kPI * r1;
        float sphi, cphi;
        sincos_w(phi, sphi, cphi);
        const float sr2 = __builtin_sqrtf(r2);
        const float lx2 = cphi * sr2;
        const float ly2 = sphi * sr2;
        sdir = (lx2 * u + ly2 * v) + z * w;
      } else {
        // sample_from_light (:163-168), not normalised
        const float r1 = rand_next(seed);
        const float r2 = rand_next(seed);
        sdir = ((lpos + r1 * lright) + r2 * lup) - h.pos;
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
      const f3 nd2 = normalize(nd);
      const float cs2 = dot(h.norm, nd2);
      const float spdf = cs2 < 0.0f ? 0.0f : cs2 * k_1_PI;
      pc = (spdf * (pc * h.col)) / pdf_val;
      ro = h.pos;
      rd = nd;
    }
    ++depth;
    if (end || depth == kRayDepth) {
      col = col + f3{max0(pc.x) / fr.fspp, max0(pc.y) / fr.fspp, max0(pc.z) / fr.fspp};
      depth = 0;
      ++k;
      if (++si == fr.sqrt_spp) { si = 0; ++sj; }
    }
  }

  const size_t o = ((size_t)tile * fr.th + ly) * fr.tw + lx;
  if (out32) out32[o] = make_float4(col.x, col.y, col.z, 1.0f);
  if (out8) out8[o] = make_uchar4(unorm8(col.x), unorm8(col.y), unorm8(col.z), 255);
  if (outhit) outhit[o] = hit0;
  if (STATS) {
    atomicAdd(&counters[CNT_QUERIES], (unsigned long long)c_q);
    atomicAdd(&counters[CNT_TRACED], (unsigned long long)c_tr);
    atomicAdd(&counters[CNT_SAMPLES], (unsigned long long)nsamp);
    atomicAdd(&counters[CNT_NAN], (unsigned long long)c_nan);
    atomicAdd(&counters[CNT_NODES], (unsigned long long)st.nodes);
    atomicAdd(&counters[CNT_TRIS], (unsigned long long)st.tris);
    atomicAdd(&counters[CNT_PIXELS], 1ull);
  }
}

template <bool TRIS>
__global__ void __launch_bounds__(kBlock)
k_trace(DevScene sc, const float* __restrict__ rays, uint32_t n, uint32_t* __restrict__ prim,
        float* __restrict__ dist) {
  __shared__ int s_stack[kStackLds * kBlock];
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const f3 o = f3{rays[i], rays[(size_t)n + i], rays[2 * (size_t)n + i]};
  const f3 d = f3{rays[3 * (size_t)n + i], rays[4 * (size_t)n + i], rays[5 * (size_t)n + i]};
  Hit h;
  TravStats st{0u, 0u};
  sample_hit<TRIS, false>(sc, o, d, s_stack + threadIdx.x, h, st);
  prim[i] = h.prim;
  dist[i] = h.dist;
}

hipError_t launch_render(const DevScene& sc, const DevFrame& fr, const wgt_tile* d_tiles,
                         uchar4* out8, float4* out32, uint32_t* outhit,
                         unsigned long long* counters, hipStream_t stream) {
  const uint32_t bx = (fr.tw + 7u) / 8u, by = (fr.th + 7u) / 8u;
  const uint64_t blocks = (uint64_t)bx * by * fr.n_tiles;
  if (blocks == 0) return hipSuccess;
  if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
  const dim3 grid((uint32_t)blocks), block(kBlock);
  const bool tris = sc.n_tris > 0;
  if (counters) {
    if (tris) k_render<true, true><<<grid, block, 0, stream>>>(sc, fr, d_tiles, out8, out32, outhit, counters);
    else k_render<false, true><<<grid, block, 0, stream>>>(sc, fr, d_tiles, out8, out32, outhit, counters);
  } else {
    if (tris) k_render<true, false><<<grid, block, 0, stream>>>(sc, fr, d_tiles, out8, out32, outhit, nullptr);
    else k_render<false, false><<<grid, block, 0, stream>>>(sc, fr, d_tiles, out8, out32, outhit, nullptr);
  }
  return hipGetLastError();
}

hipError_t launch_trace(const DevScene& sc, const float* d_rays, uint32_t n, uint32_t* prim,
                        float* dist, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const dim3 grid((n + kBlock - 1) / kBlock), block(kBlock);
  if (sc.n_tris > 0) k_trace<true><<<grid, block, 0, stream>>>(sc, d_rays, n, prim, dist);
  else k_trace<false><<<grid, block, 0, stream>>>(sc, d_rays, n, prim, dist);
  return hipGetLastError();
}

}  // namespace wgt
