// wgt_kernels.hip — the MI355X (gfx950) path-tracing kernels.
//
// One lane per pixel, one wave (64 lanes = 8x8 pixels) per block.  Each lane runs
// its pixel's whole compute_sample (path_tracer.wgsl:374-398); the per-pixel RNG
// stream is serial across samples (path_tracer.wgsl:378, 381-395), so there is no
// sample-level parallelism — parallelism is over pixels only.
//
// sample_hit (path_tracer.wgsl:290-310) = linear scan of lights and quads (scalar
// loads: the scene is wave-uniform), BVH2 traversal over triangles (per-lane LDS
// stack, Moller-Trumbore in fp32, wgt_geom.h), then the sphere scan.
//
// Two kernels compute bit-identical results:
//  * k_render (simple): a flat per-lane loop, one closest-hit query + one shading
//    step per iteration.  Used for scenes without triangles (the Cornell box).
//  * k_render_ps (phase-split, scenes with triangles): the wave alternates a
//    SERVICE phase (finalise the hit of lanes whose traversal ended, shade, start
//    the next ray: camera ray or bounce, quad scan, root-node test) and a
//    TRAVERSAL phase (one BVH node or leaf per lane per step).  A phase ends when
//    too few lanes are left for it (wave-uniform ballot counts), so lanes whose
//    ray left the BVH early pick up new rays while the long traversals continue:
//    the traversal loop runs at 10 % SIMT utilisation in k_render on the bunny
//    stand-in (profiles/r01_*), which this structure removes.
//
// NaN rays (any NaN in start/dir) are resolved without tracing: every rejection
// test of the reference is false for NaN, so the last primitive of the scan — the
// last sphere — wins.  When that sphere is not emissive the path can only
// continue NaN-absorbed to depth 50 with exactly 3 rand() per bounce and a NaN
// colour (contributing max(NaN, 0) = 0), so the LCG is advanced by 3*(50-depth)
// steps in O(8) and the sample ends: bit-identical output, ~2/3 fewer queries on
// the Cornell box.
#include "wgt_device.h"

namespace wgt {

template <bool TRIS, bool STATS>
__global__ void __launch_bounds__(kBlock)
k_render(DevScene sc, DevFrame fr, const wgt_tile* __restrict__ tiles, uchar4* __restrict__ out8,
         float4* __restrict__ out32, uint32_t* __restrict__ outhit,
         unsigned long long* __restrict__ counters) {
  __shared__ int s_stack[kStackLds * kBlock];
  uint32_t tile, lx, ly;
  Pixel px;
  if (!pixel_setup(fr, tiles, tile, lx, ly, px)) return;
  int* lds = s_stack + threadIdx.x;
  const Light L{xyz(sc.quads[0]), xyz(sc.quads[1]), xyz(sc.quads[2])};
  const uint32_t nsamp = fr.sqrt_spp * fr.sqrt_spp;
  f3 ro{}, rd{}, pc{};
  int depth = 0;
  TravStats st{0u, 0u, 0u, 0u};
  Counters c{0u, 0u, 0u, 0u, 0u};

  while (px.k < nsamp) {
    if (STATS) simt_count(c.lw, c.ll);
    if (depth == 0) {
      camera_ray(fr, px, ro, rd);
      pc = f3{1.0f, 1.0f, 1.0f};
    }
    const bool nanray = has_nan(ro) || has_nan(rd);
    if (nanray && !sc.last_sphere_emissive) {
      skip_nan_path<STATS>(sc, fr, px, depth, c);
      depth = 0;
      continue;
    }
    Hit h;
    sample_hit<TRIS, STATS>(sc, ro, rd, lds, h, st);
    if (STATS) {
      ++c.q;
      if (nanray) ++c.nan; else ++c.tr;
    }
    if (px.k == 0 && depth == 0) px.hit0 = h.prim;
    const bool end = shade(sc, L, h, depth, px.seed, ro, rd, pc);
    ++depth;
    if (end || depth == kRayDepth) {
      end_sample(fr, px, pc);
      depth = 0;
    }
  }
  write_pixel(fr, tile, lx, ly, px, out8, out32, outhit);
  if (STATS) flush_counters(counters, c, st, nsamp);
}

// Phase-split kernel for scenes with triangles (see the file comment).
template <bool STATS>
__global__ void __launch_bounds__(kBlock)
k_render_ps(DevScene sc, DevFrame fr, const wgt_tile* __restrict__ tiles, uchar4* __restrict__ out8,
            float4* __restrict__ out32, uint32_t* __restrict__ outhit,
            unsigned long long* __restrict__ counters) {
  __shared__ int s_stack[kStackLds * kBlock];
  uint32_t tile, lx, ly;
  Pixel px;
  if (!pixel_setup(fr, tiles, tile, lx, ly, px)) return;
  int* lds = s_stack + threadIdx.x;
  const Light L{xyz(sc.quads[0]), xyz(sc.quads[1]), xyz(sc.quads[2])};
  const uint32_t nsamp = fr.sqrt_spp * fr.sqrt_spp;
  f3 ro{}, rd{}, pc{};
  int depth = 0;
  TravStats st{0u, 0u, 0u, 0u};
  Counters c{0u, 0u, 0u, 0u, 0u};
  Trav t;
  uint32_t q_prim = kNoHit;  // quad part of the pending hit, rebuilt at finalisation
  float q_t = kRayMax;
  bool done = nsamp == 0, trav = false, pending = false;
  uint64_t cyc_svc = 0, cyc_trav = 0;

  for (;;) {
    // ------------------------------------------------------------ service phase
    uint64_t t_phase = STATS ? __builtin_amdgcn_s_memtime() : 0;
    for (;;) {
      const bool need = !trav && !done;
      if (!__any(need)) break;
      if (need) {
        if (STATS) simt_count(c.lw, c.ll);
        if (pending) {
          // finalise: rebuild the quad hit, merge triangles, scan spheres, shade
          Hit h;
          quad_rebuild(sc, ro, rd, q_prim, q_t, h);
          finish_hit(sc, ro, rd, t, h);
          if (STATS) { ++c.q; ++c.tr; }
          if (px.k == 0 && depth == 0) px.hit0 = h.prim;
          const bool end = shade(sc, L, h, depth, px.seed, ro, rd, pc);
          ++depth;
          if (end || depth == kRayDepth) {
            end_sample(fr, px, pc);
            depth = 0;
          }
          pending = false;
        }
        // start the next ray of this pixel
        for (;;) {
          if (px.k >= nsamp) {
            done = true;
            break;
          }
          if (depth == 0) {
            camera_ray(fr, px, ro, rd);
            pc = f3{1.0f, 1.0f, 1.0f};
          }
          if (has_nan(ro) || has_nan(rd)) {
            if (!sc.last_sphere_emissive) {
              skip_nan_path<STATS>(sc, fr, px, depth, c);
              depth = 0;
              continue;
            }
            Hit h;  // emissive last sphere: resolve the NaN ray here (no traversal)
            nan_hit(sc, ro, rd, h);
            if (STATS) { ++c.q; ++c.nan; }
            if (px.k == 0 && depth == 0) px.hit0 = h.prim;
            const bool end = shade(sc, L, h, depth, px.seed, ro, rd, pc);
            ++depth;
            if (end || depth == kRayDepth) {
              end_sample(fr, px, pc);
              depth = 0;
            }
            continue;
          }
          Hit h;
          quad_scan(sc, ro, rd, h, q_t);
          q_prim = h.prim;
          trav_init(ro, rd, q_prim != kNoHit, q_t, t);
          // the root node is tested here: rays that miss both root children never
          // enter the traversal phase
          if (trav_step<STATS>(sc, ro, rd, t, lds, st)) pending = true;
          else trav = true;
          break;
        }
      }
      if ((uint32_t)__popcll(__ballot(trav)) >= fr.ps_to_trav) break;
    }
    if (STATS) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      cyc_svc += now - t_phase;
      t_phase = now;
    }
    if (!__any(!done)) break;
    // --------------------------------------------------------- traversal phase
    for (;;) {
      if (trav && trav_step<STATS>(sc, ro, rd, t, lds, st)) {
        trav = false;
        pending = true;
      }
      const uint32_t ntrav = (uint32_t)__popcll(__ballot(trav));
      if (ntrav == 0) break;
      if (ntrav <= fr.ps_to_service && __any(!trav && !done)) break;
    }
    if (STATS) cyc_trav += __builtin_amdgcn_s_memtime() - t_phase;
  }
  write_pixel(fr, tile, lx, ly, px, out8, out32, outhit);
  if (STATS) {
    flush_counters(counters, c, st, nsamp);
    if (__lane_id() == (unsigned)(__ffsll((long long)__ballot(1)) - 1)) {
      atomicAdd(&counters[CNT_CYC_SERVICE], (unsigned long long)cyc_svc);
      atomicAdd(&counters[CNT_CYC_TRAV], (unsigned long long)cyc_trav);
    }
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
  TravStats st{0u, 0u, 0u, 0u};
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
  const bool ps = tris && fr.kernel == 2;
  if (counters) {
    if (ps) k_render_ps<true><<<grid, block, 0, stream>>>(sc, fr, d_tiles, out8, out32, outhit, counters);
    else if (tris) k_render<true, true><<<grid, block, 0, stream>>>(sc, fr, d_tiles, out8, out32, outhit, counters);
    else k_render<false, true><<<grid, block, 0, stream>>>(sc, fr, d_tiles, out8, out32, outhit, counters);
  } else {
    if (ps) k_render_ps<false><<<grid, block, 0, stream>>>(sc, fr, d_tiles, out8, out32, outhit, nullptr);
    else if (tris) k_render<true, false><<<grid, block, 0, stream>>>(sc, fr, d_tiles, out8, out32, outhit, nullptr);
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
