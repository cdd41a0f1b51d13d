// wgt_wavefront.hip — wavefront path tracer for scenes with triangles.
//
// The megakernels keep a path in registers and trace it in the same lanes, so a
// wave waits for its longest traversal: 15-33 % SIMT utilisation in the BVH loop
// on the bunny stand-in (profiles/r01_*).  Here every pixel is a SLOT whose path
// state lives in SoA arrays in HBM (they stay in the 256 MB Infinity Cache at
// 1080p), and each bounce iteration is two launches:
//
//   k_wf_shade  one thread per slot: finalise the hit the trace kernel returned
//               (quad rebuilt from (prim, t), triangle merged, spheres scanned),
//               shade (raytrace, path_tracer.wgsl:264-288), then start the next
//               ray (camera ray / bounce, NaN skip-ahead, quad scan, BVH-root
//               test).  A ray that misses the root's child boxes is finished on
//               the spot; one that needs the BVH is left in its slot, marked WAIT.
//   k_wf_trace  one wave per chunk of C slots: ballot-compacts the WAIT slots of
//               the chunk into an LDS list, then traverses them with in-wave
//               dynamic fetch — a lane whose traversal ends takes the next ray of
//               the list — so lanes stay busy until the list runs dry.  Lean (no
//               shading state): more waves per SIMD to hide node-fetch latency.
//
// Both kernels are built from the same device functions as the megakernels
// (wgt_device.h), so all three compute bit-identical images.
#include <hip/hip_runtime.h>

#include "wgt_device.h"

namespace wgt {

enum : uint32_t { PH_NEED = 0u, PH_WAIT = 1u, PH_DONE = 2u };

constexpr int kWfShadeBlock = 256;
constexpr int kWfChunkMax = 1024;


__device__ __forceinline__ f3 ld3(const float* p, uint32_t n, uint32_t i) {
  return f3{p[i], p[n + i], p[2 * n + i]};
}
__device__ __forceinline__ void st3(float* p, uint32_t n, uint32_t i, f3 v) {
  p[i] = v.x;
  p[n + i] = v.y;
  p[2 * n + i] = v.z;
}

// slot -> pixel of the tile list (compact tile-major output order == slot order)
__device__ __forceinline__ bool slot_pixel(const DevFrame& fr, const wgt_tile* __restrict__ tiles,
                                           uint32_t s, uint32_t& x, uint32_t& y, uint32_t& tseed) {
  const uint32_t per = fr.tw * fr.th;
  const uint32_t tile = s / per;
  const uint32_t r = s - tile * per;
  const uint32_t ly = r / fr.tw, lx = r - ly * fr.tw;
  const wgt_tile td = tiles[tile];
  x = td.x0 + lx;
  y = td.y0 + ly;
  tseed = td.seed;
  return x < fr.W && y < fr.H;  // path_tracer.wgsl:377
}

__global__ void __launch_bounds__(kWfShadeBlock)
k_wf_init(DevFrame fr, const wgt_tile* __restrict__ tiles, WfState st, uchar4* __restrict__ out8,
          float4* __restrict__ out32, uint32_t* __restrict__ outhit) {
  const uint32_t s = blockIdx.x * kWfShadeBlock + threadIdx.x;
  if (s >= st.n) return;
  uint32_t x, y, tseed;
  const bool in = slot_pixel(fr, tiles, s, x, y, tseed);
  const uint32_t nsamp = fr.sqrt_spp * fr.sqrt_spp;
  st.col[s] = 0.0f;
  st.col[st.n + s] = 0.0f;
  st.col[2 * st.n + s] = 0.0f;
  st.k[s] = 0u;
  if (!in || nsamp == 0) {
    st.dp[s] = PH_DONE << 8;
    if (in) {  // compute_sample with no samples: black, no primary hit
      if (out32) out32[s] = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
      if (out8) out8[s] = make_uchar4(0, 0, 0, 255);
      if (outhit) outhit[s] = kNoHit;
    }
    atomicAdd(&st.ctl[0], 1ull);
    return;
  }
  st.seed[s] = x + y * fr.W + tseed * fr.W * fr.H;  // path_tracer.wgsl:378
  st.dp[s] = PH_NEED << 8;
}

// The first traversal step on the root decides whether a ray needs the BVH at all.
__device__ __forceinline__ bool root_needs_trav(const DevScene& sc, f3 o, f3 d, bool quad_hit, float qt) {
  Trav t;
  trav_init(sc, o, d, quad_hit, qt, t);
  uint32_t k0, k1, k2, k3;
  int r0, r1, r2, r3;
  node_keys<false>(sc, t, 0, k0, k1, k2, k3, r0, r1, r2, r3);
  return (k0 & k1 & k2 & k3) != kMissKey;  // a hit key has bit 31 clear
}

template <bool STATS>
__global__ void __launch_bounds__(kWfShadeBlock)
k_wf_shade(DevScene sc, DevFrame fr, const wgt_tile* __restrict__ tiles, WfState st,
           uchar4* __restrict__ out8, float4* __restrict__ out32, uint32_t* __restrict__ outhit,
           unsigned long long* __restrict__ counters) {
  const uint32_t s = blockIdx.x * kWfShadeBlock + threadIdx.x;
  if (s >= st.n) return;
  const uint32_t dp = st.dp[s];
  uint32_t phase = dp >> 8;
  if (phase == PH_DONE) return;
  int depth = (int)(dp & 0xffu);
  const uint32_t n = st.n;
  const uint32_t nsamp = fr.sqrt_spp * fr.sqrt_spp;
  const Light L{xyz(sc.quads[0]), xyz(sc.quads[1]), xyz(sc.quads[2])};
  Pixel px;
  uint32_t tseed;
  slot_pixel(fr, tiles, s, px.x, px.y, tseed);
  px.seed = st.seed[s];
  {
    const uint32_t k = st.k[s];
    px.sij = (k % fr.sqrt_spp) | ((k / fr.sqrt_spp) << 16);
  }
  px.col = ld3(st.col, n, s);
  f3 pc = ld3(st.pc, n, s);
  f3 ro = ld3(st.ro, n, s);
  f3 rd = ld3(st.rd, n, s);
  Counters c{0u, 0u, 0u, 0u, 0u, 0u};
  TravStats ts{0u, 0u, 0u, 0u};

  auto shade_and_advance = [&](const Hit& h) {
    if (px_first(px) && depth == 0 && outhit) outhit[s] = h.prim;
    const bool end = shade(sc, L, h, depth, px.seed, ro, rd, pc);
    ++depth;
    if (end || depth == kRayDepth) {
      end_sample(fr, px, pc);
      depth = 0;
    }
  };

  if (phase == PH_WAIT) {
    Hit h;
    quad_rebuild(sc, ro, rd, st.qprim[s], st.qt[s], h);
    Trav t;
    t.bi = st.res_i[s];
    t.bt = st.res_t[s];
    finish_hit(sc, ro, rd, t, h);
    if (STATS) { ++c.q; ++c.tr; }
    shade_and_advance(h);
  }
  // start rays until one needs the BVH (at most fr.wf_rays that reach the quad scan)
  uint32_t started = 0;
  for (;;) {
    if (STATS) simt_count(c.lw, c.ll);
    if (px_done(fr, px)) {
      if (out32) out32[s] = make_float4(px.col.x, px.col.y, px.col.z, 1.0f);
      if (out8) out8[s] = make_uchar4(unorm8(px.col.x), unorm8(px.col.y), unorm8(px.col.z), 255);
      phase = PH_DONE;
      atomicAdd(&st.ctl[0], 1ull);
      break;
    }
    if (started == fr.wf_rays) {
      phase = PH_NEED;
      break;
    }
    if (depth == 0) {
      camera_ray(fr, px, ro, rd);
      pc = f3{1.0f, 1.0f, 1.0f};
    }
    if (has_nan(ro) || has_nan(rd)) {
      if (!sc.last_sphere_emissive) {
        if (px_first(px) && depth == 0 && outhit) outhit[s] = last_prim(sc);
        skip_nan_path<STATS>(sc, fr, px, depth, c);
        depth = 0;
        continue;
      }
      Hit h;
      nan_hit(sc, ro, rd, h);
      if (STATS) { ++c.q; ++c.nan; }
      shade_and_advance(h);
      continue;
    }
    ++started;
    Hit h;
    float qt;
    quad_scan(sc, ro, rd, h, qt);
    if (STATS) ts.nodes++;  // the root node fetch
    if (root_needs_trav(sc, ro, rd, h.prim != kNoHit, qt)) {
      st.qprim[s] = h.prim;
      st.qt[s] = qt;
      phase = PH_WAIT;
      break;
    }
    Trav none;
    none.bi = kNoHit;
    finish_hit(sc, ro, rd, none, h);
    if (STATS) { ++c.q; ++c.tr; }
    shade_and_advance(h);
  }
  st.dp[s] = (uint32_t)depth | (phase << 8);
  st.seed[s] = px.seed;
  st.k[s] = px_si(px) + px_sj(px) * fr.sqrt_spp;
  st3(st.col, n, s, px.col);
  if (phase != PH_DONE) {
    st3(st.pc, n, s, pc);
    st3(st.ro, n, s, ro);
    st3(st.rd, n, s, rd);
  }
  if (STATS) {
    atomicAdd(&counters[CNT_QUERIES], (unsigned long long)c.q);
    atomicAdd(&counters[CNT_TRACED], (unsigned long long)c.tr);
    atomicAdd(&counters[CNT_NAN], (unsigned long long)c.nan);
    atomicAdd(&counters[CNT_NODES], (unsigned long long)ts.nodes);
    atomicAdd(&counters[CNT_LOOP_WAVE], (unsigned long long)c.lw);
    atomicAdd(&counters[CNT_LOOP_LANE], (unsigned long long)c.ll);
    if (phase == PH_DONE) {
      atomicAdd(&counters[CNT_SAMPLES], (unsigned long long)nsamp);
      atomicAdd(&counters[CNT_PIXELS], 1ull);
    }
  }
}

template <bool STATS>
__global__ void __launch_bounds__(kBlock)
k_wf_trace(DevScene sc, DevFrame fr, WfState st, unsigned long long* __restrict__ counters) {
  __shared__ uint32_t s_list[kWfChunkMax];
  extern __shared__ int s_stack[];  // sc.stack entries per lane (stack_lds_bytes)
  const uint32_t C = fr.wf_chunk;
  const uint32_t base = blockIdx.x * C;
  if (base >= st.n) return;
  const uint32_t lane = threadIdx.x;
  const unsigned long long lt_mask = (1ull << lane) - 1ull;
  // ballot-compact the WAIT slots of this chunk into the LDS list
  uint32_t cnt = 0;
  for (uint32_t j = 0; j < C; j += kBlock) {
    const uint32_t s = base + j + lane;
    const bool v = s < st.n && (st.dp[s] >> 8) == PH_WAIT;
    const unsigned long long m = __ballot(v);
    if (v) s_list[cnt + __popcll(m & lt_mask)] = s;
    cnt += (uint32_t)__popcll(m);
  }
  __syncthreads();
  if (cnt == 0) return;
  int* lds = s_stack + lane;
  TravStats ts{0u, 0u, 0u, 0u};
  uint32_t next = 0;
  bool active = false;
  uint32_t slot = 0;
  f3 o{}, d{};
  Trav t;
  for (;;) {
    const unsigned long long idle = __ballot(!active);
    const uint32_t n_idle = (uint32_t)__popcll(idle);
    if (next < cnt && (n_idle >= fr.wf_refill || n_idle == (uint32_t)kBlock)) {
      if (!active) {
        const uint32_t j = next + (uint32_t)__popcll(idle & lt_mask);
        if (j < cnt) {
          slot = s_list[j];
          o = ld3(st.ro, st.n, slot);
          d = ld3(st.rd, st.n, slot);
          const uint32_t qp = st.qprim[slot];
          trav_init(sc, o, d, qp != kNoHit, st.qt[slot], t);
          active = true;
        }
      }
      next += n_idle;
    }
    if (!__any(active)) break;
    if (active && trav_step<STATS>(sc, o, d, t, lds, ts)) {
      st.res_i[slot] = t.bi;
      st.res_t[slot] = t.bt;
      active = false;
    }
  }
  if (STATS) {
    atomicAdd(&counters[CNT_NODES], (unsigned long long)ts.nodes);
    atomicAdd(&counters[CNT_TRIS], (unsigned long long)ts.tris);
    atomicAdd(&counters[CNT_TRAV_WAVE], (unsigned long long)ts.wave_steps);
    atomicAdd(&counters[CNT_TRAV_LANE], (unsigned long long)ts.lane_steps);
  }
}

size_t wf_state_bytes(uint32_t n) { return (size_t)n * 4 * (3 + 3 * 4 + 2 + 2); }

hipError_t wf_bind(void* mem, uint32_t n, unsigned long long* ctl, WfState& st) {
  char* p = (char*)mem;
  auto take = [&](size_t words) {
    char* r = p;
    p += words * 4 * (size_t)n;
    return r;
  };
  st.seed = (uint32_t*)take(1);
  st.k = (uint32_t*)take(1);
  st.dp = (uint32_t*)take(1);
  st.col = (float*)take(3);
  st.pc = (float*)take(3);
  st.ro = (float*)take(3);
  st.rd = (float*)take(3);
  st.qprim = (uint32_t*)take(1);
  st.qt = (float*)take(1);
  st.res_i = (uint32_t*)take(1);
  st.res_t = (float*)take(1);
  st.ctl = ctl;
  st.n = n;
  return hipSuccess;
}

hipError_t launch_wf_init(const DevFrame& fr, const wgt_tile* tiles, const WfState& st, uchar4* out8,
                          float4* out32, uint32_t* outhit, hipStream_t stream) {
  const dim3 grid((st.n + kWfShadeBlock - 1) / kWfShadeBlock), block(kWfShadeBlock);
  k_wf_init<<<grid, block, 0, stream>>>(fr, tiles, st, out8, out32, outhit);
  return hipGetLastError();
}

hipError_t launch_wf_shade(const DevScene& sc, const DevFrame& fr, const wgt_tile* tiles,
                           const WfState& st, uchar4* out8, float4* out32, uint32_t* outhit,
                           unsigned long long* counters, hipStream_t stream) {
  const dim3 grid((st.n + kWfShadeBlock - 1) / kWfShadeBlock), block(kWfShadeBlock);
  if (counters) k_wf_shade<true><<<grid, block, 0, stream>>>(sc, fr, tiles, st, out8, out32, outhit, counters);
  else k_wf_shade<false><<<grid, block, 0, stream>>>(sc, fr, tiles, st, out8, out32, outhit, nullptr);
  return hipGetLastError();
}

hipError_t launch_wf_trace(const DevScene& sc, const DevFrame& fr, const WfState& st,
                           unsigned long long* counters, hipStream_t stream) {
  if (fr.wf_chunk == 0 || fr.wf_chunk > (uint32_t)kWfChunkMax || fr.wf_chunk % kBlock != 0)
    return hipErrorInvalidValue;
  const dim3 grid((st.n + fr.wf_chunk - 1) / fr.wf_chunk), block(kBlock);
  if (counters) k_wf_trace<true><<<grid, block, stack_lds_bytes(sc), stream>>>(sc, fr, st, counters);
  else k_wf_trace<false><<<grid, block, stack_lds_bytes(sc), stream>>>(sc, fr, st, nullptr);
  return hipGetLastError();
}

}  // namespace wgt
