// wgt_kernels.hip — the MI355X (gfx950) path-tracing kernels.
//
// One lane per pixel, one wave (64 lanes = 8x8 pixels) per block.  Each lane runs
// its pixel's whole compute_sample (path_tracer.wgsl:374-398); the per-pixel RNG
// stream is serial across samples (path_tracer.wgsl:378, 381-395), so there is no
// sample-level parallelism — parallelism is over pixels only.
//
// sample_hit (path_tracer.wgsl:290-310) = linear scan of lights and quads (scalar
// loads: the scene is wave-uniform), BVH4 traversal over triangles (per-lane LDS
// stack of 4-byte entries, or 3-byte ones in k_render_ps at 6 waves per SIMD;
// Moller-Trumbore in fp32, wgt_geom.h), then the sphere scan.
//
// Two kernels compute bit-identical results:
//  * k_render (simple, WGT_KERNEL=1): a flat per-lane loop, one closest-hit query +
//    one shading step per iteration.
//  * k_render_ps (persistent, the default): the wave alternates a
//    SERVICE phase (finalise the hit of lanes whose traversal ended, shade, start
//    the next ray: camera ray or bounce, quad scan, root-node test) and a
//    TRAVERSAL phase (one BVH node or leaf per lane per step).  A phase ends when
//    too few lanes are left for it (wave-uniform ballot counts), so lanes whose
//    ray left the BVH early pick up new rays while the long traversals continue:
//    the traversal loop runs at 10 % SIMT utilisation in k_render on the bunny
//    stand-in (profiles/r01_*), which this structure removes.
//    Without triangles (TRIS = false, the Cornell box) there is no traversal phase:
//    the persistent pixel queue alone balances the pixels.
//
// NaN rays (any NaN in start/dir) are resolved without tracing: every rejection
// test of the reference is false for NaN, so the last primitive of the scan — the
// last sphere — wins.  When that sphere is not emissive the path can only
// continue NaN-absorbed to depth 50 with exactly 3 rand() per bounce and a NaN
// colour (contributing max(NaN, 0) = 0), so the LCG is advanced by 3*(50-depth)
// steps in O(8) and the sample ends: bit-identical output, ~2/3 fewer queries on
// the Cornell box.
#include <type_traits>

#include "wgt_device.h"

namespace wgt {

template <bool TRIS, bool STATS>
__global__ void __launch_bounds__(kBlock)
k_render(DevScene sc, DevFrame fr, const wgt_tile* __restrict__ tiles, uchar4* __restrict__ out8,
         float4* __restrict__ out32, uint32_t* __restrict__ outhit,
         unsigned long long* __restrict__ counters) {
  extern __shared__ int s_stack[];  // sc.stack entries per lane (stack_lds_bytes)
  uint32_t po;
  Pixel px;
  if (!pixel_setup(fr, tiles, po, px)) return;
  int* lds = s_stack + threadIdx.x;
  const Light L{xyz(sc.quads[0]), xyz(sc.quads[1]), xyz(sc.quads[2])};
  const uint32_t nsamp = fr.sqrt_spp * fr.sqrt_spp;
  f3 ro{}, rd{}, pc{};
  int depth = 0;
  TravStats st{};
  Counters c{0u, 0u, 0u, 0u, 0u, 0u, 1u};  // one pixel per lane

  while (!px_done(fr, px)) {
    if (STATS) simt_count(c.lw, c.ll);
    if (depth == 0) {
      camera_ray(fr, px, ro, rd);
      pc = f3{1.0f, 1.0f, 1.0f};
    }
    const bool nanray = has_nan(ro) || has_nan(rd);
    if (nanray && !sc.last_sphere_emissive) {
      first_hit(px, depth, last_prim(sc), po, outhit);
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
    first_hit(px, depth, h.prim, po, outhit);
    const bool end = shade(sc, L, h, depth, px.seed, ro, rd, pc);
    ++depth;
    if (end || depth == kRayDepth) {
      end_sample(fr, px, pc);
      depth = 0;
    }
  }
  write_pixel(fr, po, px, out8, out32, outhit);
  if (STATS) flush_counters(counters, c, st, nsamp);
}

// Phase-split kernel for scenes with triangles (see the file comment), persistent:
// the grid is the resident wave capacity and lanes take pixels from the launch's
// pixel queue (*queue counts handed-out pixel slots of 64 * blocks).  A lane
// whose pixel has finished all its samples writes it and takes the next slot, so
// no lane idles while its wave has work left and the launch has no tail of
// late-started expensive tiles.  Queue block q is pixel block fr.perm[q] (LPT
// order: most expensive first, from a COST pre-pass; see launch_render), so the
// pixels still in flight when the queue drains are cheap ones; a wave's first 64
// slots are one 8x8 pixel block.  Each pixel's result depends only on its
// coordinates and seed: which lane or wave computes it does not change a bit.
// COST: the 1-spp pre-pass: no output, each finished pixel adds its work units
// (fr.pq_svc_cost per ray started + 1 per traversal step) to fr.cost[its block];
// it renders every pixel of each 8x8 block (fr.pq_lpt_all) or the 16 at even (x, y).
// STATS: wave cycles per service-phase region (s_memtime; the regions run in
// divergent code, so each adds the wave's time spent issuing or waiting in it).
#define WGT_REGION(acc, ...)                                  \
  do {                                                        \
    const uint64_t r0_ = STATS ? __builtin_amdgcn_s_memtime() : 0; \
    __VA_ARGS__;                                              \
    if (STATS) acc += __builtin_amdgcn_s_memtime() - r0_;     \
  } while (0)

// PK (DevScene::ps_park): the lanes' traversal state is parked in
// LDS words (Park) while the wave runs a service pass, and the LDS holds sc.ps_cap stack
// entries per lane with the rest on a per-lane global stack (park_fix): the service code
// then holds no traversal registers, which it used to spill to scratch.
template <bool STATS, bool COST, int CN, int W, bool TRIS = true, bool PK = false>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(W)))
k_render_ps(DevScene sc, DevFrame fr, const wgt_tile* __restrict__ tiles, uchar4* __restrict__ out8,
            float4* __restrict__ out32, uint32_t* __restrict__ outhit,
            unsigned long long* __restrict__ counters, uint32_t* __restrict__ queue,
            int* __restrict__ spill) {
  // spill: the global stacks (PK, DevFrame::ps_spill), a kernel argument of its own: a
  // noalias pointer, so its stores do not clobber the scene for the compiler, whose
  // wave-uniform loads (quads, spheres, the root node) stay scalar loads
  extern __shared__ int s_stack[];  // stack entries per lane (+ parked words), ps_stack_lds_bytes
  // 6 waves per SIMD: 3-byte entries (DevScene::ps_waves guarantees the refs fit)
  using STK = typename std::conditional<W >= 6, Stack24, Stack32>::type;
  const uint32_t cap = PK ? sc.ps_cap : sc.stack;  // LDS stack entries per lane
  // PK: the highest stack top a node step may start from, cap - 4 (3 pushes and a parked
  // leaf above it); no bound when the LDS holds the builder's whole stack (cap = sc.stack),
  // which no traversal exceeds (and then no global stack exists, DevFrame::ps_spill)
  const uint32_t top_max = PK && cap < sc.stack ? cap - 4u : 0xffffffffu;
  STK lds;
  Park P;
  if constexpr (W >= 6) {
    lds.lo = (uint16_t*)s_stack + threadIdx.x;
    lds.hi = (int8_t*)((uint16_t*)s_stack + cap * kBlock) + threadIdx.x;
    P.p = (uint32_t*)((char*)s_stack + cap * kBlock * 3) + threadIdx.x;
  } else {
    lds.p = s_stack + threadIdx.x;
    P.p = (uint32_t*)(s_stack + cap * kBlock) + threadIdx.x;
  }
  const uint32_t lane = threadIdx.x;
  const Light L{xyz(sc.quads[0]), xyz(sc.quads[1]), xyz(sc.quads[2])};
  const uint32_t nsamp = fr.sqrt_spp * fr.sqrt_spp;
  const uint32_t n_slots = fr.n_slots;
  Pixel px{};
  uint32_t po = 0;  // output offset of the lane's pixel
  f3 ro{}, rd{}, pc{};
  // the path depth and the pending hit's quad (quad_scan_fast; kNoHit + 1 = 0 for none), one
  // register: depth | (q_prim + 1) << 6 (depth <= kRayDepth < 64, quads < 2^26 at upload)
  uint32_t dq = 0;
  TravStats st{};
  Counters c{0u, 0u, 0u, 0u, 0u, 0u, 0u};
  // invariant: trav == !trav_done(t) (a lane leaves the traversal exactly when
  // trav_done turns true), so a lane with a node to visit or a pending leaf is
  // traversing; a lane starts done.  PK: t lives in registers only in the traversal
  // phase (and while a service pass starts a ray); Park holds it otherwise
  Trav t;
  t.ref = kNoRef;
  t.lf = t.le = 0u;
  t.sp = 0;
  if (PK) {
    t.inv = t.ot = f3{0.0f, 0.0f, 0.0f};
    t.bt = 0.0f;
    t.bi = kNoHit;
    park_put(P, t);
    P.st(9, 0u);
  }
  float q_t = kRayMax;
  bool have = false;       // lane holds a pixel
  bool exhausted = false;  // the queue is empty for this lane
  bool trav = false, pending = false, fin = false;
  bool nanray = false;  // the pending hit is a NaN ray's (emissive last sphere), resolved at finalise
  uint64_t cyc_svc = 0, cyc_trav = 0;
  uint64_t cr_refill = 0, cr_fin = 0, cr_shade = 0, cr_cam = 0, cr_quads = 0, cr_root = 0;
  // STATS: traversal steps by BVH level (CNT_TOP_NODES .. CNT_CYC_TRI_STEPS)
  uint64_t cs_node = 0, cs_top = 0, cs_tri = 0;
  uint32_t top_visits = 0;
  uint32_t pblock = 0, work = 0;  // COST: the pixel's block and its work so far

  for (;;) {
    // ------------------------------------------------------------ service phase
    uint64_t t_phase = STATS ? __builtin_amdgcn_s_memtime() : 0;
    for (;;) {
      const uint64_t tr0 = STATS ? __builtin_amdgcn_s_memtime() : 0;
      if (fin) {  // a finished pixel: write it (here, outside the sample loop)
        if (COST) {
          atomicAdd(fr.cost + pblock, work);
          work = 0;
        } else {
          write_pixel(fr, po, px, out8, out32, outhit);
        }
        if (STATS) ++c.px;
        fin = false;
      }
      // refill: lanes without a pixel take consecutive slots, one atomic per wave
      const unsigned long long idle = __ballot(!have && !exhausted);
      if (idle != 0ull) {
        const uint32_t n_idle = (uint32_t)__popcll(idle);
        if (n_idle >= fr.pq_refill || __ballot(have) == 0ull) {
          const int leader = __ffsll((long long)idle) - 1;
          uint32_t base = 0;
          if ((int)lane == leader) base = atomicAdd(queue, n_idle);
          base = __builtin_amdgcn_readlane(base, leader);  // leader is wave-uniform: no lane index, no LDS
          if (!have && !exhausted) {
            // the lane's rank among the idle lanes (mbcnt: the set bits of idle below this lane)
            const uint32_t slot = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
            if (slot >= n_slots) {
              exhausted = true;
            } else {
              // COST pre-pass: 16 slots per block, the pixels at even (x, y) of the 8x8 block
              const bool quarter = COST && !fr.pq_lpt_all;
              const uint32_t sb = quarter ? (slot >> 4) : (slot >> 6);
              const uint32_t sl = quarter ? (((slot & 3u) << 1) | (((slot >> 2) & 3u) << 4)) : (slot & 63u);
              const uint32_t b = fr.perm ? fr.perm[sb] : sb;
              if (slot_setup(fr, tiles, b, sl, po, px)) {
                have = true;
                dq = 0u;
                pblock = b;
              }
            }
          }
        }
      }
      if (STATS) cr_refill += __builtin_amdgcn_s_memtime() - tr0;
      const bool need = have && !trav;
      if (!__any(need)) {
        if (__ballot(!have && !exhausted) != 0ull && __ballot(trav) == 0ull) continue;  // refill again
        break;
      }
      if (need) {
        if (STATS) simt_count(c.lw, c.ll);
        // PK: a lane whose traversal stopped on its LDS stack (not finished) moves stack
        // entries to or from its global stack and traverses on
        bool resume = false;
        if (PK && TRIS && pending && !nanray) {
          resume = (int)P.ld(8) != kNoRef || (P.ld(10) & kParkLeafMask) != 0u || P.ld(9) != 0u;
          if (resume) {
            // the lane's global stack: entry e at gs[e * fr.ps_spill_stride]
            const uint32_t k = park_fix(sc, P, lds, cap, spill + blockIdx.x * kBlock + lane, fr.ps_spill_stride);
            if (STATS) {
              st.spills += k == 1u ? 1u : 0u;
              st.refills += k == 2u ? 1u : 0u;
              st.overflows += k == 3u ? 1u : 0u;
            }
            pending = false;
            trav = true;
          }
        }
        if (pending) {
          // finalise: rebuild the quad hit, merge triangles, scan spheres, shade
          Hit h;
          if (nanray) {
            nan_hit(sc, ro, rd, h);
            if (STATS) { ++c.q; ++c.nan; }
            nanray = false;
          } else {
            // the traversal's result (PK: parked)
            const float bt = PK ? __uint_as_float(P.ld(6)) : t.bt;
            const uint32_t bi = PK ? P.ld(7) : t.bi;
            // no triangles (TRIS = false): no shading record exists to preload
            WGT_REGION(cr_fin, float4 pre[2]; if (TRIS) preload_tshade(sc, bi, pre[0], pre[1]);
                       quad_rebuild(sc, ro, rd, (dq >> 6) - 1u, q_t, h); finish_hit(sc, ro, rd, bt, bi, h, TRIS ? pre : nullptr));
            if (STATS) { ++c.q; ++c.tr; }
          }
          first_hit(px, (int)(dq & 63u), h.prim, po, outhit);
          const uint64_t ts0 = STATS ? __builtin_amdgcn_s_memtime() : 0;
          const bool end = shade(sc, L, h, (int)(dq & 63u), px.seed, ro, rd, pc);
          dq = (dq & 63u) + 1u;  // the quad is used: q_prim + 1 = 0
          // COST: the pre-pass's paths may end early (DevFrame::pq_depth): a cost estimate
          if (end || dq == (COST ? fr.pq_depth : (uint32_t)kRayDepth)) {
            end_sample(fr, px, pc);
            dq = 0u;
          }
          if (STATS) cr_shade += __builtin_amdgcn_s_memtime() - ts0;
          pending = false;
        }
        // start the next ray of this pixel
        if (!resume) for (;;) {
          if (px_done(fr, px)) {
            have = false;
            fin = true;
            break;
          }
          if ((dq & 63u) == 0u) {
            WGT_REGION(cr_cam, camera_ray(fr, px, ro, rd));
            pc = f3{1.0f, 1.0f, 1.0f};
          }
          if (has_nan(ro) || has_nan(rd)) {
            if (!sc.last_sphere_emissive) {
              first_hit(px, (int)(dq & 63u), last_prim(sc), po, outhit);
              skip_nan_path<STATS>(sc, fr, px, (int)(dq & 63u), c);
              dq = 0u;
              continue;
            }
            // emissive last sphere: the NaN ray's hit (the last sphere, no traversal)
            // is resolved and shaded at the next finalise, the one shading site
            nanray = true;
            pending = true;
            break;
          }
          uint32_t q_prim;
          WGT_REGION(cr_quads, const bool qx = quad_scan_fast(sc, ro, rd, q_prim, q_t);
                     if (STATS && !qx) ++c.qref; trav_init<CN>(sc, ro, rd, q_prim != kNoHit, q_t, t));
          dq = (dq & 63u) | (q_prim + 1u) << 6;
          if (COST) work += fr.pq_svc_cost;
          // the root node is tested here: rays that miss every root child never
          // enter the traversal phase
          if (TRIS) {
            WGT_REGION(cr_root, root_step<STATS, CN>(sc, t, lds, st));
            if (PK) {
              park_put(P, t);
              P.st(9, (uint32_t)t.sp);  // a new ray's global stack is empty
            }
            // (PK: a root step pushes at most 4 entries, and the LDS stack holds >= kMinPsCap
            // = 8, so the ray starts its traversal with a top <= top_max)
            if (trav_done(t)) pending = true;
            else trav = true;
          } else {
            pending = true;  // no triangles: the quad and sphere scans are the whole query
          }
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
    if (__ballot(have || !exhausted) == 0ull) break;
    // --------------------------------------------------------- traversal phase
    uint32_t to_service = fr.ps_to_service;
    if (fr.ps_svc_frac) {
      const uint32_t live = (uint32_t)__popcll(__ballot(have));
      const uint32_t sparse = (live * fr.ps_svc_frac) >> 6;
      to_service = sparse < to_service ? sparse : to_service;
    }
    // PK: every lane takes its state from Park; a lane that is not traversing holds a
    // finished one (a lane parked on its LDS bound is served before the next traversal
    // phase: the first iteration of a service phase serves every lane that needs it)
    if (PK && TRIS) park_get(P, t);
    // 1/d and the slab offsets -o / d are recomputed here from the ray (trav_init's operations:
    // bit-identical), so that they are dead through the service phase: six fewer registers where
    // its pressure spilled (scratch 52 -> 20 B/lane, sponza +4.4 %)
    if (!PK && TRIS) {
      const f3 inv = f3{safe_inv_short(rd.x), safe_inv_short(rd.y), safe_inv_short(rd.z)};
      t.ot = slab_offset(ro, inv);
      t.inv = CN ? sc.cstep * inv : inv;
    }
    bool parked = false;  // PK: the lane left on its LDS stack bound, its state parked as it was
    for (; TRIS;) {
      // one uniform mode per step: triangle steps once enough lanes hold a
      // pending leaf (weighted by the two steps' costs), else node steps
      const bool can_node = t.ref != kNoRef;  // implies trav (invariant above)
      const bool can_tri = t.lf < t.le;  // implies trav
      const uint32_t nn = (uint32_t)__popcll(__ballot(can_node));
      const uint32_t nl = (uint32_t)__popcll(__ballot(can_tri));
      const bool tri_mode = nn == 0 || nl * 100u >= nn * fr.tri_ratio;
      if (STATS && (tri_mode ? can_tri : can_node)) simt_count(st.wave_steps, st.lane_steps);
      if (COST && (tri_mode ? can_tri : can_node)) ++work;
      const uint64_t ts0 = STATS ? __builtin_amdgcn_s_memtime() : 0;
      bool all_top = false;  // STATS: every lane visiting a node this step is at level 1 or 2
      if (STATS && !tri_mode) {
        const bool top = can_node && sc.node_level[(uint32_t)t.ref / (CN ? kCRecordFloat4s * 16u : kNode4Floats * 4u)] <= 2u;
        top_visits += top ? 1u : 0u;
        all_top = __ballot(can_node && !top) == 0ull;
      }
      if (tri_mode) {
        if (can_tri) tri_step<STATS, CN>(sc, ro, rd, t, lds, st);
      } else {
        if (can_node) {
          node_step<STATS, CN>(sc, t, lds, st);
          // PK: fewer than 4 free LDS entries above the top (only node steps push): the
          // lane parks its state and leaves as if done; its service pass spills (park_fix)
          if (PK && (uint32_t)t.sp > top_max) {
            park_put(P, t);
            parked = true;
            t.ref = kNoRef;
            t.lf = t.le;
            t.sp = 0;
          }
        }
      }
      if (STATS) {
        const uint64_t dt = __builtin_amdgcn_s_memtime() - ts0;
        if (tri_mode) cs_tri += dt;
        else {
          cs_node += dt;
          cs_top += all_top ? dt : 0u;
        }
      }
      if (trav && trav_done(t)) {
        trav = false;
        pending = true;
      }
      const uint32_t ntrav = (uint32_t)__popcll(__ballot(trav));
      if (ntrav == 0) break;
      if (ntrav <= to_service && __any(!trav && (have || !exhausted))) break;
    }
    if (PK && TRIS && !parked) park_put(P, t);
    if (STATS) cyc_trav += __builtin_amdgcn_s_memtime() - t_phase;
  }
  if (STATS) {
    flush_counters(counters, c, st, nsamp);
    if (lane == 0) {
      atomicAdd(&counters[CNT_CYC_SERVICE], (unsigned long long)cyc_svc);
      atomicAdd(&counters[CNT_CYC_TRAV], (unsigned long long)cyc_trav);
      atomicAdd(&counters[CNT_CYC_REFILL], (unsigned long long)cr_refill);
      atomicAdd(&counters[CNT_CYC_FINALISE], (unsigned long long)cr_fin);
      atomicAdd(&counters[CNT_CYC_SHADE], (unsigned long long)cr_shade);
      atomicAdd(&counters[CNT_CYC_CAMERA], (unsigned long long)cr_cam);
      atomicAdd(&counters[CNT_CYC_QUADS], (unsigned long long)cr_quads);
      atomicAdd(&counters[CNT_CYC_ROOT], (unsigned long long)cr_root);
      atomicAdd(&counters[CNT_CYC_NODE_STEPS], (unsigned long long)cs_node);
      atomicAdd(&counters[CNT_CYC_TOP_STEPS], (unsigned long long)cs_top);
      atomicAdd(&counters[CNT_CYC_TRI_STEPS], (unsigned long long)cs_tri);
    }
    atomicAdd(&counters[CNT_TOP_NODES], (unsigned long long)top_visits);
  }
}

template <bool TRIS>
__global__ void __launch_bounds__(kBlock)
k_trace(DevScene sc, const float* __restrict__ rays, uint32_t n, uint32_t* __restrict__ prim,
        float* __restrict__ dist) {
  extern __shared__ int s_stack[];  // sc.stack entries per lane (stack_lds_bytes)
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const f3 o = f3{rays[i], rays[(size_t)n + i], rays[2 * (size_t)n + i]};
  const f3 d = f3{rays[3 * (size_t)n + i], rays[4 * (size_t)n + i], rays[5 * (size_t)n + i]};
  Hit h;
  TravStats st{};
  sample_hit<TRIS, false, true>(sc, o, d, s_stack + threadIdx.x, h, st);  // any caller ray: IEEE t
  prim[i] = h.prim;
  dist[i] = h.dist;
}

// LPT order of the pixel blocks from the pre-pass costs, one workgroup: bucket
// by the float bits of the cost (exponent + 3 mantissa bits: 8 buckets per
// octave), most expensive bucket first (order within a bucket is arbitrary: the
// order only shapes the schedule, never a pixel's result).  It also leaves the launch's
// scheduling words as the next launch on the same workspace needs them (launch_render): the
// costs it has read zeroed, and both queue counters zeroed (the pre-pass's is done; the main
// kernel's starts after this kernel), so that no memset kernel runs per frame.  256 threads: a
// workgroup that finds room on a CU while the previous frame's persistent grid drains (1,024
// threads needed 16 free wave slots on one CU).
constexpr int kLptThreads = 256, kLptBuckets = 1280;  // float bits >> 20 of any u32 cost
__device__ __forceinline__ uint32_t lpt_bucket(uint32_t c) { return __float_as_uint((float)c) >> 20; }
__global__ void __launch_bounds__(kLptThreads)
k_lpt_order(uint32_t* __restrict__ cost, uint32_t blocks, uint32_t* __restrict__ perm, uint32_t* __restrict__ queues) {
  __shared__ uint32_t s_cnt[kLptBuckets];
  for (int b = threadIdx.x; b < kLptBuckets; b += kLptThreads) s_cnt[b] = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < blocks; i += kLptThreads) atomicAdd(&s_cnt[lpt_bucket(cost[i])], 1u);
  __syncthreads();
  if (threadIdx.x == 0) {  // exclusive scan from the most expensive bucket down
    uint32_t run = 0;
    for (int b = kLptBuckets - 1; b >= 0; --b) {
      const uint32_t n = s_cnt[b];
      s_cnt[b] = run;
      run += n;
    }
    queues[0] = 0u;  // the pre-pass's queue (finished)
    queues[1] = 0u;  // the main kernel's queue (next in stream order)
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < blocks; i += kLptThreads) {
    const uint32_t c = cost[i];
    cost[i] = 0u;
    perm[atomicAdd(&s_cnt[lpt_bucket(c)], 1u)] = i;
  }
}

// wgt_selftest_math: the kernels' sqrt / division forms (wgt_math.h) against
// correctly rounded results: the f64 operation rounded to f32, exact for sqrt and
// division because f64 has more than 2*24 + 2 bits (double rounding is innocuous).
//   sqrt_rn   on all 2^32 bit patterns;
//   sqrt_fast on every pattern of its domain (all but 0 < x < 2^-96 and negative
//             denormals);
//   div_rn    on n pseudo-random (numerator, denominator) pairs from the quad plane
//             distance's range under the render limits: |n| <= 2^44 of any exponent
//             (zeros and denormals included), 2^-10 <= |d| < 2^35 (|d| >= kRayMin is
//             tested before the division): the accept decision t in [kRayMin,
//             kRayMax] must equal the IEEE one, and an accepted t its bits; and
//             the reciprocal 1 / det of Moller-Trumbore (mt_test<true>) for 2^-40 <=
//             |det| < 2^95 (the render limits' range past the 1e-12 rejection): its bits;
//   the short reciprocal of the traversal's 1/d (trav_init, render rays: safe_inv_short) on every
//             bit pattern with 1e-30 <= |x| <= 2^34;
//   the compiler's own lowerings (__builtin_sqrtf, n / d) on the same inputs.
// NaN equals NaN.  counts: [0] sqrt tests, [1] sqrt_rn bad, [2] div tests, [3]
// div_rn bad, [4] sqrt_fast tests, [5] sqrt_fast bad, [6] compiler sqrt bad, [7]
// compiler div bad.
__device__ __forceinline__ uint32_t st_hash(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
// sign and mantissa from h, biased exponent field uniform in [fmin, fmax]
__device__ __forceinline__ float st_float(uint32_t h, uint32_t fmin, uint32_t fmax) {
  const uint32_t e = fmin + (h >> 9) % (fmax - fmin + 1u);
  return __uint_as_float((h & 0x80000000u) | (e << 23) | (st_hash(h) & 0x7fffffu));
}
__device__ __forceinline__ bool st_same(float a, float b) {
  return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
}
__device__ __forceinline__ bool st_accept(float t) { return !(t < kRayMin || kRayMax < t); }
__global__ void __launch_bounds__(256) k_selftest_math(uint32_t n, uint32_t seed, unsigned long long* counts) {
  uint32_t bad_s = 0, bad_f = 0, n_f = 0, bad_d = 0, bad_sc = 0, bad_dc = 0;
  uint32_t bad_r = 0;  // the traversal reciprocal's failures
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32); i += stride) {
    const uint32_t bits = (uint32_t)i;
    const float x = __uint_as_float(bits);
    const float ref = (float)__builtin_sqrt((double)x);
    bad_s += st_same(sqrt_rn(x), ref) ? 0u : 1u;
    bad_sc += st_same(__builtin_sqrtf(x), ref) ? 0u : 1u;
    const uint32_t mag = bits & 0x7fffffffu;
    const bool fast_domain = mag == 0u || mag >= 0x0f800000u || (bits >> 31 && mag >= 0x00800000u);
    if (fast_domain) {
      ++n_f;
      bad_f += st_same(sqrt_fast(x), ref) ? 0u : 1u;
    }
    if (mag >= __float_as_uint(1e-30f) && mag <= __float_as_uint(0x1p34f))
      bad_r += st_same(safe_inv_short(x), (float)(1.0 / (double)x)) ? 0u : 1u;
  }
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint32_t)stride) {
    const uint32_t h = st_hash(seed * 0x9e3779b9u + i), h2 = st_hash(h ^ 0x5bd1e995u);
    const float nn = st_float(h, 0u, 127u + 44u);             // |n| <= 2^45 (zeros, denormals)
    const float dd = st_float(h2, 127u - 10u, 127u + 34u);    // 2^-10 <= |d| < 2^35 (bound 2*sqrt(3)*2^32)
    const float ref = (float)((double)nn / (double)dd);
    const float q = div_rn(nn, dd);
    const bool acc = st_accept(ref);
    bad_d += (acc != st_accept(q) || (acc && !st_same(q, ref))) ? 1u : 0u;
    bad_dc += st_same(nn / dd, ref) ? 0u : 1u;
    // Moller-Trumbore's 1/det (mt_test<true>): every det the render limits admit past
    // the |det| >= 1e-12 rejection, 2^-40 <= |det| < 2^95, must give the IEEE bits
    const float det = st_float(st_hash(h2 ^ 0x2545f491u), 127u - 40u, 127u + 94u);
    const float rref = (float)(1.0 / (double)det);
    bad_d += st_same(div_rn(1.0f, det), rref) ? 0u : 1u;
    bad_dc += st_same(1.0f / det, rref) ? 0u : 1u;
  }
  bad_d += bad_r;
  atomicAdd(&counts[1], (unsigned long long)bad_s);
  atomicAdd(&counts[3], (unsigned long long)bad_d);
  atomicAdd(&counts[4], (unsigned long long)n_f);
  atomicAdd(&counts[5], (unsigned long long)bad_f);
  atomicAdd(&counts[6], (unsigned long long)bad_sc);
  atomicAdd(&counts[7], (unsigned long long)bad_dc);
}

hipError_t launch_selftest_math(uint32_t n, uint32_t seed, unsigned long long* d_counts, hipStream_t stream) {
  k_selftest_math<<<2048, 256, 0, stream>>>(n, seed, d_counts);
  return hipGetLastError();
}

// k_render_ps at the scene's waves per SIMD (6 with 3-byte stack entries, else 5), the frame's node
// form (node_form: 0 = 128-B nodes, 1 = 80-B compact records) and the scene's traversal state (parked
// in LDS during service passes, or not: DevScene::ps_park).  Scenes without triangles run the
// traversal-free instantiation.
template <bool STATS, bool COST, int CN, int W>
void ps_launch_w(const DevScene& sc, dim3 grid, dim3 block, size_t lds, hipStream_t stream, const DevFrame& f,
                 const wgt_tile* tiles, uchar4* out8, float4* out32, uint32_t* outhit, unsigned long long* counters,
                 uint32_t* queue) {
  if (sc.ps_park)
    k_render_ps<STATS, COST, CN, W, true, true><<<grid, block, lds, stream>>>(sc, f, tiles, out8, out32, outhit, counters, queue, f.ps_spill);
  else
    k_render_ps<STATS, COST, CN, W, true, false><<<grid, block, lds, stream>>>(sc, f, tiles, out8, out32, outhit, counters, queue, f.ps_spill);
}
template <bool STATS, bool COST>
void ps_launch(const DevScene& sc, int cn, dim3 grid, dim3 block, size_t lds, hipStream_t stream, const DevFrame& f,
               const wgt_tile* tiles, uchar4* out8, float4* out32, uint32_t* outhit, unsigned long long* counters,
               uint32_t* queue) {
  if (sc.n_tris == 0) {
    k_render_ps<STATS, COST, 0, kPsWavesNoTris, false><<<grid, block, lds, stream>>>(sc, f, tiles, out8, out32, outhit, counters, queue, f.ps_spill);
  } else if (sc.ps_waves == 6) {
    if (cn) ps_launch_w<STATS, COST, 1, 6>(sc, grid, block, lds, stream, f, tiles, out8, out32, outhit, counters, queue);
    else ps_launch_w<STATS, COST, 0, 6>(sc, grid, block, lds, stream, f, tiles, out8, out32, outhit, counters, queue);
  } else {
    if (cn) ps_launch_w<STATS, COST, 1, 5>(sc, grid, block, lds, stream, f, tiles, out8, out32, outhit, counters, queue);
    else ps_launch_w<STATS, COST, 0, 5>(sc, grid, block, lds, stream, f, tiles, out8, out32, outhit, counters, queue);
  }
}

// The compact codes are exact for ray origins within their bound (the margin, wgt_geom.h):
// hit points always are, the camera is checked per frame (beyond: the 128-B nodes).
// WGT_CNODE: 0 = 128-B, 1 = 80-B (default), 2 = 80-B when the 128-B tree would not fit one XCD's
// 4 MB L2 (sponza stand-in: 7.3 MB -> 4.6 MB; the default until round 6, when the compact step's
// integer bound minimum made the 80-B records faster on the bunny's L2-resident tree too, +0.6 %,
// DESIGN.md §4.2 item 30).  (Round 6 removed the 64-B records, WGT_CNODE=3, and the wide 8-slot
// records, WGT_CNODE=4: slower on every measured scene)
int node_form(const DevScene& sc, const DevFrame& fr) {
  const float cam = fmaxf(fmaxf(fabsf(fr.ox), fabsf(fr.oy)), fabsf(fr.oz));
  if (!(cam <= sc.cbound)) return 0;
  return fr.cnode == 1 || (fr.cnode >= 2 && (size_t)sc.n_nodes * kNode4Floats * 4 > kCompactNodeBytes) ? 1 : 0;
}

// the parked kernel's global stacks: sc.stack entries per lane of every resident wave
// (only when the LDS holds fewer, sc.ps_cap < sc.stack)
size_t ps_spill_bytes(const DevScene& sc, uint32_t resident) {
  if (!sc.ps_park || sc.n_tris == 0 || sc.ps_cap >= sc.stack) return 0;
  return (size_t)resident * kBlock * sc.stack * sizeof(int);
}

size_t render_ws_bytes(const DevScene& sc, const DevFrame& fr, uint32_t resident) {
  const uint64_t bx = (fr.tw + 7u) / 8u, by = (fr.th + 7u) / 8u;
  return ((256 + 8 * bx * by * fr.n_tiles + 255) & ~(uint64_t)255) + ps_spill_bytes(sc, resident);
}

hipError_t launch_render(const DevScene& sc, const DevFrame& fr, const wgt_tile* d_tiles,
                         uchar4* out8, float4* out32, uint32_t* outhit,
                         unsigned long long* counters, uint32_t resident, void* ws, size_t ws_cap,
                         hipStream_t stream, uint32_t& ws_clean_nb) {
  const uint32_t bx = (fr.tw + 7u) / 8u, by = (fr.th + 7u) / 8u;
  const uint64_t blocks = (uint64_t)bx * by * fr.n_tiles;
  if (blocks == 0) return hipSuccess;
  if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
  DevFrame fm = fr;  // + slot_setup's division multipliers
  fm.div_bx = 0xffffffffu / bx;
  fm.div_bpt = 0xffffffffu / (bx * by);
  const dim3 block(kBlock);
  const size_t lds = stack_lds_bytes(sc);
  const bool tris = sc.n_tris > 0;
  if (fr.kernel == 2) {
    const size_t plds = ps_stack_lds_bytes(sc);
    if (blocks * 64ull > 0xffffffffull || resident == 0) return hipErrorInvalidValue;
    if (!ws || ws_cap < render_ws_bytes(sc, fr, resident)) return hipErrorInvalidValue;
    const uint32_t nb = (uint32_t)blocks;
    const dim3 grid(nb < resident ? nb : resident);
    // workspace (the context's, used in stream order): [0] pre-pass queue,
    // [1] queue | cost[nb] | perm[nb]
    const bool lpt = fr.pq_lpt && fr.sqrt_spp > fr.pq_lpt;
    const int cn = node_form(sc, fr);
    uint32_t* q = (uint32_t*)ws;
    DevFrame f = fm;
    // phase thresholds swept per wave budget (profiles/sweeps/r01_sweep_compact_knobs.jsonl)
    if (f.ps_to_trav == 0) f.ps_to_trav = sc.ps_waves >= 6 ? 16u : 18u;
    if (f.ps_to_service == 0) f.ps_to_service = sc.ps_waves >= 6 ? 14u : 16u;
    if (f.pq_refill == 0) f.pq_refill = 2u;
    f.n_slots = nb * 64u;
    f.perm = nullptr;
    f.cost = nullptr;
    // the global stacks follow the queue, costs and order (render_ws_bytes); the grid has at
    // most `resident` waves
    const uint64_t sched = (256 + 8ull * nb + 255) & ~255ull;
    f.ps_spill = ps_spill_bytes(sc, resident) ? (int*)((char*)ws + sched) : nullptr;
    f.ps_spill_stride = grid.x * kBlock;
    // the queues and costs start at zero: a memset, unless the previous LPT launch on this workspace
    // had the same block count and left them zero (k_lpt_order; ws_clean_nb = nb)
    hipError_t e = lpt && ws_clean_nb == nb ? hipSuccess : hipMemsetAsync(ws, 0, 256 + (lpt ? 4ull * nb : 0), stream);
    if (e == hipSuccess && lpt) {
      DevFrame fc = f;  // the pre-pass: fr.pq_lpt^2 samples per pixel
      fc.sqrt_spp = fr.pq_lpt < fr.sqrt_spp ? fr.pq_lpt : fr.sqrt_spp;
      fc.recip_sqrt_spp = 1.0f / (float)fc.sqrt_spp;
      fc.fspp = (float)(fc.sqrt_spp * fc.sqrt_spp);
      fc.inv_fspp = pow2_recip(fc.sqrt_spp * fc.sqrt_spp);
      fc.cost = (uint32_t*)((char*)ws + 256);
      fc.n_slots = nb * (fr.pq_lpt_all ? 64u : 16u);  // by default a quarter of each block's pixels estimate its cost
      ps_launch<false, true>(sc, cn, grid, block, plds, stream, fc, d_tiles, nullptr, nullptr, nullptr, nullptr, q);
      k_lpt_order<<<1, kLptThreads, 0, stream>>>(fc.cost, nb, fc.cost + nb, q);
      f.perm = fc.cost + nb;
      e = hipGetLastError();
    }
    if (e == hipSuccess) {
      if (counters) ps_launch<true, false>(sc, cn, grid, block, plds, stream, f, d_tiles, out8, out32, outhit, counters, q + 1);
      else ps_launch<false, false>(sc, cn, grid, block, plds, stream, f, d_tiles, out8, out32, outhit, nullptr, q + 1);
      e = hipGetLastError();
    }
    // after an LPT launch k_lpt_order has left the queues and nb costs zero for the next one
    ws_clean_nb = e == hipSuccess && lpt ? nb : 0u;
    return e;
  }
  const dim3 grid((uint32_t)blocks);
  if (counters) {
    if (tris) k_render<true, true><<<grid, block, lds, stream>>>(sc, fm, d_tiles, out8, out32, outhit, counters);
    else k_render<false, true><<<grid, block, lds, stream>>>(sc, fm, d_tiles, out8, out32, outhit, counters);
  } else {
    if (tris) k_render<true, false><<<grid, block, lds, stream>>>(sc, fm, d_tiles, out8, out32, outhit, nullptr);
    else k_render<false, false><<<grid, block, lds, stream>>>(sc, fm, d_tiles, out8, out32, outhit, nullptr);
  }
  return hipGetLastError();
}

// k_render_ps<STATS = false, COST = false, CN, W, true, PK> of a launchable form
template <int W, bool PK>
const void* ps_kernel(int cn) {
  return cn ? reinterpret_cast<const void*>(&k_render_ps<false, false, 1, W, true, PK>)
            : reinterpret_cast<const void*>(&k_render_ps<false, false, 0, W, true, PK>);
}

// The persistent grid: the smaller resident capacity of the two node forms the scene's launches can
// read (node_form), so that every wave of a launch is resident from its start.
hipError_t ps_resident_waves(const DevScene& sc, int device, uint32_t& waves) {
  int per_cu = 0, cus = 0;
  if (sc.n_tris == 0) {
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu, reinterpret_cast<const void*>(&k_render_ps<false, false, 0, kPsWavesNoTris, false>), kBlock,
        stack_lds_bytes(sc));
    if (e != hipSuccess) return e;
  } else {
    per_cu = 1 << 30;
    for (int cn = 0; cn < 2; ++cn) {
      const void* k = sc.ps_waves == 6 ? (sc.ps_park ? ps_kernel<6, true>(cn) : ps_kernel<6, false>(cn))
                                       : (sc.ps_park ? ps_kernel<5, true>(cn) : ps_kernel<5, false>(cn));
      int n = 0;
      const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, kBlock, ps_stack_lds_bytes(sc));
      if (e != hipSuccess) return e;
      per_cu = n < per_cu ? n : per_cu;
    }
  }
  const hipError_t e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  if (e != hipSuccess) return e;
  waves = (uint32_t)((per_cu > 0 ? per_cu : 1) * (cus > 0 ? cus : 1));
  return hipSuccess;
}

hipError_t launch_trace(const DevScene& sc, const float* d_rays, uint32_t n, uint32_t* prim,
                        float* dist, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const dim3 grid((n + kBlock - 1) / kBlock), block(kBlock);
  if (sc.n_tris > 0) k_trace<true><<<grid, block, stack_lds_bytes(sc), stream>>>(sc, d_rays, n, prim, dist);
  else k_trace<false><<<grid, block, stack_lds_bytes(sc), stream>>>(sc, d_rays, n, prim, dist);
  return hipGetLastError();
}

}  // namespace wgt
