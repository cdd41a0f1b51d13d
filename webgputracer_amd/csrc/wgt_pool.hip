// wgt_pool.hip — k_render_pool: the persistent phase-split kernel (k_render_ps,
// wgt_kernels.hip) with a RAY POOL shared by the 4 waves of a workgroup, so that a
// traversal step runs on the lanes of any wave's rays (cross-wave compaction).
//
// k_render_ps keeps every ray in the lane that owns its pixel: a wave's traversal
// phase runs with the lanes whose own ray is still in the BVH, and those lanes wait
// through the wave's service pass (finalise, shade, next ray: ~2,300 VALU) once too
// few are left.  Its traversal steps run at 43 % SIMT utilisation on the sponza
// stand-in.  Here a ray can move between the lanes of a workgroup:
//
//  * TICKETS.  Each wave owns `fr.pool_tickets` ray records (64 B in LDS: o, d, the
//    traversal state, the column of its stack).  A ray parked in a ticket is AVAIL
//    (a bit per ticket, one word per wave); a lane of ANY wave of the workgroup that
//    holds no ray claims it (LDS atomic AND), loads the record and traverses it.  The
//    ray's LDS stack stays where it is: column c of the workgroup's stacks belongs to
//    lane c's pixel, and whichever lane traverses the ray pushes and pops there.
//  * A wave LEAVES its traversal phase as k_render_ps does (few rays left, lanes of
//    its own waiting for service).  It first writes every ray it holds for another
//    lane back to that ray's ticket (AVAIL again), and parks its own unfinished rays
//    in free tickets of its own, so that other waves' lanes continue them during its
//    service pass instead of idling with them.
//  * A ray finished by a lane other than its owner leaves (bt, bi) in its ticket and
//    sets the ticket's DONE bit; the owner picks the result up at its next service
//    pass.  A ray finished by its owner lane (never parked) keeps the result in
//    registers, as in k_render_ps.
//
// Every pixel is still computed by its own lane from its own coordinates and seed,
// and the closest hit of a ray is a minimum over (t, index) of the triangles whose
// boxes it enters, whichever lanes run its steps: the output is bit-identical to
// k_render_ps and to the oracle (tests/test_gpu_parity.py).  Requires 3-byte stack
// entries (DevScene::ps_waves == 6: refs fit 24 bits, which the record packs).
#include "wgt_device.h"

namespace wgt {

constexpr int kPoolWaves = 4;
constexpr int kPoolBlock = kPoolWaves * kBlock;

struct PoolHdr {
  uint32_t avail[kPoolWaves];  // bit k of word w: ticket k of wave w holds a ray to traverse
  uint32_t done[kPoolWaves];   // bit k of word w: ticket k's ray has finished, (bt, bi) in it
};

// LDS layout at fixed offsets (constants in the ds instructions, no base registers):
// the workgroup's stacks for the largest bound (kStackMax + 1 = 32 entries of 3 B per
// column: an 8-bit array, then a 16-bit array), the header, then the tickets.
constexpr uint32_t kPoolStack = kStackMax + 1;
constexpr uint32_t kPoolHiOff = 0;
constexpr uint32_t kPoolLoOff = kPoolStack * kPoolBlock;
constexpr uint32_t kPoolHdrOff = kPoolLoOff + 2 * kPoolStack * kPoolBlock;  // 24,576
constexpr uint32_t kPoolRecOff = kPoolHdrOff + sizeof(PoolHdr);
// tickets per wave: as many as keep W workgroups per CU (6: 10 tickets; 5: 31)
template <int W>
constexpr uint32_t pool_tickets() {
  return ((160u * 1024u / (uint32_t)W - kPoolRecOff) / (kPoolWaves * 64u)) < 32u
             ? (160u * 1024u / (uint32_t)W - kPoolRecOff) / (kPoolWaves * 64u)
             : 32u;
}
template <int W>
constexpr size_t pool_lds_bytes() { return kPoolRecOff + (size_t)kPoolWaves * pool_tickets<W>() * 64; }
static_assert(pool_tickets<6>() >= 8 && pool_lds_bytes<6>() * 6 <= 160 * 1024, "6 workgroups per CU");
static_assert(pool_lds_bytes<5>() * 5 <= 160 * 1024, "5 workgroups per CU");

// A ray's stack: column `col` of the workgroup's stack arrays (entry i at i * kPoolBlock + col).
struct PoolStack {
  uint32_t col;
  __device__ __forceinline__ int ld(int i) const {
    extern __shared__ int s_lds[];
    const uint32_t x = (uint32_t)i * kPoolBlock + col;
    const int8_t* hi = (const int8_t*)s_lds + kPoolHiOff;
    const uint16_t* lo = (const uint16_t*)((const char*)s_lds + kPoolLoOff);
    return ((int)hi[x] << 16) | (int)lo[x];
  }
  __device__ __forceinline__ void st(int i, int v) const {
    extern __shared__ int s_lds[];
    const uint32_t x = (uint32_t)i * kPoolBlock + col;
    int8_t* hi = (int8_t*)s_lds + kPoolHiOff;
    uint16_t* lo = (uint16_t*)((char*)s_lds + kPoolLoOff);
    lo[x] = (uint16_t)v;
    hi[x] = (int8_t)(v >> 16);
  }
};

// Position of the n-th (from 0) set bit of m (n < popcount(m)).
__device__ __forceinline__ uint32_t nth_set_bit(uint32_t m, uint32_t n) {
  uint32_t pos = 0, c = (uint32_t)__popc(m & 0xffffu);
  if (n >= c) { n -= c; m >>= 16; pos += 16; }
  c = (uint32_t)__popc(m & 0xffu);
  if (n >= c) { n -= c; m >>= 8; pos += 8; }
  c = (uint32_t)__popc(m & 0xfu);
  if (n >= c) { n -= c; m >>= 4; pos += 4; }
  c = (uint32_t)__popc(m & 0x3u);
  if (n >= c) { n -= c; m >>= 2; pos += 2; }
  return pos + (n >= (m & 1u) ? 1u : 0u);
}
// The lowest m set bits of mask.
__device__ __forceinline__ uint32_t lowest_bits(uint32_t mask, uint32_t m) {
  if (m >= (uint32_t)__popc(mask)) return mask;
  return mask & ((1u << nth_set_bit(mask, m)) - 1u);
}

// Ray record, 4 x float4: (o, bt), (d, bi), (inv, ref | sp << 23), (ot, triangle | count << 20 | col << 24)
// (the open leaf's next triangle and the triangles left in it, in records of kTriRecordBytes).
// Exact for Stack24 trees: internal refs are byte offsets < 2^23 (kNoRef coded 0x7fffff,
// never a multiple of 80 or 128), sp <= 32, triangles < 2^20, a leaf <= 8 triangles,
// stack columns < 256.
constexpr uint32_t kRecNoRef = 0x7fffffu;
__device__ __forceinline__ void rec_put(float4* __restrict__ r, f3 o, f3 d, const Trav& t, uint32_t col) {
  const uint32_t ref = t.ref == kNoRef ? kRecNoRef : (uint32_t)t.ref;
  r[0] = make_float4(o.x, o.y, o.z, t.bt);
  r[1] = make_float4(d.x, d.y, d.z, __uint_as_float(t.bi));
  r[2] = make_float4(t.inv.x, t.inv.y, t.inv.z, __uint_as_float(ref | ((uint32_t)t.sp << 23)));
  r[3] = make_float4(t.ot.x, t.ot.y, t.ot.z,
                     __uint_as_float((t.lf / kTriRecordBytes) | (((t.le - t.lf) / kTriRecordBytes) << 20) |
                                     (col << 24)));
}
__device__ __forceinline__ void rec_get(const float4* __restrict__ r, f3& o, f3& d, Trav& t, uint32_t& col) {
  const float4 a = r[0], b = r[1], c = r[2], e = r[3];
  o = f3{a.x, a.y, a.z};
  d = f3{b.x, b.y, b.z};
  t.bt = a.w;
  t.bi = __float_as_uint(b.w);
  t.inv = f3{c.x, c.y, c.z};
  t.ot = f3{e.x, e.y, e.z};
  const uint32_t w2 = __float_as_uint(c.w), w3 = __float_as_uint(e.w);
  const uint32_t ref = w2 & kRecNoRef;
  t.ref = ref == kRecNoRef ? kNoRef : (int)ref;
  t.sp = (int)(w2 >> 23);
  t.lf = (w3 & 0xfffffu) * kTriRecordBytes;
  t.le = t.lf + ((w3 >> 20) & 0xfu) * kTriRecordBytes;
  col = w3 >> 24;
}

__device__ __forceinline__ uint32_t lds_load_acq(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t lds_and(uint32_t* p, uint32_t v) {
  return __hip_atomic_fetch_and(p, v, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_or_rel(uint32_t* p, uint32_t v) {
  (void)__hip_atomic_fetch_or(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// W: waves per SIMD (register budget).  STATS: the instrumented pass (counters as k_render_ps).
//
// Registers as k_render_ps: the lane's ray registers (ro, rd, t, stk) hold the ray it
// traverses, its own or an adopted one.  A lane whose own ray has finished keeps the
// result there (pend) until its service pass; to adopt another ray first, it stashes
// (o, d, bt, bi) in a free ticket of its wave, marked done for its own service pass to
// pick up.
template <bool STATS, bool CN, int W>
__global__ void __launch_bounds__(kPoolBlock) __attribute__((amdgpu_waves_per_eu(W)))
k_render_pool(DevScene sc, DevFrame fr, const wgt_tile* __restrict__ tiles, uchar4* __restrict__ out8,
              float4* __restrict__ out32, uint32_t* __restrict__ outhit, unsigned long long* __restrict__ counters,
              uint32_t* __restrict__ queue) {
  extern __shared__ int s_lds[];
  constexpr uint32_t ntk = pool_tickets<W>();
  PoolHdr* const hdr = (PoolHdr*)((char*)s_lds + kPoolHdrOff);
  float4* const recs = (float4*)((char*)s_lds + kPoolRecOff);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const unsigned long long lt_mask = (1ull << lane) - 1ull;
  if (threadIdx.x < 2 * kPoolWaves) ((uint32_t*)hdr)[threadIdx.x] = 0u;
  __syncthreads();  // the only barrier: waves run independently from here

  const Light L{xyz(sc.quads[0]), xyz(sc.quads[1]), xyz(sc.quads[2])};
  const uint32_t nsamp = fr.sqrt_spp * fr.sqrt_spp;
  const uint32_t n_slots = fr.n_slots;
  Pixel px{};
  uint32_t po = 0;
  f3 ro{}, rd{}, pc{};  // the held ray (or the own finished ray while pend)
  int depth = 0;
  TravStats st{0u, 0u, 0u, 0u};
  Counters c{0u, 0u, 0u, 0u, 0u, 0u};
  Trav t;
  t.ref = kNoRef;
  t.lf = t.le = 0u;
  t.sp = 0;
  t.bt = 0.0f;
  t.bi = kNoHit;
  PoolStack stk{threadIdx.x};
  int hticket = -1;  // held ray's ticket (wave * 32 + k), -1: the lane's own ray, never parked
  uint32_t q_prim = kNoHit;
  float q_t = kRayMax;
  uint32_t tk = 0;  // own ticket while away
  bool have = false, exhausted = false, fin = false, nanray = false;
  bool pend = false;  // own ray finished, result in (ro, rd, t.bt, t.bi), or a NaN ray (nanray)
  bool away = false;  // own ray in ticket tk: parked, taken by some lane, done or stashed
  bool hold = false;  // lane holds a ray to traverse (own or adopted) in ro / rd / t / stk
  // this wave's tickets (wave-uniform): free ones, and stashed ones (done, known locally)
  uint32_t tfree = ntk >= 32u ? 0xffffffffu : ((1u << ntk) - 1u);
  uint32_t tdone = 0u;
  // STATS: wave cycles in service / traversal, and pool events (lane counts; wave counts
  // for phases and sleeps), reported in the wgt_stats cycle fields (tests, probes)
  uint64_t cyc_svc = 0, cyc_trav = 0;
  uint32_t ev_adopt = 0, ev_miss = 0, ev_park = 0, ev_return = 0, ev_stash = 0, ev_phase = 0;

  for (;;) {
    // ------------------------------------------------------------ service phase
    uint64_t t_phase = STATS ? __builtin_amdgcn_s_memtime() : 0;
    for (;;) {
      // own rays finished elsewhere (or stashed): (o, d, bt, bi) from their tickets
      if (__ballot(away) != 0ull) {
        const uint32_t dl = __builtin_amdgcn_readfirstlane(lds_load_acq(&hdr->done[wv]));
        const uint32_t dm = dl | tdone;
        if (dm != 0u) {
          if (away && ((dm >> tk) & 1u)) {
            const float4* r = recs + (wv * ntk + tk) * 4u;
            const float4 a = r[0], b = r[1];
            ro = f3{a.x, a.y, a.z};
            rd = f3{b.x, b.y, b.z};
            t.bt = a.w;
            t.bi = __float_as_uint(b.w);
            pend = true;
            away = false;
          }
          if (dl != 0u && lane == 0) (void)lds_and(&hdr->done[wv], ~dl);
          tfree |= dm;
          tdone = 0u;
        }
      }
      if (fin) {  // a finished pixel: write it
        write_pixel(fr, po, px, out8, out32, outhit);
        if (STATS) ++c.px;
        fin = false;
      }
      // refill: lanes without a pixel take consecutive slots, one atomic per wave
      const unsigned long long idle = __ballot(!have && !exhausted);
      if (idle != 0ull) {
        const uint32_t n_idle = (uint32_t)__popcll(idle);
        if (n_idle >= fr.pq_refill || __ballot(have && !away) == 0ull) {
          const int leader = __ffsll((long long)idle) - 1;
          uint32_t base = 0;
          if ((int)lane == leader) base = atomicAdd(queue, n_idle);
          base = __shfl(base, leader);
          if (!have && !exhausted) {
            const uint32_t slot = base + (uint32_t)__popcll(idle & lt_mask);
            if (slot >= n_slots) {
              exhausted = true;
            } else {
              const uint32_t b = fr.perm ? fr.perm[slot >> 6] : (slot >> 6);
              if (slot_setup(fr, tiles, b, slot & 63u, po, px)) {
                have = true;
                depth = 0;
              }
            }
          }
        }
      }
      const bool need = have && (pend || !(hold || away));
      if (!__any(need)) {
        if (__ballot(!have && !exhausted) != 0ull && __ballot(hold || away) == 0ull) continue;  // refill again
        break;
      }
      if (need) {
        if (STATS) simt_count(c.lw, c.ll);
        if (pend) {
          // finalise: rebuild the quad hit, merge the triangle, scan spheres, shade
          Hit h;
          if (nanray) {
            nan_hit(sc, ro, rd, h);
            if (STATS) { ++c.q; ++c.nan; }
            nanray = false;
          } else {
            float4 pre[2];
            preload_tshade(sc, t, pre[0], pre[1]);
            quad_rebuild(sc, ro, rd, q_prim, q_t, h);
            finish_hit(sc, ro, rd, t, h, pre);
            if (STATS) { ++c.q; ++c.tr; }
          }
          first_hit(px, depth, h.prim, po, outhit);
          const bool end = shade(sc, L, h, depth, px.seed, ro, rd, pc);
          ++depth;
          if (end || depth == kRayDepth) {
            end_sample(fr, px, pc);
            depth = 0;
          }
          pend = false;
        }
        // start the next ray of this pixel
        for (;;) {
          if (px_done(fr, px)) {
            have = false;
            fin = true;
            break;
          }
          if (depth == 0) {
            camera_ray(fr, px, ro, rd);
            pc = f3{1.0f, 1.0f, 1.0f};
          }
          if (has_nan(ro) || has_nan(rd)) {
            if (!sc.last_sphere_emissive) {
              first_hit(px, depth, last_prim(sc), po, outhit);
              skip_nan_path<STATS>(sc, fr, px, depth, c);
              depth = 0;
              continue;
            }
            nanray = true;  // the last sphere's hit, resolved and shaded at the next finalise
            pend = true;
            break;
          }
          Hit h;
          quad_scan(sc, ro, rd, h, q_t);
          q_prim = h.prim;
          trav_init<CN>(sc, ro, rd, q_prim != kNoHit, q_t, t);
          stk.col = threadIdx.x;
          hticket = -1;
          root_step<STATS, CN>(sc, t, stk, st);  // the root: rays that miss it never traverse
          if (trav_done(t)) pend = true;
          else hold = true;
          break;
        }
      }
      if ((uint32_t)__popcll(__ballot(hold)) >= fr.ps_to_trav) break;
    }
    if (STATS) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      cyc_svc += now - t_phase;
      t_phase = now;
      ++ev_phase;
    }
    if (__ballot(have || !exhausted) == 0ull) break;  // holds nothing: adopted rays went back at the last exit
    // --------------------------------------------------------- traversal phase
    uint32_t to_service = fr.ps_to_service;
    if (fr.ps_svc_frac) {
      const uint32_t live = (uint32_t)__popcll(__ballot(have));
      const uint32_t sparse = (live * fr.ps_svc_frac) >> 6;
      to_service = sparse < to_service ? sparse : to_service;
    }
    for (;;) {
      // adopt: lanes without a ray take parked rays of the workgroup's waves
      if ((uint32_t)__popcll(__ballot(!hold)) >= fr.pool_adopt_min) {
        // a snapshot (one 16-B read): a ray is only taken by the atomic claim below
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 av = *(const volatile u32x4*)hdr->avail;
        const uint32_t a0 = __builtin_amdgcn_readfirstlane(av.x), a1 = __builtin_amdgcn_readfirstlane(av.y),
                       a2 = __builtin_amdgcn_readfirstlane(av.z), a3 = __builtin_amdgcn_readfirstlane(av.w);
        const uint32_t c0 = (uint32_t)__popc(a0), c1 = (uint32_t)__popc(a1), c2 = (uint32_t)__popc(a2),
                       c3 = (uint32_t)__popc(a3);
        const uint32_t na = c0 + c1 + c2 + c3;
        if (na != 0u) {
          // lanes with a finished own ray stash it first (as many as the pool can use)
          const uint32_t nf = (uint32_t)__popcll(__ballot(!hold && !pend));
          const unsigned long long pl = __ballot(!hold && pend);
          uint32_t ns = na > nf ? na - nf : 0u;
          ns = ns < (uint32_t)__popcll(pl) ? ns : (uint32_t)__popcll(pl);
          ns = ns < (uint32_t)__popc(tfree) ? ns : (uint32_t)__popc(tfree);
          if (ns != 0u) {
            const uint32_t sm = lowest_bits(tfree, ns);
            if (!hold && pend) {
              const uint32_t r = (uint32_t)__popcll(pl & lt_mask);
              if (r < ns) {
                tk = nth_set_bit(sm, r);
                float4* q = recs + (wv * ntk + tk) * 4u;
                q[0] = make_float4(ro.x, ro.y, ro.z, t.bt);
                q[1] = make_float4(rd.x, rd.y, rd.z, __uint_as_float(t.bi));
                pend = false;
                away = true;
                if (STATS) ++ev_stash;
              }
            }
            tfree &= ~sm;
            tdone |= sm;
          }
          const unsigned long long fl = __ballot(!hold && !pend);
          if (!hold && !pend) {
            uint32_t r = (uint32_t)__popcll(fl & lt_mask);
            if (r < na) {
              uint32_t w = 0, m = a0;
              if (r >= c0) { r -= c0; w = 1; m = a1;
                if (r >= c1) { r -= c1; w = 2; m = a2;
                  if (r >= c2) { r -= c2; w = 3; m = a3; } } }
              const uint32_t k = nth_set_bit(m, r);
              const uint32_t old = lds_and(&hdr->avail[w], ~(1u << k));
              if ((old >> k) & 1u) {  // claimed (another wave may have taken it first)
                uint32_t col;
                rec_get(recs + (w * ntk + k) * 4u, ro, rd, t, col);
                stk.col = col;
                hticket = (int)(w * 32u + k);
                hold = true;
                if (STATS) ++ev_adopt;
              } else if (STATS) {
                ++ev_miss;
              }
            }
          }
        }
      }
      if (__ballot(hold) == 0ull) {
        // nothing to traverse: the wave's own rays (if any) are with other waves
        if (!__any(pend) && __ballot(!have && !exhausted) == 0ull && tdone == 0u) __builtin_amdgcn_s_sleep(2);
        break;
      }
      // one uniform mode per step (k_render_ps): triangle steps once enough lanes hold a
      // pending leaf, else node steps
      const bool can_node = hold && t.ref != kNoRef;
      const bool can_tri = hold && t.lf < t.le;
      const uint32_t nn = (uint32_t)__popcll(__ballot(can_node));
      const uint32_t nl = (uint32_t)__popcll(__ballot(can_tri));
      const bool tri_mode = nn == 0 || nl * 100u >= nn * fr.tri_ratio;
      if (STATS && (tri_mode ? can_tri : can_node)) simt_count(st.wave_steps, st.lane_steps);
      if (tri_mode) {
        if (can_tri) tri_step<STATS, CN>(sc, ro, rd, t, stk, st);
      } else {
        if (can_node) node_step<STATS, CN>(sc, t, stk, st);
      }
      if (hold && trav_done(t)) {
        hold = false;
        if (hticket < 0) {
          pend = true;  // own ray: the result stays in the registers
        } else {  // another lane's ray: the result to its ticket, the owner collects it
          const uint32_t w = (uint32_t)hticket >> 5, k = (uint32_t)hticket & 31u;
          float4* r = recs + (w * ntk + k) * 4u;
          r[0].w = t.bt;
          r[1].w = __uint_as_float(t.bi);
          lds_or_rel(&hdr->done[w], 1u << k);
        }
      }
      // leave once few rays are left and lanes of this wave wait for service (checked
      // after a step, so that every traversal phase advances its rays)
      const uint32_t nh = (uint32_t)__popcll(__ballot(hold));
      if (nh == 0) break;
      if (nh <= to_service) {
        bool svc = __any(have ? pend : !exhausted) || tdone != 0u;
        if (!svc && __ballot(away) != 0ull) svc = lds_load_acq(&hdr->done[wv]) != 0u;
        if (svc) {
          // leave: adopted rays back to their tickets, own unfinished rays into free tickets
          if (hold && hticket >= 0) {
            const uint32_t w = (uint32_t)hticket >> 5, k = (uint32_t)hticket & 31u;
            rec_put(recs + (w * ntk + k) * 4u, ro, rd, t, stk.col);
            lds_or_rel(&hdr->avail[w], 1u << k);
            hold = false;
            if (STATS) ++ev_return;
          }
          const unsigned long long own = __ballot(hold);  // hticket < 0 for every held ray now
          if (fr.pool_park && own != 0ull && tfree != 0u) {
            const uint32_t alloc = lowest_bits(tfree, (uint32_t)__popcll(own));
            if (hold) {
              const uint32_t r = (uint32_t)__popcll(own & lt_mask);
              if (r < (uint32_t)__popc(alloc)) {
                tk = nth_set_bit(alloc, r);
                rec_put(recs + (wv * ntk + tk) * 4u, ro, rd, t, threadIdx.x);
                away = true;
                hold = false;
                if (STATS) ++ev_park;
              }
            }
            tfree &= ~alloc;
            if (lane == 0) lds_or_rel(&hdr->avail[wv], alloc);
          }
          break;
        }
      }
    }
    if (STATS) cyc_trav += __builtin_amdgcn_s_memtime() - t_phase;
  }
  if (STATS) {
    flush_counters(counters, c, st, nsamp);
    atomicAdd(&counters[CNT_CYC_REFILL], (unsigned long long)ev_adopt);
    atomicAdd(&counters[CNT_CYC_FINALISE], (unsigned long long)ev_miss);
    atomicAdd(&counters[CNT_CYC_SHADE], (unsigned long long)ev_park);
    atomicAdd(&counters[CNT_CYC_CAMERA], (unsigned long long)ev_return);
    atomicAdd(&counters[CNT_CYC_QUADS], (unsigned long long)ev_stash);
    if (lane == 0) {
      atomicAdd(&counters[CNT_CYC_SERVICE], (unsigned long long)cyc_svc);
      atomicAdd(&counters[CNT_CYC_TRAV], (unsigned long long)cyc_trav);
      atomicAdd(&counters[CNT_CYC_ROOT], (unsigned long long)ev_phase);
    }
  }
}

// Waves per SIMD of the pool kernel: 6 (the 80-VGPR budget of k_render_ps, 3-byte stack
// entries), or 5 (96 VGPRs, WGT_POOL=5)
template <bool STATS>
static void pool_launch(const DevScene& sc, bool cn, int w, dim3 grid, size_t lds, hipStream_t stream,
                        const DevFrame& f, const wgt_tile* tiles, uchar4* out8, float4* out32, uint32_t* outhit,
                        unsigned long long* counters, uint32_t* queue) {
  const dim3 block(kPoolBlock);
  if (w == 5) {
    if (cn) k_render_pool<STATS, true, 5><<<grid, block, lds, stream>>>(sc, f, tiles, out8, out32, outhit, counters, queue);
    else k_render_pool<STATS, false, 5><<<grid, block, lds, stream>>>(sc, f, tiles, out8, out32, outhit, counters, queue);
  } else {
    if (cn) k_render_pool<STATS, true, 6><<<grid, block, lds, stream>>>(sc, f, tiles, out8, out32, outhit, counters, queue);
    else k_render_pool<STATS, false, 6><<<grid, block, lds, stream>>>(sc, f, tiles, out8, out32, outhit, counters, queue);
  }
}

hipError_t launch_pool(const DevScene& sc, const DevFrame& f, bool cn, uint32_t resident_wgs, const wgt_tile* tiles,
                       uchar4* out8, float4* out32, uint32_t* outhit, unsigned long long* counters, uint32_t* queue,
                       hipStream_t stream) {
  if (sc.stack > kPoolStack) return hipErrorInvalidValue;
  const uint32_t nb = f.n_slots / 64u;  // pixel blocks = waves' worth of slots
  const uint32_t wgs = (nb + kPoolWaves - 1) / kPoolWaves;
  const dim3 grid(wgs < resident_wgs ? wgs : resident_wgs);
  const size_t lds = f.pool == 5 ? pool_lds_bytes<5>() : pool_lds_bytes<6>();
  if (counters) pool_launch<true>(sc, cn, (int)f.pool, grid, lds, stream, f, tiles, out8, out32, outhit, counters, queue);
  else pool_launch<false>(sc, cn, (int)f.pool, grid, lds, stream, f, tiles, out8, out32, outhit, nullptr, queue);
  return hipGetLastError();
}

uint32_t pool_tickets_for(int w) { return w == 5 ? pool_tickets<5>() : pool_tickets<6>(); }

hipError_t pool_resident_wgs(int w, int device, uint32_t& wgs) {
  const void* k[2] = {w == 5 ? reinterpret_cast<const void*>(&k_render_pool<false, true, 5>)
                             : reinterpret_cast<const void*>(&k_render_pool<false, true, 6>),
                      w == 5 ? reinterpret_cast<const void*>(&k_render_pool<false, false, 5>)
                             : reinterpret_cast<const void*>(&k_render_pool<false, false, 6>)};
  const size_t lds = w == 5 ? pool_lds_bytes<5>() : pool_lds_bytes<6>();
  int per_cu = 0, cus = 0;
  for (const void* f : k) {
    int n = 0;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, kPoolBlock, lds);
    if (e != hipSuccess) return e;
    per_cu = n > per_cu ? n : per_cu;
  }
  const hipError_t e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  if (e != hipSuccess) return e;
  wgs = (uint32_t)((per_cu > 0 ? per_cu : 1) * (cus > 0 ? cus : 1));
  return hipSuccess;
}

}  // namespace wgt
