// wgt_internal.h — device-side data layout shared by the kernel TU and the
// runtime TU (not part of the public ABI).
//
// HBM layout of a scene:
//   quads   : lights then quads, 96-B reference records (6 x float4) — read with
//             wave-uniform (scalar) loads, 1.7 KB for the Cornell box
//   spheres : 32-B reference records (2 x float4)
//   nodes   : BVH4 nodes, 128 B (8 x float4, one cache line), root = node 0,
//             see wgt_geom.h
//   tris    : leaf-ordered Moller-Trumbore records, 64 B (4 x float4) carrying
//             the padded triangle box, see wgt_geom.h
//   tshade  : per ORIGINAL triangle, 32 B: (face_norm.xyz, emissive), (col.xyz, 0)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/wgt_api.h"

namespace wgt {

constexpr int kBlock = 64;        // one wave per block: 8x8 pixels
// Per-lane traversal stack in LDS, stride kBlock (conflict-free), sized per scene
// at launch (dynamic LDS) to the builder's exact worst case DevScene::stack, so it
// cannot overflow and needs no spill path.  kMaxBvhDepth bounds the SAH BVH2 the
// BVH4 is collapsed from; kStackMax bounds the builder's stack need: + 1 parking
// slot, so that LDS (160 KB per CU) admits 5 waves per SIMD (4 SIMDs per CU):
// 32 entries = 8 KB per wave.  k_render_ps stores 3-byte entries when the tree's
// refs fit them (6 KB per wave): 6 waves per SIMD at 80 VGPRs (DESIGN.md §4.2,
// DevScene::ps_waves).  kStackNarrow is the optional narrow collapse (WGT_NARROW).
constexpr int kMaxBvhDepth = 24;
constexpr int kStackMax = 31;
constexpr int kStackNarrow = 25;
// k_render_ps on scenes without triangles (no traversal, no stack): its register budget
constexpr int kPsWavesNoTris = 8;
static_assert((kStackMax + 1) * kBlock * 4 * 5 * 4 <= 160 * 1024, "5 waves per SIMD");
static_assert((kStackNarrow + 1) * kBlock * 4 * 6 * 4 <= 160 * 1024, "6 waves per SIMD");
static_assert((kStackMax + 1) * kBlock * 3 * 6 * 4 <= 160 * 1024, "6 waves per SIMD, 3-byte entries");

struct DevScene {
  const float4* __restrict__ quads;   // n_lights + n_quads records
  const float4* __restrict__ spheres; // n_spheres records
  const float4* __restrict__ nodes;
  const float4* __restrict__ tris;
  const float4* __restrict__ tshade;
  const float4* __restrict__ cnodes;  // the same tree as 80-B compact records (wgt_geom.h)
  // the level of each BVH4 node (root 0), by node index: read by the instrumented (STATS) passes
  // only, to split node visits and traversal-step cycles by tree level
  const uint8_t* __restrict__ node_level;
  float cstep;                        // scene-wide decode step of the compact nodes (a power of two)
  float rcstep;                       // 1 / cstep
  float cbound;                       // the compact codes hold for ray origins with |coordinate| <= cbound
  uint32_t n_lights, n_quads, n_spheres, n_tris;
  uint32_t n_nodes;
  uint32_t last_sphere_emissive;
  float light_area;  // length(cross(lights[0].right, lights[0].up)) (path_tracer.wgsl:205)
  uint32_t stack;     // traversal stack entries per lane (>= 1)
  // k_render_ps waves per SIMD: 6 (3-byte stack entries, Stack24) when every ref of
  // the tree fits 24 bits (kStack24Nodes, kStack24Tris), else 5
  uint32_t ps_waves;
  // k_render_ps with parked traversal state (ps_park = 1): the
  // LDS holds ps_cap stack entries per lane (<= stack) plus kParkWords words of the
  // lane's traversal state; entries beyond ps_cap move to a per-lane global stack
  // (DevFrame::ps_spill) in the service phase.  ps_park = 0: the whole stack in LDS.
  uint32_t ps_park, ps_cap;
};
constexpr uint32_t kStack24Nodes = 1u << 16;  // 128-B node byte offsets < 2^23
constexpr uint32_t kStack24Tris = 1u << 20;   // leaf refs ~(first << 3 | count - 1) >= -2^23
// Parked traversal state per lane (wgt_device.h Park): 1/d (3), slab offsets (3), best t,
// best index, node ref, stack top | global depth << 16, open leaf (offset | count)
constexpr uint32_t kParkWords = 11;
// The smallest LDS stack the parked kernel runs with: a node step needs 4 free entries
// above the top (3 pushes and a parked leaf), and a ray's root step, which pushes at most
// 4, must leave its top within that bound (top <= cap - 4), so a new ray never starts
// past it
constexpr uint32_t kMinPsCap = 8;
// Dynamic LDS bytes of a traversal kernel launch (4-byte entries).
inline size_t stack_lds_bytes(const DevScene& sc) { return (size_t)sc.stack * kBlock * sizeof(int); }
// ... of a k_render_ps launch: 3-byte entries at 6 waves per SIMD, ps_cap entries and
// the parked state when ps_park
inline size_t ps_stack_lds_bytes(const DevScene& sc) {
  const size_t entry = sc.ps_waves >= 6 ? 3 : sizeof(int);
  if (sc.ps_park) return (size_t)sc.ps_cap * kBlock * entry + (size_t)kParkWords * kBlock * 4;
  return (size_t)sc.stack * kBlock * entry;
}
// LDS entries the parked kernel can hold at its wave budget: the stack and the parked words
// of 4 * waves one-wave workgroups per CU within kPsLdsPerCu.  Measured (profiles/r04/
// lds_sweep_*.jsonl): 24 workgroups per CU run at full speed with 6,272 B each and lose 8-20 %
// from 6,464 B on, although the occupancy API still reports 24 (and 160 KiB would hold 24 of
// 6,656 B): the usable budget lies between 24 x 6,400 and 24 x 6,656 B, so 150 KiB is taken
// (6 waves: 18 entries of 3 B beside the 11 parked words; 5 waves: 19 of 4 B)
constexpr size_t kPsLdsPerCu = 150 * 1024;
inline uint32_t ps_cap_max(uint32_t waves) {
  const size_t per_wave = kPsLdsPerCu / (4 * waves), entry = waves >= 6 ? 3 : 4;
  return (uint32_t)((per_wave - (size_t)kParkWords * kBlock * 4) / (kBlock * entry));
}

// 1 / spp when spp is a power of two (exact in fp32: end_sample multiplies), else 0
inline float pow2_recip(uint32_t spp) { return (spp != 0u && (spp & (spp - 1u)) == 0u) ? 1.0f / (float)spp : 0.0f; }

// Per-frame camera constants of setup_camera_ray (path_tracer.wgsl:239-262),
// computed once on the host with the same fp32 operations (wgt_math.h).
struct DevFrame {
  float ox, oy, oz;    // origin
  float pox, poy, poz; // pixel_origin
  float dux, duy, duz; // pixel_delta_u
  float dvx, dvy, dvz; // pixel_delta_v
  float recip_sqrt_spp;
  float fspp;          // f32(camera.spp)
  float inv_fspp;      // 1 / fspp when spp is a power of two (exact), else 0
  uint32_t sqrt_spp;
  uint32_t W, H;
  uint32_t tw, th, n_tiles;
  // kernel selection and phase-split thresholds (k_render_ps): switch from the
  // service to the traversal phase once >= ps_to_trav lanes traverse, and back
  // once <= ps_to_service lanes still traverse.
  uint32_t kernel;  // 2 = the persistent phase-split kernel (default), else the simple one
  uint32_t ps_to_trav, ps_to_service;
  // a wave with fewer live pixels leaves the traversal phase at <= live *
  // ps_svc_frac / 64 traversing lanes (if lower): a sparse wave (the end of a
  // launch) would otherwise pay a service pass for every finished ray (0 = off)
  uint32_t ps_svc_frac;
  // speculative traversal: a triangle step runs when lanes with a pending leaf
  // number >= tri_ratio % of the lanes with a node to visit
  uint32_t tri_ratio;
  // BVH node form of k_render_ps: 0 = 128-B nodes, 1 = 80-B compact records, 2 = 80-B
  // compact records when the 128-B tree exceeds kCompactNodeBytes (default) (node_form)
  uint32_t cnode;
  // persistent k_render_ps: pixel slots of the launch (64 per 8x8 block), the
  // idle lanes that trigger a refill from the pixel queue, LPT ordering (0 = off,
  // n = order from an n*n-spp cost pre-pass),
  // the queue order (queue block q renders pixel block perm[q]; NULL = identity)
  // and the pre-pass cost per pixel block (set by launch_render)
  uint32_t n_slots, pq_refill, pq_lpt;
  uint32_t pq_lpt_all;  // the pre-pass renders all 64 pixels of each block (else the 16 at even x, y)
  uint32_t pq_svc_cost;  // pre-pass work units per ray started (a service iteration ~ 7 traversal steps)
  uint32_t pq_depth;     // the pre-pass's paths end at this depth (kRayDepth: the full path)
  const uint32_t* perm;
  uint32_t* cost;
  // parked k_render_ps (DevScene::ps_park): the global part of the lanes' stacks, entry e
  // of the lane (wave w, lane l) at ps_spill[e * ps_spill_stride + w * 64 + l] (launch_render)
  int* ps_spill;
  uint32_t ps_spill_stride;
  // (2^32 - 1) / d for the 8x8 blocks per tile row (bx) and per tile (bx * by) of the launch
  // (launch_render): slot_setup's divisions by them (wgt_device.h udiv_by)
  uint32_t div_bx, div_bpt;
};

enum {
  CNT_QUERIES = 0,
  CNT_TRACED,
  CNT_SAMPLES,
  CNT_NAN,
  CNT_NODES,
  CNT_TRIS,
  CNT_PIXELS,
  CNT_LOOP_WAVE,
  CNT_LOOP_LANE,
  CNT_TRAV_WAVE,
  CNT_TRAV_LANE,
  CNT_CYC_SERVICE,  // s_memtime cycles per wave spent in each phase (instrumented pass)
  CNT_CYC_TRAV,
  CNT_CYC_REFILL,  // service-phase regions (k_render_ps, instrumented pass)
  CNT_CYC_FINALISE,
  CNT_CYC_SHADE,
  CNT_CYC_CAMERA,
  CNT_CYC_QUADS,
  CNT_CYC_ROOT,
  CNT_STACK_SPILLS,   // parked k_render_ps: LDS stack overflows moved to the global stack
  CNT_STACK_REFILLS,  // ... and refills from it
  CNT_STACK_OVERFLOWS,  // ... and traversals park_fix ended on its overflow exit (a wrong pixel)
  // traversal phase by tree level (instrumented pass): lane visits of nodes at levels 1-2 (the
  // root's children and grandchildren; the root itself is visited in the service phase), and the
  // cycles of node steps, of node steps whose every visiting lane is at levels 1-2, and of
  // triangle steps
  CNT_TOP_NODES,
  CNT_CYC_NODE_STEPS,
  CNT_CYC_TOP_STEPS,
  CNT_CYC_TRI_STEPS,
  CNT_QUAD_REF,  // rays whose quad scan fell back to the reference scan (quad_scan_fast)
  CNT_N = 29
};

// Launchers implemented in wgt_kernels.hip
// k_render_ps runs persistent: at most `resident` waves (ps_resident_waves),
// lanes pulling pixel slots from a per-launch queue in LPT order (1-spp cost
// pre-pass + k_lpt_order), all stream-ordered on `stream`.
// ws: scheduling workspace of >= render_ws_bytes(sc, fr, resident) bytes, used in stream
// order (one launch in flight per workspace): the queues, the LPT costs and order, and the
// parked kernel's global stacks.
size_t render_ws_bytes(const DevScene& sc, const DevFrame& fr, uint32_t resident);
// ws_clean_nb: in, the block count whose queues and costs the workspace's previous LPT launch left
// zero (0: unknown, a memset clears them); out, the same for this launch
hipError_t launch_render(const DevScene& sc, const DevFrame& fr, const wgt_tile* d_tiles,
                         uchar4* out8, float4* out32, uint32_t* outhit,
                         unsigned long long* counters, uint32_t resident, void* ws, size_t ws_cap,
                         hipStream_t stream, uint32_t& ws_clean_nb);
// The node form k_render_ps reads for this scene and frame (DevFrame::cnode): 0 = 128-B
// nodes, 1 = 80-B compact records.
int node_form(const DevScene& sc, const DevFrame& fr);
// Waves of k_render_ps resident on the whole device for this scene's LDS stack.
hipError_t ps_resident_waves(const DevScene& sc, int device, uint32_t& waves);
hipError_t launch_selftest_math(uint32_t n, uint32_t seed, unsigned long long* d_counts, hipStream_t stream);
hipError_t launch_trace(const DevScene& sc, const float* d_rays, uint32_t n, uint32_t* prim,
                        float* dist, hipStream_t stream);

}  // namespace wgt
