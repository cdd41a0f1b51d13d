// wgt_runtime.cpp — the C-ABI (include/wgt_api.h) over HIP: device context and
// stream (replacing Renderer::InitDevice, render.cpp:49-147), scene upload with
// BVH build (replacing Scene::InitBuffers, scene.cpp:161-165), the render launch
// (replacing the compute pass of Renderer::OnRender, render.cpp:461-491) and the
// readback (replacing saveTexture's copyTextureToBuffer + mapAsync,
// save_texture.h:10-87).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/wgt_api.h"
#include "host/bvh.h"
#include "wgt_error.h"
#include "wgt_geom.h"
#include "wgt_internal.h"

using namespace wgt;

namespace {
thread_local std::string g_err;

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};
}  // namespace

namespace wgt {
void set_thread_error(const std::string& msg) { g_err = msg; }
}  // namespace wgt

struct wgt_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::string err;
  bool has_scene = false;
  DevScene sc{};
  void* scene_mem = nullptr;
  wgt_scene_info info{};
  // scratch for the synchronous entry points
  DevBuf tiles, out8, out32, hit, counters, rays, prim, dist;
  uint32_t ps_resident = 0;
  // Scheduling workspaces of the persistent kernel (queues, LPT costs and order),
  // used round-robin by its launches.  A launch waits (on the device) only for the
  // previous launch that used the same slot, so consecutive frames issued on two
  // streams overlap: the next frame's pre-pass and first waves fill the CUs that the
  // previous frame's end-of-launch drain leaves idle.
  static constexpr int kMaxWsSlots = 4;
  struct WsSlot {
    DevBuf ws;
    hipEvent_t ev = nullptr;  // recorded after the slot's last launch
    uint32_t clean_nb = 0;    // launch_render: the block count its last LPT launch left zero
  };
  WsSlot slots[kMaxWsSlots];
  uint32_t next_slot = 0;
  // wgt_pipeline_stream: streams for frames issued round-robin, each created with a
  // full CU mask, which gives it a hardware queue of its own (two plain streams may
  // share one, and launches on one hardware queue never overlap)
  hipStream_t pipe[kMaxWsSlots] = {};
  // recorded after every other launch that reads the scene (trace queries); each such
  // launch first waits for the previous one.  The scene
  // and the workspaces are freed (re-upload, destroy, regrow) only after this event
  // and every slot's event have completed
  hipEvent_t use_ev = nullptr;
  std::vector<hipEvent_t> evpool;  // per-launch timing (profile runs only)
};

namespace {

int fail(wgt_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  g_err = msg;
  return code;
}

#define WGT_HIP(ctx, expr)                                                                    \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess)                                                                     \
      return fail((ctx), WGT_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));       \
  } while (0)

// Order a launch on stream s after every earlier launch of the context (any stream).
int use_begin(wgt_ctx* ctx, hipStream_t s) {
  if (!ctx->use_ev) WGT_HIP(ctx, hipEventCreateWithFlags(&ctx->use_ev, hipEventDisableTiming));
  else WGT_HIP(ctx, hipStreamWaitEvent(s, ctx->use_ev, 0));
  return WGT_OK;
}
int use_end(wgt_ctx* ctx, hipStream_t s) {
  WGT_HIP(ctx, hipEventRecord(ctx->use_ev, s));
  return WGT_OK;
}
// Host wait for every launch of the context (before freeing what they read).
int use_drain(wgt_ctx* ctx) {
  if (ctx->use_ev) WGT_HIP(ctx, hipEventSynchronize(ctx->use_ev));
  for (auto& sl : ctx->slots)
    if (sl.ev) WGT_HIP(ctx, hipEventSynchronize(sl.ev));
  WGT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return WGT_OK;
}

int ensure(wgt_ctx* ctx, DevBuf& b, size_t bytes) {
  if (b.bytes >= bytes) return WGT_OK;
  if (b.p) {
    (void)use_drain(ctx);  // launches on any stream may still use the old buffer
    (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
  }
  size_t want = std::max<size_t>(bytes, 256);
  WGT_HIP(ctx, hipMalloc(&b.p, want));
  b.bytes = want;
  return WGT_OK;
}

void free_buf(DevBuf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
}

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Tuning knobs (read per launch; defaults are the measured best).
uint32_t env_u32(const char* name, uint32_t dflt) {
  const char* v = std::getenv(name);
  if (!v || !*v) return dflt;
  return (uint32_t)std::strtoul(v, nullptr, 10);
}

// setup_camera_ray's frame-invariant terms (path_tracer.wgsl:239-257), same fp32
// operations as the WGSL per-invocation evaluation.
// The builder's stack bound (WGT_STACK_LIMIT overrides kStackMax for sweeps).
uint32_t stack_limit() { return std::min(env_u32("WGT_STACK_LIMIT", (uint32_t)kStackMax), (uint32_t)kStackMax); }
// The narrow collapse (a 25-entry stack bound), off by default since 3-byte stack
// entries give 6 waves per SIMD the full bound: WGT_NARROW=1 takes it when its SAH
// cost is within kNarrowNodeRatio of the wide tree's, 2 whenever the BVH2 is shallow
// enough (sweeps).
uint32_t narrow_limit() { return env_u32("WGT_NARROW", 0) ? (uint32_t)kStackNarrow : 0u; }
double narrow_ratio() { return env_u32("WGT_NARROW", 0) == 2 ? 1e30 : kNarrowNodeRatio; }
// k_render_ps waves per SIMD (DevScene::ps_waves): 6 with 3-byte stack entries when
// every ref fits them, else 5; WGT_PS_WAVES=5 forces 5 (sweeps).
uint32_t ps_waves_for(const BvhOut& bvh, uint32_t n_tris) {
  // no triangles: the kernel without traversal (4-byte stack bytes in the launch and
  // the occupancy query alike, ps_stack_lds_bytes)
  if (n_tris == 0) return (uint32_t)kPsWavesNoTris;
  if (env_u32("WGT_PS_WAVES", 0) == 5) return 5u;
  const bool fits24 = bvh.n_nodes < kStack24Nodes && n_tris < kStack24Tris;
  return fits24 ? 6u : 5u;
}

// Parked traversal state of k_render_ps (opt-in: WGT_PARK=1; it
// removes the service phase's scratch stores but measured 5 % slower, profiles/r04/): the LDS
// stack holds what fits beside the parked words at the wave budget,
// or the whole stack (`stack` entries) when that is smaller; WGT_PS_CAP lowers it, down to
// kMinPsCap, for tests.
void ps_park_cap(uint32_t n_tris, uint32_t stack, uint32_t waves, uint32_t& park, uint32_t& cap) {
  park = n_tris > 0 && env_u32("WGT_PARK", 0) ? 1u : 0u;
  cap = stack;
  if (!park) return;
  uint32_t c = std::min(stack, ps_cap_max(waves));
  c = std::min(c, std::max(env_u32("WGT_PS_CAP", c), kMinPsCap));
  cap = std::max(c, kMinPsCap);
}

DevFrame make_frame(const wgt_camera_param& cam, uint32_t W, uint32_t H) {
  DevFrame fr{};
  const float theta = radians_w(cam.fovy);
  const f3 origin = f3{cam.origin[0], cam.origin[1], cam.origin[2]};
  const f3 end = f3{cam.target[0], cam.target[1], cam.target[2]};
  const float focal_length = length(origin - end);
  const float h = tan_w(theta * 0.5f);
  const float viewport_height = 2.0f * h * focal_length;
  const float viewport_width = viewport_height * cam.aspect;
  const f3 w = normalize(origin - end);
  const f3 u = normalize(cross(f3{0.0f, 1.0f, 0.0f}, w));
  const f3 v = cross(w, u);
  const f3 viewport_u = viewport_width * u;
  const f3 viewport_v = viewport_height * (-v);
  const f3 du = viewport_u / (float)W;
  const f3 dv = viewport_v / (float)H;
  const f3 vul = ((origin - focal_length * w) - 0.5f * viewport_u) - 0.5f * viewport_v;
  const f3 po = vul + 0.5f * (du + dv);
  fr.ox = origin.x; fr.oy = origin.y; fr.oz = origin.z;
  fr.pox = po.x; fr.poy = po.y; fr.poz = po.z;
  fr.dux = du.x; fr.duy = du.y; fr.duz = du.z;
  fr.dvx = dv.x; fr.dvy = dv.y; fr.dvz = dv.z;
  fr.recip_sqrt_spp = 1.0f / __builtin_sqrtf((float)cam.spp);
  fr.fspp = (float)cam.spp;
  fr.inv_fspp = pow2_recip(cam.spp);
  fr.sqrt_spp = (uint32_t)__builtin_sqrtf((float)cam.spp);
  fr.W = W;
  fr.H = H;
  fr.kernel = env_u32("WGT_KERNEL", 2);
  // swept on the persistent BVH4 kernel with compact nodes (DESIGN.md §4.2,
  // profiles/sweeps/r01_sweep_compact_knobs.jsonl)
  // 0 = by the kernel's waves per SIMD: 18/16 at 5, 16/14 at 6 (launch_render)
  fr.ps_to_trav = env_u32("WGT_PS_TO_TRAV", 0);
  fr.ps_to_service = env_u32("WGT_PS_TO_SERVICE", 0);
  fr.ps_svc_frac = env_u32("WGT_PS_SVC_FRAC", 16);  // sweep: profiles/sweeps/r01_ps_svc_frac.jsonl
  // >= 1: with 0 a wave whose lanes all hold a node but no open leaf would take triangle steps forever
  fr.tri_ratio = std::max<uint32_t>(env_u32("WGT_TRI_RATIO", 100), 1u);
  fr.cnode = env_u32("WGT_CNODE", 1);  // compact nodes (2: only once the 128-B tree outgrows an XCD's L2)
  fr.pq_refill = env_u32("WGT_PQ_REFILL", 0);  // 0 = the default, 2 (launch_render)
  // 0: block order (A/B); n: LPT order from an n*n-spp cost pre-pass (when spp > n*n)
  fr.pq_lpt = env_u32("WGT_PQ_LPT", 1);
  fr.pq_svc_cost = env_u32("WGT_PQ_SVC_COST", 7);
  // the pre-pass's paths end at depth 6 (a cost estimate needs the path's first bounces, and
  // the full 50-bounce tail set the pre-pass's own drain): sponza +0.4%, bunny +0.7%, the frame
  // alone -0.6% against full paths, 3 rounds on one box (profiles/sweeps/r04_pq_depth.log)
  fr.pq_depth = std::min<uint32_t>(std::max<uint32_t>(env_u32("WGT_PQ_DEPTH", 6), 1u), (uint32_t)kRayDepth);
  fr.pq_lpt_all = env_u32("WGT_PQ_LPT_ALL", 1);  // sweep: all pixels -3% (sponza), -4% (bunny) at 256 spp
  return fr;
}

// Numeric limits under which the kernels' short division (wgt_math.h div_rn, the
// quad plane distance) is exact wherever it decides anything:
// scene coordinates and ray origins within 2^40, quad normals within 2 per
// component (or NaN: a degenerate quad), triangle edge components within 2^30 (the
// short 1/det of Moller-Trumbore), primary ray directions within 2^32
// (scattered directions are unit).  Everything else in the kernels is exact for
// any input.  Outside the limits the calls fail with WGT_E_INVALID.
constexpr double kCoordLimit = 1099511627776.0;  // 2^40
constexpr double kEdgeLimit = 1073741824.0;      // 2^30: triangle edges (Moller-Trumbore's short 1/det)
constexpr double kPrimaryDirLimit = 4294967296.0;  // 2^32

bool finite_within(const float* v, int n, double lim) {
  for (int i = 0; i < n; ++i)
    if (!(std::fabs((double)v[i]) <= lim)) return false;  // NaN and inf fail too
  return true;
}

std::string check_scene_limits(const wgt_quad* lq, uint32_t nlq, const wgt_sphere* sp, uint32_t ns,
                               const wgt_triangle* tr, uint32_t nt) {
  for (uint32_t i = 0; i < nlq; ++i) {
    const wgt_quad& q = lq[i];
    if (!finite_within(q.pos, 3, kCoordLimit) || !finite_within(q.right, 3, kCoordLimit) ||
        !finite_within(q.up, 3, kCoordLimit) || !finite_within(&q.d, 1, kCoordLimit * 4.0))
      return "quad " + std::to_string(i) + ": position, edges and plane offset must be finite and within 2^40";
    const bool nan_norm = q.norm[0] != q.norm[0] || q.norm[1] != q.norm[1] || q.norm[2] != q.norm[2];
    if (!nan_norm && !finite_within(q.norm, 3, 2.0))
      return "quad " + std::to_string(i) + ": normal components must be within 2 (a unit normal) or NaN";
  }
  for (uint32_t i = 0; i < ns; ++i)
    if (!finite_within(sp[i].center, 3, kCoordLimit) || !finite_within(&sp[i].radius, 1, kCoordLimit))
      return "sphere " + std::to_string(i) + ": center and radius must be finite and within 2^40";
  for (uint32_t i = 0; i < nt; ++i) {
    if (!finite_within(tr[i].v0, 3, kCoordLimit) || !finite_within(tr[i].e1, 3, kCoordLimit) ||
        !finite_within(tr[i].e2, 3, kCoordLimit))
      return "triangle " + std::to_string(i) + ": vertices must be finite and within 2^40";
    // |det| <= |e1| |e2| |d| <= (sqrt(3) 2^30)^2 sqrt(3) 2^32 = 3 sqrt(3) 2^92 < 2^95 (edge components
    // within 2^30, primary-direction components within 2^32): mt_test's short 1/det is exact
    if (!finite_within(tr[i].e1, 3, kEdgeLimit) || !finite_within(tr[i].e2, 3, kEdgeLimit))
      return "triangle " + std::to_string(i) + ": edge components must be within 2^30";
  }
  return "";
}

double sq(double x) { return x * x; }

// Largest |coordinate| any point of the scene's primitives can have (quad corners,
// sphere boxes, triangle vertices): hit points, i.e. secondary ray origins, lie
// within it.  The compact nodes are built for ray origins within 4x this bound,
// which holds the reference camera outside its Cornell box (BuildBvh origin_bound).
double scene_extent(const wgt_quad* lq, uint32_t nlq, const wgt_sphere* sp, uint32_t ns, const wgt_triangle* tr,
                    uint32_t nt) {
  double m = 0.0;
  for (uint32_t i = 0; i < nlq; ++i)
    for (int c = 0; c < 3; ++c) {
      const double p = lq[i].pos[c], r = lq[i].right[c], u = lq[i].up[c];
      m = std::max({m, std::fabs(p), std::fabs(p + r), std::fabs(p + u), std::fabs(p + r + u)});
    }
  for (uint32_t i = 0; i < ns; ++i)
    for (int c = 0; c < 3; ++c) m = std::max(m, std::fabs((double)sp[i].center[c]) + std::fabs((double)sp[i].radius));
  for (uint32_t i = 0; i < nt; ++i)
    for (int c = 0; c < 3; ++c) {
      const double v = tr[i].v0[c];
      m = std::max({m, std::fabs(v), std::fabs(v + tr[i].e1[c]), std::fabs(v + tr[i].e2[c])});
    }
  return m;
}
constexpr double kOriginBoundScale = 4.0;

int check_render_args(wgt_ctx* ctx, const wgt_camera_param* cam, uint32_t W, uint32_t H,
                      uint32_t tw, uint32_t th) {
  if (!ctx) return fail(nullptr, WGT_E_INVALID, "null context");
  if (!cam) return fail(ctx, WGT_E_INVALID, "null camera");
  if (!ctx->has_scene) return fail(ctx, WGT_E_NOSCENE, "no scene uploaded");
  if (W == 0 || H == 0) return fail(ctx, WGT_E_INVALID, "empty frame");
  if (tw == 0 || th == 0) return fail(ctx, WGT_E_INVALID, "empty tile");
  if (!(cam->aspect == cam->aspect) || !(cam->fovy == cam->fovy))
    return fail(ctx, WGT_E_INVALID, "NaN camera parameter");
  // the kernels pack a sample's (s_i, s_j) into 16 bits each and count sqrt_spp^2
  // samples in 32 bits: u32(sqrt(f32(spp))) must stay <= 65535 (spp < 2^32 - 2^8)
  // the kernels keep a pixel's coordinates as 16-bit halves of one register (wgt_device.h Pixel)
  if (W > 65535u || H > 65535u) return fail(ctx, WGT_E_INVALID, "frame width and height must be <= 65535");
  if ((uint32_t)__builtin_sqrtf((float)cam->spp) > 65535u)
    return fail(ctx, WGT_E_INVALID, "spp too large (u32(sqrt(f32(spp))) must be <= 65535)");
  if (!finite_within(cam->origin, 3, kCoordLimit) || !finite_within(cam->target, 3, kCoordLimit))
    return fail(ctx, WGT_E_INVALID, "camera origin and target must be finite and within 2^40");
  // primary directions: viewport point - origin, the viewport spanning [-1/2, W+1/2] x
  // [-1/2, H+1/2] pixels around po (make_frame, setup_camera_ray)
  const DevFrame fr = make_frame(*cam, W, H);
  const double po = std::sqrt(sq((double)fr.pox - fr.ox) + sq((double)fr.poy - fr.oy) + sq((double)fr.poz - fr.oz));
  const double du = std::sqrt(sq((double)fr.dux) + sq((double)fr.duy) + sq((double)fr.duz));
  const double dv = std::sqrt(sq((double)fr.dvx) + sq((double)fr.dvy) + sq((double)fr.dvz));
  if (!(po + (W + 1.0) * du + (H + 1.0) * dv <= kPrimaryDirLimit))
    return fail(ctx, WGT_E_INVALID, "camera: primary ray directions must be finite and within 2^32 "
                                    "(viewport and focal length out of range)");
  return WGT_OK;
}

void fill_stats(const unsigned long long* c, wgt_stats* s) {
  s->queries = c[CNT_QUERIES];
  s->traced_rays = c[CNT_TRACED];
  s->samples = c[CNT_SAMPLES];
  s->nan_rays = c[CNT_NAN];
  s->node_visits = c[CNT_NODES];
  s->tri_tests = c[CNT_TRIS];
  s->pixels = c[CNT_PIXELS];
  s->loop_wave_iters = c[CNT_LOOP_WAVE];
  s->loop_lane_iters = c[CNT_LOOP_LANE];
  s->trav_wave_steps = c[CNT_TRAV_WAVE];
  s->trav_lane_steps = c[CNT_TRAV_LANE];
  s->cyc_service = c[CNT_CYC_SERVICE];
  s->cyc_trav = c[CNT_CYC_TRAV];
  s->cyc_refill = c[CNT_CYC_REFILL];
  s->cyc_finalise = c[CNT_CYC_FINALISE];
  s->cyc_shade = c[CNT_CYC_SHADE];
  s->cyc_camera = c[CNT_CYC_CAMERA];
  s->cyc_quads = c[CNT_CYC_QUADS];
  s->cyc_root = c[CNT_CYC_ROOT];
  s->stack_spills = c[CNT_STACK_SPILLS];
  s->stack_refills = c[CNT_STACK_REFILLS];
  s->stack_overflows = c[CNT_STACK_OVERFLOWS];
  s->top_node_visits = c[CNT_TOP_NODES];
  s->cyc_node_steps = c[CNT_CYC_NODE_STEPS];
  s->cyc_top_steps = c[CNT_CYC_TOP_STEPS];
  s->cyc_tri_steps = c[CNT_CYC_TRI_STEPS];
  s->quad_ref_scans = c[CNT_QUAD_REF];
}


// Times of one frame's launch (profile runs only).
struct FrameTiming {
  float total_ms = 0.0f;
};

hipEvent_t pool_event(wgt_ctx* ctx, size_t i) {
  while (ctx->evpool.size() <= i) {
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    ctx->evpool.push_back(e);
  }
  return ctx->evpool[i];
}

// Render the tile list: one launch of the persistent kernel (or, WGT_KERNEL=1, of the
// simple one), asynchronous on stream s unless timed.
int render_frame(wgt_ctx* ctx, const DevFrame& fr, const wgt_tile* d_tiles, uchar4* out8, float4* out32,
                 uint32_t* outhit, unsigned long long* counters, hipStream_t s, FrameTiming* timing) {
  const uint64_t n64 = (uint64_t)fr.tw * fr.th * fr.n_tiles;
  if (n64 == 0) return WGT_OK;
  // 32-bit pixel offsets in the kernels (slot_setup)
  if (n64 > 0x7fffffffull) return fail(ctx, WGT_E_INVALID, "too many pixels in one launch");
  hipEvent_t e0 = timing ? pool_event(ctx, 0) : nullptr, e1 = timing ? pool_event(ctx, 1) : nullptr;
  if (timing && (!e0 || !e1)) return fail(ctx, WGT_E_HIP, "hipEventCreate failed");
  if (timing) WGT_HIP(ctx, hipEventRecord(e0, s));
  int rc;
  // the next workspace slot: a launch on any stream first waits for the previous
  // launch that used it (WGT_WS_SLOTS = 1 serialises every launch of the context; 4 by
  // default, one per pipeline stream, so that up to 4 frames are in flight: a strongly scaled
  // rank's share of a frame holds fewer pixels than the device has lanes)
  const uint32_t n_slots = std::min<uint32_t>(std::max<uint32_t>(env_u32("WGT_WS_SLOTS", wgt_ctx::kMaxWsSlots), 1u),
                                              (uint32_t)wgt_ctx::kMaxWsSlots);
  wgt_ctx::WsSlot& sl = ctx->slots[ctx->next_slot % n_slots];
  ctx->next_slot = (ctx->next_slot + 1) % n_slots;
  const size_t ws_need = render_ws_bytes(ctx->sc, fr, ctx->ps_resident);
  if (sl.ws.bytes < ws_need && (rc = use_drain(ctx))) return rc;  // before regrowing
  const void* old_ws = sl.ws.p;
  const size_t old_bytes = sl.ws.bytes;
  if ((rc = ensure(ctx, sl.ws, ws_need))) return rc;
  // a new workspace (ensure reallocated: its size changed, whatever address hipMalloc returned):
  // nothing is known zero
  if (sl.ws.p != old_ws || sl.ws.bytes != old_bytes) sl.clean_nb = 0;
  if (!sl.ev) WGT_HIP(ctx, hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming));
  else WGT_HIP(ctx, hipStreamWaitEvent(s, sl.ev, 0));
  {
    const hipError_t e = launch_render(ctx->sc, fr, d_tiles, out8, out32, outhit, counters, ctx->ps_resident,
                                       sl.ws.p, sl.ws.bytes, s, sl.clean_nb);
    if (e != hipSuccess) {
      sl.clean_nb = 0;
      return fail(ctx, WGT_E_HIP, std::string("launch_render: ") + hipGetErrorString(e));
    }
  }
  WGT_HIP(ctx, hipEventRecord(sl.ev, s));
  if (timing) {
    WGT_HIP(ctx, hipEventRecord(e1, s));
    WGT_HIP(ctx, hipEventSynchronize(e1));
    WGT_HIP(ctx, hipEventElapsedTime(&timing->total_ms, e0, e1));
  }
  return WGT_OK;
}

}  // namespace

extern "C" {

int wgt_version(void) { return WGT_API_VERSION; }

const char* wgt_last_error(const wgt_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

int wgt_device_count(int* count) {
  if (!count) return fail(nullptr, WGT_E_INVALID, "null count");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *count = 0;
    return fail(nullptr, WGT_E_HIP, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
  }
  *count = n;
  return WGT_OK;
}

int wgt_create(int hip_device, wgt_ctx** out) {
  if (!out) return fail(nullptr, WGT_E_INVALID, "null out");
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0)
    return fail(nullptr, WGT_E_HIP, "no HIP device available (the product has no CPU fallback)");
  if (hip_device < 0 || hip_device >= n) return fail(nullptr, WGT_E_INVALID, "bad device index");
  wgt_ctx* ctx = new wgt_ctx();
  ctx->device = hip_device;
  auto cleanup = [&](const char* what, hipError_t err) {
    std::string m = std::string(what) + ": " + hipGetErrorString(err);
    wgt_destroy(ctx);
    return fail(nullptr, WGT_E_HIP, m);
  };
  if ((e = hipSetDevice(hip_device)) != hipSuccess) return cleanup("hipSetDevice", e);
  if ((e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) != hipSuccess)
    return cleanup("hipStreamCreate", e);
  if ((e = hipEventCreate(&ctx->ev0)) != hipSuccess) return cleanup("hipEventCreate", e);
  if ((e = hipEventCreate(&ctx->ev1)) != hipSuccess) return cleanup("hipEventCreate", e);
  *out = ctx;
  return WGT_OK;
}

void wgt_destroy(wgt_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  // every launch that may read the scene or a buffer of the context (trace queries,
  // the workspace slots' renders on any stream, the context stream) ends first
  (void)use_drain(ctx);
  for (hipStream_t p : ctx->pipe)
    if (p) (void)hipStreamSynchronize(p);
  if (ctx->scene_mem) (void)hipFree(ctx->scene_mem);
  free_buf(ctx->tiles); free_buf(ctx->out8); free_buf(ctx->out32); free_buf(ctx->hit);
  free_buf(ctx->counters); free_buf(ctx->rays); free_buf(ctx->prim); free_buf(ctx->dist);
  for (auto& sl : ctx->slots) {
    if (sl.ev) (void)hipEventSynchronize(sl.ev);
    free_buf(sl.ws);
    if (sl.ev) (void)hipEventDestroy(sl.ev);
  }
  for (hipStream_t& p : ctx->pipe) {
    if (p) (void)hipStreamSynchronize(p);
    if (p) (void)hipStreamDestroy(p);
    p = nullptr;
  }
  if (ctx->use_ev) (void)hipEventDestroy(ctx->use_ev);
  for (hipEvent_t e : ctx->evpool) (void)hipEventDestroy(e);
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

void* wgt_stream(wgt_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

void* wgt_pipeline_stream(wgt_ctx* ctx, uint32_t i) {
  if (!ctx || i >= (uint32_t)wgt_ctx::kMaxWsSlots) {
    (void)fail(ctx, WGT_E_INVALID, "pipeline stream index out of range");
    return nullptr;
  }
  if (!ctx->pipe[i]) {
    if (hipSetDevice(ctx->device) != hipSuccess) return nullptr;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess || cus <= 0)
      return nullptr;
    std::vector<uint32_t> mask(((size_t)cus + 31) / 32, 0xffffffffu);
    const hipError_t e = hipExtStreamCreateWithCUMask(&ctx->pipe[i], (uint32_t)mask.size(), mask.data());
    if (e != hipSuccess) {
      ctx->pipe[i] = nullptr;
      (void)fail(ctx, WGT_E_HIP, std::string("hipExtStreamCreateWithCUMask: ") + hipGetErrorString(e));
      return nullptr;
    }
  }
  return (void*)ctx->pipe[i];
}

int wgt_sync(wgt_ctx* ctx) {
  if (!ctx) return fail(nullptr, WGT_E_INVALID, "null context");
  WGT_HIP(ctx, hipSetDevice(ctx->device));
  WGT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return WGT_OK;
}

// Host-only: build the BVH exactly as wgt_upload_scene does and export it.
int wgt_bvh_build(const wgt_triangle* tris, uint32_t n_tris, float* nodes_out, uint32_t nodes_cap,
                  float* tris_out, wgt_scene_info* info) {
  if (!tris || n_tris == 0 || !info) return fail(nullptr, WGT_E_INVALID, "null triangles or info");
  BvhOut bvh;
  std::string err;
  if (!BuildBvh(tris, n_tris, (uint32_t)kMaxBvhDepth, stack_limit(), narrow_limit(), narrow_ratio(),
                kOriginBoundScale * scene_extent(nullptr, 0, nullptr, 0, tris, n_tris), bvh, err))
    return fail(nullptr, WGT_E_INVALID, err);
  *info = wgt_scene_info{};
  info->n_tris = n_tris;
  info->bvh_nodes = bvh.n_nodes;
  info->bvh_leaves = bvh.n_leaves;
  info->bvh_max_depth = bvh.max_depth;
  info->bvh_max_leaf = bvh.max_leaf;
  info->device_bytes = (bvh.nodes.size() + bvh.tris.size() + bvh.tshade.size()) * 4;
  info->sah_cost = bvh.sah_cost;
  info->bvh_width = (uint32_t)kBvhWidth;
  info->bvh_stack = bvh.stack_need > 0 ? bvh.stack_need : 1u;
  info->bvh2_nodes = bvh.n_nodes2;
  info->bvh2_depth = bvh.depth2;
  if (nodes_out) {
    if (nodes_cap < bvh.n_nodes) return fail(nullptr, WGT_E_INVALID, "node capacity too small");
    std::memcpy(nodes_out, bvh.nodes.data(), bvh.nodes.size() * 4);
  }
  if (tris_out) std::memcpy(tris_out, bvh.tris.data(), bvh.tris.size() * 4);
  info->bvh_compact = (size_t)bvh.n_nodes * kNode4Floats * 4 > kCompactNodeBytes ? 1u : 0u;
  info->bvh_compact_step = bvh.cstep;
  info->ps_waves = ps_waves_for(bvh, n_tris);
  ps_park_cap(n_tris, (bvh.stack_need > 0 ? bvh.stack_need : 1u) + 1u, info->ps_waves, info->ps_park,
              info->ps_stack);
  return WGT_OK;
}

int wgt_bvh_build_compact(const wgt_triangle* tris, uint32_t n_tris, uint32_t* cnodes_out, int32_t* crefs_out,
                          uint32_t nodes_cap, float* step_out) {
  if (!tris || n_tris == 0 || !cnodes_out || !crefs_out || !step_out)
    return fail(nullptr, WGT_E_INVALID, "null triangles or outputs");
  BvhOut bvh;
  std::string err;
  if (!BuildBvh(tris, n_tris, (uint32_t)kMaxBvhDepth, stack_limit(), narrow_limit(), narrow_ratio(),
                kOriginBoundScale * scene_extent(nullptr, 0, nullptr, 0, tris, n_tris), bvh, err))
    return fail(nullptr, WGT_E_INVALID, err);
  if (nodes_cap < bvh.n_nodes) return fail(nullptr, WGT_E_INVALID, "node capacity too small");
  std::memcpy(cnodes_out, bvh.cnodes.data(), bvh.cnodes.size() * 4);
  std::memcpy(crefs_out, bvh.crefs.data(), bvh.crefs.size() * 4);
  *step_out = bvh.cstep;
  return WGT_OK;
}

int wgt_upload_scene(wgt_ctx* ctx, const wgt_quad* lights, uint32_t n_lights, const wgt_quad* quads,
                     uint32_t n_quads, const wgt_sphere* spheres, uint32_t n_spheres,
                     const wgt_triangle* tris, uint32_t n_tris) {
  if (!ctx) return fail(nullptr, WGT_E_INVALID, "null context");
  if (n_lights < 1 || !lights)
    return fail(ctx, WGT_E_INVALID, "need >= 1 light (sample_from_light reads lights[0])");
  if (n_spheres < 1 || !spheres)
    return fail(ctx, WGT_E_INVALID, "need >= 1 sphere (the reference binds a dummy sphere)");
  if (n_quads > 0 && !quads) return fail(ctx, WGT_E_INVALID, "null quads");
  if (n_tris > 0 && !tris) return fail(ctx, WGT_E_INVALID, "null triangles");
  // the persistent kernel keeps a pending quad hit's index + 1 in 26 bits (wgt_kernels.hip dq)
  if ((uint64_t)n_lights + n_quads >= (1u << 26) - 1u) return fail(ctx, WGT_E_INVALID, "too many lights and quads");
  {
    std::string lim = check_scene_limits(lights, n_lights, spheres, n_spheres, tris, n_tris);
    if (lim.empty() && n_quads) lim = check_scene_limits(quads, n_quads, nullptr, 0, nullptr, 0);
    if (!lim.empty()) return fail(ctx, WGT_E_INVALID, lim);
  }
  WGT_HIP(ctx, hipSetDevice(ctx->device));

  BvhOut bvh;
  if (n_tris > 0) {
    std::string err;
    const double ext = std::max({scene_extent(lights, n_lights, spheres, n_spheres, tris, n_tris),
                                 scene_extent(quads, n_quads, nullptr, 0, nullptr, 0)});
    if (!BuildBvh(tris, n_tris, (uint32_t)kMaxBvhDepth, stack_limit(), narrow_limit(), narrow_ratio(),
                  kOriginBoundScale * ext, bvh, err))
      return fail(ctx, WGT_E_INVALID, err);
  }
  const uint32_t nlq = n_lights + n_quads;
  const size_t b_quads = align256((size_t)nlq * 96);
  const size_t b_sph = align256((size_t)n_spheres * 32);
  // both node forms stay resident (the compact one is 63% of the 128-B one); the
  // launch picks one per frame (DevFrame::cnode)
  const size_t b_nodes = align256(bvh.nodes.size() * 4);
  // compact records: the 64-B node followed by its 16-B refs (wgt_geom.h)
  std::vector<uint32_t> crec((size_t)bvh.n_nodes * kCRecordFloat4s * 4);
  for (size_t i = 0; i < bvh.n_nodes; ++i) {
    std::memcpy(&crec[i * kCRecordFloat4s * 4], &bvh.cnodes[i * kCNodeFloats], kCNodeFloats * 4);
    std::memcpy(&crec[i * kCRecordFloat4s * 4 + kCNodeFloats], &bvh.crefs[i * 4], 16);
  }
  // device copies address child nodes by byte offset (one add to the uniform base in
  // the kernels instead of an index multiply); leaf refs are unchanged
  for (size_t i = 0; i < bvh.n_nodes; ++i)
    for (int k = 0; k < 4; ++k) {
      int32_t& r = reinterpret_cast<int32_t&>(crec[i * kCRecordFloat4s * 4 + kCNodeFloats + k]);
      if (r >= 0) r *= (int32_t)(kCRecordFloat4s * 16);
      int32_t r128;
      std::memcpy(&r128, &bvh.nodes[i * kNode4Floats + 24 + k], 4);
      if (r128 >= 0) r128 *= (int32_t)(kNode4Floats * 4);
      std::memcpy(&bvh.nodes[i * kNode4Floats + 24 + k], &r128, 4);
    }
  const size_t b_cnodes = align256(crec.size() * 4);
  // each node's level (root 0, saturating at 255): preorder refs point forward, so one pass
  std::vector<uint8_t> level(bvh.n_nodes, 0);
  for (size_t i = 0; i < bvh.n_nodes; ++i)
    for (int k = 0; k < 4; ++k) {
      int32_t r;
      std::memcpy(&r, &bvh.crefs[i * 4 + k], 4);
      if (r >= 0 && (size_t)r < bvh.n_nodes) level[r] = (uint8_t)std::min(255, level[i] + 1);
    }
  const size_t b_level = align256(level.size());
  // the device triangle records (wgt_geom.h kTriRecordBytes): the builder's 64-B records
  static_assert(kTriRecordBytes == kTriRecordFloats * 4, "device and host triangle records");
  const std::vector<float>& dtris = bvh.tris;
  const size_t b_tris = align256(dtris.size() * 4);
  const size_t b_shade = align256(bvh.tshade.size() * 4);
  const uint32_t waves = ps_waves_for(bvh, n_tris);
  const size_t total = b_quads + b_sph + b_nodes + b_tris + b_shade + b_cnodes + b_level;

  {
    int rc = use_drain(ctx);  // no launch on any stream may still read the old scene
    if (rc) return rc;
  }
  if (ctx->scene_mem) {
    (void)hipFree(ctx->scene_mem);
    ctx->scene_mem = nullptr;
  }
  ctx->has_scene = false;
  // a new scene: the workspaces' scheduling words are re-zeroed by the next launch's memset
  for (auto& sl : ctx->slots) sl.clean_nb = 0;
  WGT_HIP(ctx, hipMalloc(&ctx->scene_mem, total));
  char* base = (char*)ctx->scene_mem;
  std::vector<char> host(total, 0);
  std::memcpy(host.data(), lights, (size_t)n_lights * 96);
  if (n_quads) std::memcpy(host.data() + (size_t)n_lights * 96, quads, (size_t)n_quads * 96);
  std::memcpy(host.data() + b_quads, spheres, (size_t)n_spheres * 32);
  if (n_tris) {
    std::memcpy(host.data() + b_quads + b_sph, bvh.nodes.data(), bvh.nodes.size() * 4);
    std::memcpy(host.data() + b_quads + b_sph + b_nodes, dtris.data(), dtris.size() * 4);
    std::memcpy(host.data() + b_quads + b_sph + b_nodes + b_tris, bvh.tshade.data(),
                bvh.tshade.size() * 4);
    std::memcpy(host.data() + b_quads + b_sph + b_nodes + b_tris + b_shade, crec.data(), crec.size() * 4);
    std::memcpy(host.data() + b_quads + b_sph + b_nodes + b_tris + b_shade + b_cnodes, level.data(), level.size());
  }
  WGT_HIP(ctx, hipMemcpy(base, host.data(), total, hipMemcpyHostToDevice));

  DevScene& sc = ctx->sc;
  sc = DevScene{};
  sc.quads = (const float4*)base;
  sc.spheres = (const float4*)(base + b_quads);
  sc.nodes = (const float4*)(base + b_quads + b_sph);
  sc.tris = (const float4*)(base + b_quads + b_sph + b_nodes);
  sc.tshade = (const float4*)(base + b_quads + b_sph + b_nodes + b_tris);
  sc.cnodes = (const float4*)(base + b_quads + b_sph + b_nodes + b_tris + b_shade);
  sc.node_level = (const uint8_t*)(base + b_quads + b_sph + b_nodes + b_tris + b_shade + b_cnodes);
  sc.cstep = bvh.cstep;
  sc.cbound = bvh.cbound;
  sc.rcstep = 1.0f / sc.cstep;  // a power of two: exact
  sc.n_lights = n_lights;
  sc.n_quads = n_quads;
  sc.n_spheres = n_spheres;
  sc.n_tris = n_tris;
  sc.n_nodes = bvh.n_nodes;
  sc.last_sphere_emissive = spheres[n_spheres - 1].emissive > 0.0f ? 1u : 0u;
  const f3 lr = f3{lights[0].right[0], lights[0].right[1], lights[0].right[2]};
  const f3 lu = f3{lights[0].up[0], lights[0].up[1], lights[0].up[2]};
  sc.light_area = length(cross(lr, lu));  // path_tracer.wgsl:205
  // + 1: the speculative traversal parks a second leaf on the stack (wgt_device.h)
  sc.stack = (bvh.stack_need > 0 ? bvh.stack_need : 1u) + 1u;
  sc.ps_waves = waves;
  // parked traversal state (WGT_PARK=0: the whole stack in LDS);
  // the LDS stack holds what fits beside the parked words at the wave budget, or the whole
  // stack when that is smaller (WGT_PS_CAP lowers it, down to kMinPsCap, for tests)
  ps_park_cap(n_tris, sc.stack, sc.ps_waves, sc.ps_park, sc.ps_cap);
  WGT_HIP(ctx, ps_resident_waves(sc, ctx->device, ctx->ps_resident));
  if (env_u32("WGT_DEBUG", 0))
    std::fprintf(stderr, "[wgt] resident: k_render_ps %u waves; LDS stack %u of %u entries, parked %u\n",
                 ctx->ps_resident, sc.ps_cap, sc.stack, sc.ps_park);

  wgt_scene_info& in = ctx->info;
  in = wgt_scene_info{};
  in.n_lights = n_lights;
  in.n_quads = n_quads;
  in.n_spheres = n_spheres;
  in.n_tris = n_tris;
  in.bvh_nodes = bvh.n_nodes;
  in.bvh_leaves = bvh.n_leaves;
  in.bvh_max_depth = bvh.max_depth;
  in.bvh_max_leaf = bvh.max_leaf;
  in.device_bytes = total;
  in.sah_cost = bvh.sah_cost;
  in.bvh_width = n_tris ? (uint32_t)kBvhWidth : 0u;
  in.bvh_stack = n_tris ? std::max(bvh.stack_need, 1u) : 0u;
  in.bvh2_nodes = bvh.n_nodes2;
  in.bvh2_depth = bvh.depth2;
  in.bvh_compact = (size_t)bvh.n_nodes * kNode4Floats * 4 > kCompactNodeBytes ? 1u : 0u;
  in.bvh_compact_step = bvh.cstep;
  in.ps_waves = n_tris ? sc.ps_waves : 0u;
  in.ps_park = sc.ps_park;
  in.ps_stack = n_tris ? sc.ps_cap : 0u;
  {
    const wgt_camera_param cam{{278.0f, 278.0f, -800.0f}, 0.0f, {278.0f, 278.0f, 0.0f}, 0.0f, 1.0f, 40.0f, 1u, 0u};
    in.node_form = n_tris ? (uint32_t)node_form(sc, make_frame(cam, 1, 1)) : 0u;
  }
  in.ps_resident = ctx->ps_resident;
  ctx->has_scene = true;
  return WGT_OK;
}

int wgt_scene_info_get(const wgt_ctx* ctx, wgt_scene_info* info) {
  if (!ctx || !info) return fail(nullptr, WGT_E_INVALID, "null argument");
  if (!ctx->has_scene) return fail(const_cast<wgt_ctx*>(ctx), WGT_E_NOSCENE, "no scene uploaded");
  *info = ctx->info;
  return WGT_OK;
}

int wgt_render_tiles_async(wgt_ctx* ctx, const wgt_camera_param* cam, uint32_t W, uint32_t H,
                           uint32_t tw, uint32_t th, const wgt_tile* d_tiles, uint32_t n_tiles,
                           void* d_rgba8, float* d_rgba32f, uint32_t* d_hit_id, void* stream) {
  int rc = check_render_args(ctx, cam, W, H, tw, th);
  if (rc) return rc;
  if (n_tiles == 0) return WGT_OK;
  if (!d_tiles) return fail(ctx, WGT_E_INVALID, "null tile list");
  WGT_HIP(ctx, hipSetDevice(ctx->device));
  DevFrame fr = make_frame(*cam, W, H);
  fr.tw = tw;
  fr.th = th;
  fr.n_tiles = n_tiles;
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  return render_frame(ctx, fr, d_tiles, (uchar4*)d_rgba8, (float4*)d_rgba32f, d_hit_id, nullptr, s,
                      nullptr);
}

int wgt_render_tiles_stats(wgt_ctx* ctx, const wgt_camera_param* cam, uint32_t W, uint32_t H,
                           uint32_t tw, uint32_t th, const wgt_tile* d_tiles, uint32_t n_tiles,
                           wgt_stats* stats) {
  int rc = check_render_args(ctx, cam, W, H, tw, th);
  if (rc) return rc;
  if (!stats) return fail(ctx, WGT_E_INVALID, "null stats");
  std::memset(stats, 0, sizeof *stats);
  if (n_tiles == 0) return WGT_OK;
  if (!d_tiles) return fail(ctx, WGT_E_INVALID, "null tile list");
  WGT_HIP(ctx, hipSetDevice(ctx->device));
  if ((rc = ensure(ctx, ctx->counters, CNT_N * 8))) return rc;
  WGT_HIP(ctx, hipMemsetAsync(ctx->counters.p, 0, CNT_N * 8, ctx->stream));
  DevFrame fr = make_frame(*cam, W, H);
  fr.tw = tw;
  fr.th = th;
  fr.n_tiles = n_tiles;
  if ((rc = render_frame(ctx, fr, d_tiles, nullptr, nullptr, nullptr,
                         (unsigned long long*)ctx->counters.p, ctx->stream, nullptr)))
    return rc;
  unsigned long long c[CNT_N];
  WGT_HIP(ctx, hipMemcpyAsync(c, ctx->counters.p, sizeof c, hipMemcpyDeviceToHost, ctx->stream));
  WGT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  fill_stats(c, stats);
  return WGT_OK;
}

int wgt_render_tiles_profile(wgt_ctx* ctx, const wgt_camera_param* cam, uint32_t W, uint32_t H,
                             uint32_t tw, uint32_t th, const wgt_tile* d_tiles, uint32_t n_tiles,
                             wgt_stats* stats) {
  int rc = check_render_args(ctx, cam, W, H, tw, th);
  if (rc) return rc;
  if (!stats) return fail(ctx, WGT_E_INVALID, "null stats");
  std::memset(stats, 0, sizeof *stats);
  if (n_tiles == 0) return WGT_OK;
  if (!d_tiles) return fail(ctx, WGT_E_INVALID, "null tile list");
  WGT_HIP(ctx, hipSetDevice(ctx->device));
  DevFrame fr = make_frame(*cam, W, H);
  fr.tw = tw;
  fr.th = th;
  fr.n_tiles = n_tiles;
  FrameTiming timing;
  if ((rc = render_frame(ctx, fr, d_tiles, nullptr, nullptr, nullptr, nullptr, ctx->stream, &timing)))
    return rc;
  WGT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  stats->kernel_ms = timing.total_ms;
  stats->trace_ms = timing.total_ms;
  stats->iterations = 1;
  return WGT_OK;
}

int wgt_render_frames(wgt_ctx* ctx, const wgt_camera_param* cam, uint32_t W, uint32_t H,
                      const uint32_t* seeds, uint32_t n_frames, uint8_t* rgba8_out, wgt_stats* stats) {
  int rc = check_render_args(ctx, cam, W, H, W, H);
  if (rc) return rc;
  if (n_frames == 0) return WGT_OK;
  if (!seeds || !rgba8_out) return fail(ctx, WGT_E_INVALID, "null seeds or output");
  const size_t npx = (size_t)W * H;
  if (npx * n_frames > 0xffffffffull / 4) return fail(ctx, WGT_E_INVALID, "batch too large");
  WGT_HIP(ctx, hipSetDevice(ctx->device));
  // one full-frame tile per frame: the compact tile output is frame after frame
  std::vector<wgt_tile> tl(n_frames);
  for (uint32_t j = 0; j < n_frames; ++j) tl[j] = wgt_tile{0u, 0u, seeds[j], j};
  if ((rc = ensure(ctx, ctx->tiles, n_frames * sizeof(wgt_tile)))) return rc;
  if ((rc = ensure(ctx, ctx->out8, npx * n_frames * 4))) return rc;
  WGT_HIP(ctx, hipMemcpyAsync(ctx->tiles.p, tl.data(), n_frames * sizeof(wgt_tile), hipMemcpyHostToDevice,
                              ctx->stream));
  DevFrame fr = make_frame(*cam, W, H);
  fr.tw = W;
  fr.th = H;
  fr.n_tiles = n_frames;
  FrameTiming timing;
  if ((rc = render_frame(ctx, fr, (const wgt_tile*)ctx->tiles.p, (uchar4*)ctx->out8.p, nullptr, nullptr, nullptr,
                         ctx->stream, stats ? &timing : nullptr)))
    return rc;
  WGT_HIP(ctx, hipMemcpyAsync(rgba8_out, ctx->out8.p, npx * n_frames * 4, hipMemcpyDeviceToHost, ctx->stream));
  WGT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (stats) {
    rc = wgt_render_tiles_stats(ctx, cam, W, H, W, H, (const wgt_tile*)ctx->tiles.p, n_frames, stats);
    if (rc) return rc;
    stats->kernel_ms = timing.total_ms;
    stats->trace_ms = timing.total_ms;
    stats->iterations = 1;
  }
  return WGT_OK;
}

int wgt_render_tile(wgt_ctx* ctx, const wgt_camera_param* cam, uint32_t W, uint32_t H, uint32_t x0,
                    uint32_t y0, uint32_t tw, uint32_t th, uint8_t* rgba8_out, float* rgba32f_out,
                    uint32_t* hit_id_out, wgt_stats* stats) {
  int rc = check_render_args(ctx, cam, W, H, tw, th);
  if (rc) return rc;
  if (x0 >= W || y0 >= H) return fail(ctx, WGT_E_INVALID, "tile origin outside the frame");
  WGT_HIP(ctx, hipSetDevice(ctx->device));
  const size_t npx = (size_t)tw * th;
  wgt_tile tile{x0, y0, cam->seed, 0u};
  if ((rc = ensure(ctx, ctx->tiles, sizeof tile))) return rc;
  if (rgba8_out && (rc = ensure(ctx, ctx->out8, npx * 4))) return rc;
  if (rgba32f_out && (rc = ensure(ctx, ctx->out32, npx * 16))) return rc;
  if (hit_id_out && (rc = ensure(ctx, ctx->hit, npx * 4))) return rc;
  WGT_HIP(ctx, hipMemcpyAsync(ctx->tiles.p, &tile, sizeof tile, hipMemcpyHostToDevice, ctx->stream));
  // Pixels of a partially covered tile that fall outside the frame are not written
  // by the kernel (path_tracer.wgsl:377); give them defined contents.
  if (x0 + (uint64_t)tw > W || y0 + (uint64_t)th > H) {
    if (rgba8_out) WGT_HIP(ctx, hipMemsetAsync(ctx->out8.p, 0, npx * 4, ctx->stream));
    if (rgba32f_out) WGT_HIP(ctx, hipMemsetAsync(ctx->out32.p, 0, npx * 16, ctx->stream));
    if (hit_id_out) WGT_HIP(ctx, hipMemsetAsync(ctx->hit.p, 0xff, npx * 4, ctx->stream));
  }
  DevFrame fr = make_frame(*cam, W, H);
  fr.tw = tw;
  fr.th = th;
  fr.n_tiles = 1;
  FrameTiming timing;
  if ((rc = render_frame(ctx, fr, (const wgt_tile*)ctx->tiles.p, rgba8_out ? (uchar4*)ctx->out8.p : nullptr,
                         rgba32f_out ? (float4*)ctx->out32.p : nullptr,
                         hit_id_out ? (uint32_t*)ctx->hit.p : nullptr, nullptr, ctx->stream,
                         stats ? &timing : nullptr)))
    return rc;
  if (rgba8_out)
    WGT_HIP(ctx, hipMemcpyAsync(rgba8_out, ctx->out8.p, npx * 4, hipMemcpyDeviceToHost, ctx->stream));
  if (rgba32f_out)
    WGT_HIP(ctx, hipMemcpyAsync(rgba32f_out, ctx->out32.p, npx * 16, hipMemcpyDeviceToHost, ctx->stream));
  if (hit_id_out)
    WGT_HIP(ctx, hipMemcpyAsync(hit_id_out, ctx->hit.p, npx * 4, hipMemcpyDeviceToHost, ctx->stream));
  WGT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (stats) {
    rc = wgt_render_tiles_stats(ctx, cam, W, H, tw, th, (const wgt_tile*)ctx->tiles.p, 1, stats);
    if (rc) return rc;
    stats->kernel_ms = timing.total_ms;
    stats->trace_ms = timing.total_ms;
    stats->iterations = 1;
  }
  return WGT_OK;
}

int wgt_trace_rays_async(wgt_ctx* ctx, const float* d_rays, uint32_t n, uint32_t* d_prim_id,
                         float* d_dist, void* stream) {
  if (!ctx) return fail(nullptr, WGT_E_INVALID, "null context");
  if (!ctx->has_scene) return fail(ctx, WGT_E_NOSCENE, "no scene uploaded");
  if (n == 0) return WGT_OK;
  if (!d_rays || !d_prim_id || !d_dist) return fail(ctx, WGT_E_INVALID, "null buffer");
  WGT_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  int rc;
  if ((rc = use_begin(ctx, s))) return rc;
  WGT_HIP(ctx, launch_trace(ctx->sc, d_rays, n, d_prim_id, d_dist, s));
  return use_end(ctx, s);
}

int wgt_selftest_math(wgt_ctx* ctx, uint32_t n, uint32_t seed, uint64_t counts[8]) {
  if (!ctx) return fail(nullptr, WGT_E_INVALID, "null context");
  if (!counts) return fail(ctx, WGT_E_INVALID, "null counts");
  WGT_HIP(ctx, hipSetDevice(ctx->device));
  int rc;
  if ((rc = ensure(ctx, ctx->prim, 64))) return rc;
  WGT_HIP(ctx, hipMemsetAsync(ctx->prim.p, 0, 64, ctx->stream));
  WGT_HIP(ctx, launch_selftest_math(n, seed, (unsigned long long*)ctx->prim.p, ctx->stream));
  WGT_HIP(ctx, hipMemcpyAsync(counts, ctx->prim.p, 64, hipMemcpyDeviceToHost, ctx->stream));
  WGT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  counts[0] = 1ull << 32;  // sqrt: every bit pattern
  // n quad-distance quotients, n Moller-Trumbore reciprocals, and every pattern 1e-30 <= |x| <= 2^34
  // of the traversal's reciprocal
  uint32_t lo, hi;
  const float flo = 1e-30f, fhi = 0x1p34f;
  std::memcpy(&lo, &flo, 4);
  std::memcpy(&hi, &fhi, 4);
  counts[2] = 2ull * n + 2ull * (hi - lo + 1u);
  return WGT_OK;
}

int wgt_trace_rays(wgt_ctx* ctx, const float* rays, uint32_t n, uint32_t* prim_id, float* dist) {
  if (!ctx) return fail(nullptr, WGT_E_INVALID, "null context");
  if (!ctx->has_scene) return fail(ctx, WGT_E_NOSCENE, "no scene uploaded");
  if (n == 0) return WGT_OK;
  if (!rays || !prim_id || !dist) return fail(ctx, WGT_E_INVALID, "null buffer");
  WGT_HIP(ctx, hipSetDevice(ctx->device));
  int rc;
  if ((rc = ensure(ctx, ctx->rays, (size_t)n * 24))) return rc;
  if ((rc = ensure(ctx, ctx->prim, (size_t)n * 4))) return rc;
  if ((rc = ensure(ctx, ctx->dist, (size_t)n * 4))) return rc;
  WGT_HIP(ctx, hipMemcpyAsync(ctx->rays.p, rays, (size_t)n * 24, hipMemcpyHostToDevice, ctx->stream));
  if ((rc = use_begin(ctx, ctx->stream))) return rc;
  WGT_HIP(ctx, launch_trace(ctx->sc, (const float*)ctx->rays.p, n, (uint32_t*)ctx->prim.p,
                            (float*)ctx->dist.p, ctx->stream));
  if ((rc = use_end(ctx, ctx->stream))) return rc;
  WGT_HIP(ctx, hipMemcpyAsync(prim_id, ctx->prim.p, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
  WGT_HIP(ctx, hipMemcpyAsync(dist, ctx->dist.p, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
  WGT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return WGT_OK;
}

}  // extern "C"
