/*
 * wgt_api.h — C-ABI of the MI355X-native path-tracing hot path (libwgt.so).
 *
 * This is the drop-in boundary that replaces the WebGPU compute dispatch of the
 * reference (kugimasa/WebGPUTracer):
 *
 *   reference                                         replaced by
 *   ----------------------------------------------    -------------------------------
 *   Renderer::InitDevice  render.cpp:49-147           wgt_create
 *   Scene::InitBuffers    scene.cpp:161-165           wgt_upload_scene (+ BVH build)
 *     CreateQuadBuffer    scene.cpp:223-271             same 96-B quad records
 *     CreateSphereBuffer  scene.cpp:276-306             same 32-B sphere records
 *     CreateTriangleBuffer scene.cpp:170-218            same 80-B triangle records
 *   Camera::Update        camera.cpp:64-70            wgt_camera_param (48 B, same layout)
 *   OnRender compute pass render.cpp:461-491          wgt_render_tile / wgt_render_tiles_async
 *     dispatchWorkgroups  render.cpp:477-484            one HIP launch
 *   saveTexture readback  save_texture.h:10-87        rgba8 output (+ wgt_write_png)
 *   Scene::Release / OnFinish scene.cpp:41-50         wgt_destroy
 *   Error(...) / callbacks render.cpp:120-133         int status + wgt_last_error
 *   sample_hit            path_tracer.wgsl:290-310    wgt_trace_rays (closest-hit query)
 *
 * Conventions: every call returns 0 on success or a negative WGT_E_* code; the
 * message is available from wgt_last_error(ctx) (per-context, or thread-local
 * for calls without a context).  No exceptions cross the ABI.  Host arrays are
 * borrowed for the duration of the call.  "_async" entry points take device
 * pointers and a hipStream_t passed as void* (NULL = the context's stream) and
 * return immediately; everything else is synchronous.  All structs are POD,
 * little-endian, with exactly the reference GPU buffer layouts.
 */
#ifndef WGT_API_H
#define WGT_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WGT_API_VERSION 2  /* 2: the 64-B and wide node forms removed (scene info fields) */

enum {
  WGT_OK = 0,
  WGT_E_INVALID = -1,  /* bad argument / shape */
  WGT_E_HIP = -2,      /* a HIP runtime call failed */
  WGT_E_NOSCENE = -3,  /* render before wgt_upload_scene */
  WGT_E_IO = -4,       /* file could not be read/written/parsed */
  WGT_E_NOMEM = -5     /* host or device allocation failed */
};

/* 96 B — path_tracer.wgsl:50-59 <-> Scene::CreateQuadBuffer scene.cpp:223-271 */
typedef struct {
  float pos[4];   /* q.xyz, 1.0 */
  float right[4]; /* right.xyz, 1.0 */
  float up[4];    /* up.xyz, 1.0 */
  float norm[4];  /* normalize(cross(right, up)).xyz, 1.0 */
  float w[3];     /* n / dot(n, n) */
  float d;        /* dot(norm, q) */
  float col[3];
  float emissive; /* 1.0 or 0.0 */
} wgt_quad;

/* 32 B — path_tracer.wgsl:61-66 <-> Scene::CreateSphereBuffer scene.cpp:276-306 */
typedef struct {
  float center[3];
  float radius;
  float col[3];
  float emissive;
} wgt_sphere;

/* 80 B — Scene::CreateTriangleBuffer scene.cpp:170-218 (tri_stride_ = 80, scene.h:45) */
typedef struct {
  float v0[4];        /* v0.xyz, 1.0 */
  float e1[4];        /* v1 - v0, 1.0 */
  float e2[4];        /* v2 - v0, 1.0 */
  float face_norm[4]; /* normalize(cross(e1, e2)), 1.0 */
  float col[3];
  float emissive;
} wgt_triangle;

/* 48 B — Camera::CameraParam camera.h:19-31 <-> path_tracer.wgsl:17-24 */
typedef struct {
  float origin[3];
  float pad0;
  float target[3];
  float pad1;
  float aspect;
  float fovy; /* degrees */
  uint32_t spp;
  uint32_t seed;
} wgt_camera_param;

/* One tile of a frame for the tile-list launch.  The camera seed is per tile so
 * one launch can cover tiles of several frames (seed = frame index). */
typedef struct {
  uint32_t x0, y0; /* tile origin in global pixel coordinates */
  uint32_t seed;   /* camera.seed for this tile's frame */
  uint32_t frame;  /* caller's frame tag (not used by the kernel) */
} wgt_tile;

/* Counters from a render (filled when a stats pointer is given; counting runs a
 * separate instrumented launch so the timed launch carries no atomics). */
typedef struct {
  uint64_t queries;      /* reference sample_hit calls (path_tracer.wgsl:266), incl. skipped */
  uint64_t traced_rays;  /* closest-hit queries actually traced (non-NaN rays) */
  uint64_t samples;      /* camera paths */
  uint64_t nan_rays;     /* queries on NaN rays (resolved without tracing) */
  uint64_t node_visits;  /* BVH nodes fetched */
  uint64_t tri_tests;    /* Moller-Trumbore tests */
  uint64_t pixels;
  /* SIMT efficiency: iterations of the per-lane path loop / BVH loop counted once
   * per wave (wave_*) and once per active lane (lane_*); lane/(64*wave) = utilisation */
  uint64_t loop_wave_iters, loop_lane_iters, trav_wave_steps, trav_lane_steps;
  /* phase-split kernel: wave cycles (s_memtime) in the service / traversal phase */
  uint64_t cyc_service, cyc_trav;
  float kernel_ms;       /* hipEvent time of the (uninstrumented) render launch of the frame */
  float trace_ms;        /* = kernel_ms (one launch traces and shades; kept for the layout) */
  float shade_ms;        /* 0 (kept for the layout) */
  uint32_t iterations;   /* launches per frame: 1 */
  /* phase-split kernel: wave cycles of the service phase by region: pixel refill +
   * writes, finalise (quad rebuild, triangle merge, spheres), shading, camera ray +
   * NaN handling, quad scan, root-node test */
  uint64_t cyc_refill, cyc_finalise, cyc_shade, cyc_camera, cyc_quads, cyc_root;
  /* persistent kernel with parked traversal state: LDS stack overflows moved to the
   * lane's global stack, and refills from it */
  uint64_t stack_spills, stack_refills;
  /* ... and traversals ended on the global stack's overflow exit (a wrong pixel; never taken:
   * the global stack holds the builder's bound, and the parity tests assert 0) */
  uint64_t stack_overflows;
  /* traversal phase by BVH level: lane visits of nodes at levels 1-2 (the root is
   * tested in the service phase), wave cycles of node steps, of the node steps whose visiting lanes
   * are all at levels 1-2 (what an LDS copy of the top levels could shorten), and of triangle steps */
  uint64_t top_node_visits, cyc_node_steps, cyc_top_steps, cyc_tri_steps;
  /* rays whose quad scan took the reference path with per-quad distances (an almost-tie in
   * distance between two quads) */
  uint64_t quad_ref_scans;
} wgt_stats;

typedef struct {
  uint32_t n_lights, n_quads, n_spheres, n_tris;
  uint32_t bvh_nodes, bvh_leaves, bvh_max_depth, bvh_max_leaf; /* the traversed (BVH4) tree */
  uint64_t device_bytes; /* scene bytes resident in HBM */
  double sah_cost;       /* of the SAH BVH2 the BVH4 is collapsed from */
  uint32_t bvh_width;    /* children per node (4) */
  uint32_t bvh_stack;    /* worst-case traversal stack entries per ray (LDS) */
  uint32_t bvh2_nodes, bvh2_depth;
  uint32_t bvh_compact;   /* 1: the tree exceeds one XCD's L2 as 128-B nodes, so the persistent
                           * kernel reads its compact form (64-B nodes + 16-B refs) by default */
  float bvh_compact_step; /* scene-wide decode step of the compact nodes (wgt_geom.h) */
  uint32_t ps_waves;      /* waves per SIMD of the persistent kernel: 6 with 3-byte stack entries
                           * when every ref of the tree fits 24 bits, else 5 */
  uint32_t ps_park;       /* 1: the persistent kernel parks its traversal state in LDS during
                           * service passes */
  uint32_t ps_stack;      /* stack entries per lane it keeps in LDS (the rest: a global stack) */
  uint32_t node_form;     /* node form of the persistent kernel for the reference camera: 0 = 128-B,
                           * 1 = 80-B compact (WGT_CNODE) */
  uint32_t ps_resident;   /* waves of the persistent grid (the device's resident capacity) */
} wgt_scene_info;

typedef struct wgt_ctx wgt_ctx;

/* ---- lifecycle ---------------------------------------------------------- */
int wgt_create(int hip_device, wgt_ctx **out);
void wgt_destroy(wgt_ctx *ctx); /* idempotent for NULL */
const char *wgt_last_error(const wgt_ctx *ctx); /* ctx may be NULL */
int wgt_version(void);
/* 16 hex digits identifying the kernel build (a hash of the HIP sources, the headers
 * they include and the compile flags): profiles key their counters by it (bench.py) */
const char *wgt_build_id(void);
int wgt_device_count(int *count);

/* ---- scene upload (replaces Scene::InitBuffers) ------------------------- */
/* n_lights >= 1 (sample_from_light reads lights[0], path_tracer.wgsl:165) and
 * n_spheres >= 1 (the reference always binds a dummy sphere, scene.cpp:31).
 * Triangles (n_tris may be 0) get a SAH BVH built on the host and uploaded as
 * SoA node/triangle arrays. */
int wgt_upload_scene(wgt_ctx *ctx, const wgt_quad *lights, uint32_t n_lights,
                     const wgt_quad *quads, uint32_t n_quads, const wgt_sphere *spheres,
                     uint32_t n_spheres, const wgt_triangle *tris, uint32_t n_tris);
int wgt_scene_info_get(const wgt_ctx *ctx, wgt_scene_info *info);
/* Host only (no device): build the BVH exactly as wgt_upload_scene does and
 * export it for inspection.  info gets the counts; nodes_out (may be NULL) gets
 * bvh_nodes x 32 floats (BVH4 layout, wgt_geom.h) if nodes_cap >= bvh_nodes;
 * tris_out (may be NULL) gets n_tris x 16 floats (leaf-ordered records).
 * Call once with NULL outputs to size them. */
int wgt_bvh_build(const wgt_triangle *tris, uint32_t n_tris, float *nodes_out, uint32_t nodes_cap,
                  float *tris_out, wgt_scene_info *info);
/* Host only: the compact form of the same tree (wgt_geom.h): cnodes_out gets
 * bvh_nodes x 16 words, crefs_out bvh_nodes x 4 child refs, step_out the decode
 * step.  Both outputs are required; nodes_cap must be >= bvh_nodes. */
int wgt_bvh_build_compact(const wgt_triangle *tris, uint32_t n_tris, uint32_t *cnodes_out,
                          int32_t *crefs_out, uint32_t nodes_cap, float *step_out);

/* ---- rendering (replaces the compute pass of Renderer::OnRender) --------- */
/* Synchronous: render the rectangle [x0,x0+tw) x [y0,y0+th) of a W x H frame
 * into caller-owned HOST buffers (row-major tw x th; any may be NULL):
 * rgba8_out (4 B/px, rgba8unorm store), rgba32f_out (16 B/px, radiance before
 * quantisation), hit_id_out (primitive id of sample 0's primary ray).
 * Pixel (x, y) is computed exactly as invocation (x, y) of compute_sample
 * (path_tracer.wgsl:374-398), so any tiling reproduces the full frame. */
int wgt_render_tile(wgt_ctx *ctx, const wgt_camera_param *cam, uint32_t W, uint32_t H,
                    uint32_t x0, uint32_t y0, uint32_t tw, uint32_t th, uint8_t *rgba8_out,
                    float *rgba32f_out, uint32_t *hit_id_out, wgt_stats *stats);

/* Synchronous multi-frame render (replaces Renderer::OnCompute's frame loop,
 * render.cpp:430-449, for a static scene): n_frames whole W x H frames, frame j
 * with seed seeds[j], in ONE launch (the persistent kernel's end-of-launch drain
 * is paid once per batch).  rgba8_out: n_frames x H x W x 4 bytes, frame after
 * frame.  Frame j equals wgt_render_tile of the full frame with cam->seed =
 * seeds[j], bit for bit. */
int wgt_render_frames(wgt_ctx *ctx, const wgt_camera_param *cam, uint32_t W, uint32_t H,
                      const uint32_t *seeds, uint32_t n_frames, uint8_t *rgba8_out, wgt_stats *stats);

/* Tile-list launch with DEVICE buffers: n_tiles tiles of tw x th (d_tiles: device
 * array of wgt_tile) written compactly, tile after tile (out[(t*th + ly)*tw + lx]).
 * cam->seed is ignored (per-tile seeds).  Always asynchronous: the call returns
 * as soon as the launches are queued, ordered on `stream`; read the outputs only
 * after synchronising `stream`.  The context's launches use its scheduling
 * workspaces round-robin (4 by default, WGT_WS_SLOTS = 1..4), and a launch waits
 * on the device only for the previous launch that used the same workspace: two
 * consecutive calls on different streams may run concurrently (the next frame's
 * waves fill the CUs the previous frame's end-of-launch drain leaves idle), so the
 * caller gives such calls distinct output buffers.  wgt_upload_scene
 * and wgt_destroy wait for every launch of the context before freeing what it
 * reads. */
int wgt_render_tiles_async(wgt_ctx *ctx, const wgt_camera_param *cam, uint32_t W, uint32_t H,
                           uint32_t tw, uint32_t th, const wgt_tile *d_tiles, uint32_t n_tiles,
                           void *d_rgba8, float *d_rgba32f, uint32_t *d_hit_id, void *stream);
/* Timing pass for the same launch: uninstrumented kernels with a hipEvent pair per
 * launch; fills kernel_ms / trace_ms / shade_ms / iterations (synchronous). */
int wgt_render_tiles_profile(wgt_ctx *ctx, const wgt_camera_param *cam, uint32_t W, uint32_t H,
                             uint32_t tw, uint32_t th, const wgt_tile *d_tiles, uint32_t n_tiles,
                             wgt_stats *stats);
/* Counting pass for the same launch (instrumented kernel; synchronous). */
int wgt_render_tiles_stats(wgt_ctx *ctx, const wgt_camera_param *cam, uint32_t W, uint32_t H,
                           uint32_t tw, uint32_t th, const wgt_tile *d_tiles, uint32_t n_tiles,
                           wgt_stats *stats);

/* ---- closest-hit queries (sample_hit, path_tracer.wgsl:290-310) ---------- */
/* Rays as SoA host arrays ox,oy,oz,dx,dy,dz (each n floats, packed in that order
 * in `rays`, i.e. rays[k*n + i]).  Writes prim id (lights, quads, triangles,
 * spheres numbered consecutively; 0xffffffff = miss) and hit distance. */
int wgt_trace_rays(wgt_ctx *ctx, const float *rays, uint32_t n, uint32_t *prim_id, float *dist);
int wgt_trace_rays_async(wgt_ctx *ctx, const float *d_rays, uint32_t n, uint32_t *d_prim_id,
                         float *d_dist, void *stream);

int wgt_sync(wgt_ctx *ctx);
/* Diagnostics: the kernels' short sqrt / division forms (wgt_math.h sqrt_rn,
 * sqrt_fast, div_rn) against correctly rounded results (the f64 operation rounded
 * to f32): sqrt_rn on all 2^32 inputs, sqrt_fast on every input of its domain,
 * div_rn on n pseudo-random operand pairs of the quad distance under the render
 * limits (accept decision and accepted bits) and on n Moller-Trumbore reciprocals
 * 1/det (bits).  counts[0..7] = sqrt tests (2^32),
 * sqrt_rn mismatches, div tests (2n), div_rn mismatches, sqrt_fast tests,
 * sqrt_fast mismatches, and the mismatches of the compiler's own f32 sqrt and
 * division on the same inputs (synchronous). */
int wgt_selftest_math(wgt_ctx *ctx, uint32_t n, uint32_t seed, uint64_t counts[8]);

/* The context's HIP stream (hipStream_t) for callers that share it. */
void *wgt_stream(wgt_ctx *ctx);
/* Stream i (0..3) of the context's pipeline streams, created on first use with a
 * full CU mask so that each has a hardware queue of its own: frames issued
 * round-robin on them overlap (wgt_render_tiles_async).  NULL on error. */
void *wgt_pipeline_stream(wgt_ctx *ctx, uint32_t i);

/* ---- host-side scene helpers (no GPU needed) ----------------------------- */
/* Scene::Scene (scene.cpp:14-36): the reference Cornell box, 1 light, 17 quads,
 * 1 dummy sphere.  Capacities in *n_*; returns counts in *n_*. */
int wgt_scene_cornell(wgt_quad *lights, uint32_t *n_lights, wgt_quad *quads, uint32_t *n_quads,
                      wgt_sphere *spheres, uint32_t *n_spheres);
/* Triangle ctor (triangle.cpp:3-16): verts = n x 9 floats (v0, v1, v2). */
int wgt_make_triangles(const float *verts, uint32_t n, const float col[3], int emissive,
                       const float translation[3], wgt_triangle *out);
/* Scene::LoadObj (scene.cpp:56-131): OBJ -> triangles (fan-triangulated faces).
 * Call with out=NULL to get the count, then with a buffer of that capacity. */
int wgt_load_obj(const char *path, const float col[3], const float translation[3], int emissive,
                 wgt_triangle *out, uint32_t *n_inout);
/* Procedural stand-in meshes for absent assets: kind 0 = "bunny"
 * (displaced closed blob, ~target tris), kind 1 = "sponza" (colonnade/arch
 * architecture, ~target tris), placed inside the Cornell box. */
int wgt_procedural_mesh(int kind, uint32_t target_tris, uint32_t seed, wgt_triangle *out,
                        uint32_t *n_inout);
int wgt_write_obj(const char *path, const wgt_triangle *tris, uint32_t n);
int wgt_write_png(const char *path, const uint8_t *rgba8, uint32_t w, uint32_t h);

#ifdef __cplusplus
}
#endif
#endif /* WGT_API_H */
