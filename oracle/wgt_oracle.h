/*
 * wgt_oracle.h — TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of the reference hot path `resources/shader/path_tracer.wgsl`
 * (kugimasa/WebGPUTracer) plus the host-side scene construction it consumes
 * (`src/scene.cpp`, `src/objects/` sources, `src/camera.cpp`).  Only `tests/`,
 * `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may load it.
 *
 * PARITY STATUS: UNPINNED by the reference.  The reference ships no tests,
 * golden images or known-answer vectors, and its WGSL cannot run in this
 * image (no Dawn / wgpu-native / tint / naga).  The restatement is pinned by
 * (a) analytic known-answer tests, (b) a second, independent numpy
 * restatement in tests/, and (c) fixtures it generated itself
 * (tests/golden/, regression only).  See DESIGN.md §3.
 *
 * Byte layouts are exactly the reference's GPU buffers.
 */
#ifndef WGT_ORACLE_H
#define WGT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 96 B — scene.cpp:223-271, path_tracer.wgsl:50-59 */
typedef struct {
  float pos[4], right[4], up[4], norm[4];
  float w[3], d;
  float col[3], emissive;
} o_quad;

/* 32 B — scene.cpp:276-306, path_tracer.wgsl:61-66 */
typedef struct {
  float center[3], radius;
  float col[3], emissive;
} o_sphere;

/* 80 B — scene.cpp:170-218 (CreateTriangleBuffer; unused by the reference shader) */
typedef struct {
  float v0[4], e1[4], e2[4], fn[4];
  float col[3], emissive;
} o_tri;

/* 48 B — camera.h:19-31, path_tracer.wgsl:17-24 */
typedef struct {
  float origin[3], pad0;
  float target[3], pad1;
  float aspect, fovy;
  uint32_t spp, seed;
} o_camera;

/* counters written by o_render (index meaning) */
enum {
  O_CNT_QUERIES = 0, /* sample_hit calls, path_tracer.wgsl:266 (all of them) */
  O_CNT_TRACED = 1,  /* sample_hit calls whose ray has no NaN component     */
  O_CNT_SAMPLES = 2, /* camera samples (paths) started                       */
  O_CNT_NAN_RAYS = 3,/* sample_hit calls on NaN rays                         */
  O_CNT_N = 8
};

/* ---- numerics contract ---- */
float o_sin(float x);
float o_cos(float x);
float o_tan(float x);
float o_radians(float deg);
/* n values of rand() starting from `seed` (path_tracer.wgsl:90-95); returns final seed */
uint32_t o_rand_seq(uint32_t seed, int n, float *out);

/* ---- host scene restatement ---- */
/* Scene::Scene (scene.cpp:14-36): fills 1 light, 17 quads, 1 sphere. */
void o_cornell_scene(o_quad *lights, int *n_lights, o_quad *quads, int *n_quads,
                     o_sphere *spheres, int *n_spheres);
/* Quad ctor (quad.cpp:3-13), optionally RotateY (quad.cpp:15-25) + Translate (quad.cpp:27-35) */
void o_make_quad(const float q[3], const float right[3], const float up[3],
                 const float col[3], int emissive, o_quad *out);
/* Triangle ctor (triangle.cpp:3-16) packed like CreateTriangleBuffer (scene.cpp:182-215) */
void o_make_triangle(const float v0[3], const float v1[3], const float v2[3],
                     const float col[3], int emissive, o_tri *out);
/* Camera::Update (camera.cpp:64-70) with an explicit seed instead of RandSeed() */
void o_camera_param(float aspect, uint32_t spp, uint32_t seed, o_camera *out);

/* ---- scene handle (owns an oracle-side BVH over the triangles) ---- */
typedef struct o_scene o_scene;
o_scene *o_scene_create(const o_quad *lights, int n_lights, const o_quad *quads, int n_quads,
                        const o_sphere *spheres, int n_spheres, const o_tri *tris, int n_tris);
void o_scene_destroy(o_scene *s);

/* Closest-hit query = sample_hit (path_tracer.wgsl:290-310) extended with triangles.
 * prim id: lights [0,nL) quads [nL,nL+nQ) tris [..+nT) spheres [..+nS); 0xffffffff = no hit.
 * brute != 0: linear scan over all triangles (the triangle SPEC); else oracle BVH. */
void o_trace(const o_scene *s, int n, const float *start, const float *dir,
             uint32_t *prim_id, float *dist, int brute);

/* Triangle-only closest hit (min (t, index) among valid triangles).
 * Writes index or 0xffffffff and t. */
void o_trace_tris(const o_scene *s, int n, const float *start, const float *dir,
                  uint32_t *tri_id, float *t, int brute);

/* compute_sample (path_tracer.wgsl:374-398) for the tile [x0,x0+tw)x[y0,y0+th) of a
 * W x H frame.  Any output may be NULL.  rgba32f: pre-quantisation radiance
 * (col, 1.0); rgba8: rgba8unorm store; hit_id: prim id of sample 0's primary ray.
 * counters: O_CNT_N uint64.  nthreads<=0: OpenMP default. */
int o_render(const o_scene *s, const o_camera *cam, uint32_t W, uint32_t H,
             uint32_t x0, uint32_t y0, uint32_t tw, uint32_t th,
             float *rgba32f, uint8_t *rgba8, uint32_t *hit_id, uint64_t *counters,
             int nthreads);

#ifdef __cplusplus
}
#endif
#endif
