/*
 * wgt_oracle.c — TEST INFRASTRUCTURE ONLY.  The parity checker for the HIP path;
 * never linked into, called by, or shipped with the product (webgputracer_amd/).
 * Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 *
 * A literal, scalar C99 restatement of the reference hot path
 *   resources/shader/path_tracer.wgsl:1-398   (kugimasa/WebGPUTracer)
 * and of the host code that builds its inputs
 *   src/scene.cpp:14-36, 170-306, src/objects/{quad,box,cornell_box,triangle}.cpp,
 *   src/camera.cpp:64-70, src/include/utils/color_util.h:5-10
 * with glm's arithmetic (cross/dot/normalize/rotate/translate, mat4*vec4) restated
 * operation by operation.
 *
 * PARITY STATUS: **parity unpinned** by the reference — it has no tests, fixtures
 * or golden vectors and its WGSL cannot execute in this image.
 * Pinned instead by analytic KATs + an independent numpy restatement (tests/).
 *
 * Numerics contract (WGSL leaves these open):
 *   IEEE fp32, no contraction (-ffp-contract=off), correctly rounded / and sqrt,
 *   left-to-right evaluation (dot = (x*x + y*y) + z*z), normalize(v) = v / length(v),
 *   sin/cos/tan = the Cody-Waite + polynomial functions below, radians(x) = x*0.017453292,
 *   max(NaN, 0) = 0, rgba8 = floor(clamp(c,0,1)*255 + 0.5).
 *
 * Triangles/BVH are NEW semantics (the reference shader has none):
 * the triangle hit is min (t, index) over triangles that pass Moller-Trumbore and
 * whose own padded box contains t.  o_trace(..., brute=1) is that
 * spec by linear scan; the oracle's own median-split BVH must (and is tested to)
 * return the identical answer.
 */
#include "wgt_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ constants */
/* path_tracer.wgsl:1-10 (abstract-float literals rounded to f32) */
#define kPI 3.14159265359f
#define k_1_PI 0.318309886184f
#define kNoHit 0xffffffffu
#define kRayDepth 50
#define kRayMin 0.001f
#define kRayMax 1e20f

typedef struct { float x, y, z; } v3;

static inline v3 V(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
static inline v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vscale(float s, v3 a) { return V(s * a.x, s * a.y, s * a.z); }
static inline v3 vdivs(v3 a, float s) { return V(a.x / s, a.y / s, a.z / s); }
static inline v3 vneg(v3 a) { return V(-a.x, -a.y, -a.z); }
static inline float vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 vcross(v3 a, v3 b) {
  return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline float vlength(v3 a) { return sqrtf(vdot(a, a)); }
static inline v3 vnormalize(v3 a) { return vdivs(a, vlength(a)); }
static inline float vdistance(v3 a, v3 b) { return vlength(vsub(a, b)); }
static inline v3 vload(const float *p) { return V(p[0], p[1], p[2]); }
static inline int visnan(v3 a) { return isnan(a.x) || isnan(a.y) || isnan(a.z); }

/* path_tracer.wgsl:68-70 */
static inline float fabs_w(float x) { return x < 0.0f ? -x : x; }
/* WGSL sign() */
static inline float sign_w(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }
/* WGSL max(e, 0) with max(NaN, 0) = 0 (numerics contract) */
static inline float max0(float x) { return x > 0.0f ? x : 0.0f; }

/* -------------------------------------------- deterministic transcendentals */
/* Cody-Waite reduction by pi/2 (17 + 24 bit split) and fdlibm-style minimax
 * polynomials on [-pi/4, pi/4].  Only +,-,*,floor,compare: bit-identical on
 * x86 and gfx950 given no contraction. */
#define O_2_OVER_PI 0.636619772367581343f
#define O_PIO2_HI 1.5707855225e+00f /* 0x3fc90f80 */
#define O_PIO2_LO 1.0804334124e-05f /* 0x37354443 */
#define O_S1 -1.6666667163e-01f
#define O_S2 8.3333337680e-03f
#define O_S3 -1.9841270114e-04f
#define O_S4 2.7557314297e-06f
#define O_C1 4.1666667908e-02f
#define O_C2 -1.3888889225e-03f
#define O_C3 2.4801587642e-05f
#define O_C4 -2.7557314297e-07f

static inline float o_reduce(float x, float *q) {
  float k = floorf(x * O_2_OVER_PI + 0.5f);
  *q = k - 4.0f * floorf(k * 0.25f);
  return (x - k * O_PIO2_HI) - k * O_PIO2_LO;
}
static inline float o_ksin(float r) {
  float z = r * r;
  return r + (r * z) * (O_S1 + z * (O_S2 + z * (O_S3 + z * O_S4)));
}
static inline float o_kcos(float r) {
  float z = r * r;
  return (1.0f - 0.5f * z) + (z * z) * (O_C1 + z * (O_C2 + z * (O_C3 + z * O_C4)));
}
float o_sin(float x) {
  float q, r = o_reduce(x, &q);
  if (q == 0.0f) return o_ksin(r);
  if (q == 1.0f) return o_kcos(r);
  if (q == 2.0f) return -o_ksin(r);
  return -o_kcos(r);
}
float o_cos(float x) {
  float q, r = o_reduce(x, &q);
  if (q == 0.0f) return o_kcos(r);
  if (q == 1.0f) return -o_ksin(r);
  if (q == 2.0f) return -o_kcos(r);
  return o_ksin(r);
}
float o_tan(float x) { return o_sin(x) / o_cos(x); }
float o_radians(float deg) { return deg * 0.017453292519943295f; }

/* ------------------------------------------------------------------- rand() */
/* path_tracer.wgsl:88-95 (PCG-hash; bitcast<f32>(0x2f800004u)) */
static float rand_scale(void) {
  uint32_t b = 0x2f800004u;
  float f;
  memcpy(&f, &b, 4);
  return f;
}
static inline float rnd(uint32_t *seed) {
  uint32_t s = *seed * 747796405u + 2891336453u;
  *seed = s;
  uint32_t word = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
  return (float)((word >> 22u) ^ word) * rand_scale();
}
uint32_t o_rand_seq(uint32_t seed, int n, float *out) {
  for (int i = 0; i < n; ++i) out[i] = rnd(&seed);
  return seed;
}

/* ------------------------------------------------ glm restatement (host side) */
/* glm 0.9.9 semantics used by quad.cpp / box.cpp: column-major mat4. */
typedef struct { float c[4][4]; } m4; /* c[col][row] */
typedef struct { float x, y, z, w; } v4;

static v4 v4scale(v4 a, float s) { v4 r = {a.x * s, a.y * s, a.z * s, a.w * s}; return r; }
static v4 v4add(v4 a, v4 b) { v4 r = {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; return r; }
static v4 m4col(const m4 *m, int i) { v4 r = {m->c[i][0], m->c[i][1], m->c[i][2], m->c[i][3]}; return r; }
static void m4setcol(m4 *m, int i, v4 v) { m->c[i][0] = v.x; m->c[i][1] = v.y; m->c[i][2] = v.z; m->c[i][3] = v.w; }
static m4 m4identity(void) {
  m4 m;
  memset(&m, 0, sizeof m);
  for (int i = 0; i < 4; ++i) m.c[i][i] = 1.0f;
  return m;
}
/* glm operator*(mat4, vec4): (m0*x + m1*y) + (m2*z + m3*w) */
static v4 m4mulv(const m4 *m, v4 v) {
  v4 add0 = v4add(v4scale(m4col(m, 0), v.x), v4scale(m4col(m, 1), v.y));
  v4 add1 = v4add(v4scale(m4col(m, 2), v.z), v4scale(m4col(m, 3), v.w));
  return v4add(add0, add1);
}
/* glm dot (vec3): tmp = a*b; (tmp.x + tmp.y) + tmp.z */
static float gdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
/* glm cross */
static v3 gcross(v3 x, v3 y) {
  return V(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
/* glm normalize: x * inversesqrt(dot(x,x)), inversesqrt = 1/sqrt */
static v3 gnormalize(v3 x) {
  float inv = 1.0f / sqrtf(gdot(x, x));
  return V(x.x * inv, x.y * inv, x.z * inv);
}
/* glm::rotate(m, angle, v) (matrix_transform.inl) */
static m4 grotate(const m4 *m, float angle, v3 v) {
  float a = angle;
  float c = cosf(a);
  float s = sinf(a);
  v3 axis = gnormalize(v);
  float omc = 1.0f - c;
  v3 temp = V(omc * axis.x, omc * axis.y, omc * axis.z);
  float R[3][3];
  R[0][0] = c + temp.x * axis.x;
  R[0][1] = temp.x * axis.y + s * axis.z;
  R[0][2] = temp.x * axis.z - s * axis.y;
  R[1][0] = temp.y * axis.x - s * axis.z;
  R[1][1] = c + temp.y * axis.y;
  R[1][2] = temp.y * axis.z + s * axis.x;
  R[2][0] = temp.z * axis.x + s * axis.y;
  R[2][1] = temp.z * axis.y - s * axis.x;
  R[2][2] = c + temp.z * axis.z;
  m4 out;
  for (int i = 0; i < 3; ++i) {
    v4 r = v4add(v4add(v4scale(m4col(m, 0), R[i][0]), v4scale(m4col(m, 1), R[i][1])),
                 v4scale(m4col(m, 2), R[i][2]));
    m4setcol(&out, i, r);
  }
  m4setcol(&out, 3, m4col(m, 3));
  return out;
}
/* glm::translate(m, v): Result[3] = m[0]*v[0] + m[1]*v[1] + m[2]*v[2] + m[3] */
static m4 gtranslate(const m4 *m, v3 v) {
  m4 out = *m;
  v4 r = v4add(v4add(v4add(v4scale(m4col(m, 0), v.x), v4scale(m4col(m, 1), v.y)),
                     v4scale(m4col(m, 2), v.z)),
               m4col(m, 3));
  m4setcol(&out, 3, r);
  return out;
}
/* glm::radians(float) */
static float gradians(float deg) { return deg * (float)0.01745329251994329576923690768489; }

/* Quad host object (quad.h) */
typedef struct { v3 q, right, up, norm, w; float d; v3 col; int emissive; } hquad;

static void hquad_recalc(hquad *h) {
  v3 n = gcross(h->right, h->up);
  h->norm = gnormalize(n);
  h->d = gdot(h->norm, h->q);
  float nn = gdot(n, n);
  h->w = V(n.x / nn, n.y / nn, n.z / nn);
}
/* quad.cpp:3-13 */
static hquad hquad_make(v3 q, v3 right, v3 up, v3 col, int emissive) {
  hquad h;
  h.q = q; h.right = right; h.up = up;
  hquad_recalc(&h);
  h.col = col; h.emissive = emissive;
  return h;
}
static v3 xform_point(const m4 *m, v3 p) {
  v4 in = {p.x, p.y, p.z, 1.0f};
  v4 o = m4mulv(m, in);
  return V(o.x, o.y, o.z);
}
/* quad.cpp:15-25 — note right/up are transformed with w = 1 as in the reference */
static void hquad_rotate_y(hquad *h, float angle) {
  m4 I = m4identity();
  m4 R = grotate(&I, gradians(angle), V(0.0f, 1.0f, 0.0f));
  h->q = xform_point(&R, h->q);
  h->right = xform_point(&R, h->right);
  h->up = xform_point(&R, h->up);
  hquad_recalc(h);
}
/* quad.cpp:27-35 */
static void hquad_translate(hquad *h, v3 dir) {
  m4 I = m4identity();
  m4 T = gtranslate(&I, dir);
  h->q = xform_point(&T, h->q);
  hquad_recalc(h);
}
/* CreateQuadBuffer (scene.cpp:235-268) */
static void hquad_pack(const hquad *h, o_quad *o) {
  const float dummy = 1.0f;
  o->pos[0] = h->q.x; o->pos[1] = h->q.y; o->pos[2] = h->q.z; o->pos[3] = dummy;
  o->right[0] = h->right.x; o->right[1] = h->right.y; o->right[2] = h->right.z; o->right[3] = dummy;
  o->up[0] = h->up.x; o->up[1] = h->up.y; o->up[2] = h->up.z; o->up[3] = dummy;
  o->norm[0] = h->norm.x; o->norm[1] = h->norm.y; o->norm[2] = h->norm.z; o->norm[3] = dummy;
  o->w[0] = h->w.x; o->w[1] = h->w.y; o->w[2] = h->w.z; o->d = h->d;
  o->col[0] = h->col.x; o->col[1] = h->col.y; o->col[2] = h->col.z;
  o->emissive = h->emissive ? 1.0f : 0.0f;
}

void o_make_quad(const float q[3], const float right[3], const float up[3],
                 const float col[3], int emissive, o_quad *out) {
  hquad h = hquad_make(vload(q), vload(right), vload(up), vload(col), emissive);
  hquad_pack(&h, out);
}

/* color_util.h:5-10 (double literals narrowed to float) */
#define COL(r, g, b) V((float)(r), (float)(g), (float)(b))

/* box.cpp:3-20 */
static int hbox_make(v3 aabb_min, v3 aabb_max, v3 col, hquad out[6]) {
  v3 mn = V(fminf(aabb_min.x, aabb_max.x), fminf(aabb_min.y, aabb_max.y), fminf(aabb_min.z, aabb_max.z));
  v3 mx = V(fmaxf(aabb_min.x, aabb_max.x), fmaxf(aabb_min.y, aabb_max.y), fmaxf(aabb_min.z, aabb_max.z));
  v3 dx = V(mx.x - mn.x, 0.0f, 0.0f);
  v3 dy = V(0.0f, mx.y - mn.y, 0.0f);
  v3 dz = V(0.0f, 0.0f, mx.z - mn.z);
  out[0] = hquad_make(V(mn.x, mn.y, mx.z), dx, dy, col, 0);
  out[1] = hquad_make(V(mx.x, mn.y, mx.z), vneg(dz), dy, col, 0);
  out[2] = hquad_make(V(mx.x, mn.y, mn.z), vneg(dx), dy, col, 0);
  out[3] = hquad_make(V(mn.x, mn.y, mn.z), dz, dy, col, 0);
  out[4] = hquad_make(V(mn.x, mx.y, mx.z), dx, vneg(dz), col, 0);
  out[5] = hquad_make(V(mn.x, mn.y, mn.z), dx, dz, col, 0);
  return 6;
}

void o_cornell_scene(o_quad *lights, int *n_lights, o_quad *quads, int *n_quads,
                     o_sphere *spheres, int *n_spheres) {
  const v3 RED = COL(.65, .05, .05), GREEN = COL(.12, .45, .15), WHITE = COL(.73, .73, .73),
           LIGHT = COL(15, 15, 15), ZERO = COL(0, 0, 0);
  /* scene.cpp:16 */
  hquad L = hquad_make(V(213, 554, 227), V(130, 0, 0), V(0, 0, 105), LIGHT, 1);
  hquad_pack(&L, &lights[0]);
  *n_lights = 1;
  /* cornell_box.cpp:6-10 */
  hquad q[17];
  q[0] = hquad_make(V(555, 0, 0), V(0, 0, 555), V(0, 555, 0), GREEN, 0);
  q[1] = hquad_make(V(0, 0, 555), V(0, 0, -555), V(0, 555, 0), RED, 0);
  q[2] = hquad_make(V(0, 555, 0), V(555, 0, 0), V(0, 0, 555), WHITE, 0);
  q[3] = hquad_make(V(0, 0, 555), V(555, 0, 0), V(0, 0, -555), WHITE, 0);
  q[4] = hquad_make(V(555, 0, 555), V(-555, 0, 0), V(0, 555, 0), WHITE, 0);
  /* scene.cpp:21-28 */
  hquad b1[6], b2[6];
  hbox_make(V(0, 0, 0), V(165, 330, 165), WHITE, b1);
  for (int i = 0; i < 6; ++i) hquad_rotate_y(&b1[i], 15.0f);
  for (int i = 0; i < 6; ++i) hquad_translate(&b1[i], V(265, 0, 295));
  hbox_make(V(0, 0, 0), V(165, 165, 165), WHITE, b2);
  for (int i = 0; i < 6; ++i) hquad_rotate_y(&b2[i], -18.0f);
  for (int i = 0; i < 6; ++i) hquad_translate(&b2[i], V(130, 0, 65));
  for (int i = 0; i < 6; ++i) q[5 + i] = b1[i];
  for (int i = 0; i < 6; ++i) q[11 + i] = b2[i];
  for (int i = 0; i < 17; ++i) hquad_pack(&q[i], &quads[i]);
  *n_quads = 17;
  /* scene.cpp:31 dummy sphere; CreateSphereBuffer scene.cpp:288-302 */
  spheres[0].center[0] = 0; spheres[0].center[1] = 0; spheres[0].center[2] = 0;
  spheres[0].radius = 0;
  spheres[0].col[0] = ZERO.x; spheres[0].col[1] = ZERO.y; spheres[0].col[2] = ZERO.z;
  spheres[0].emissive = 0.0f;
  *n_spheres = 1;
}

/* triangle.cpp:3-16 + CreateTriangleBuffer scene.cpp:182-215 */
void o_make_triangle(const float v0[3], const float v1[3], const float v2[3],
                     const float col[3], int emissive, o_tri *out) {
  v3 a = vload(v0), b = vload(v1), c = vload(v2);
  v3 e1 = vsub(b, a), e2 = vsub(c, a);
  v3 fn = gnormalize(gcross(e1, e2));
  const float dummy = 1.0f;
  out->v0[0] = a.x; out->v0[1] = a.y; out->v0[2] = a.z; out->v0[3] = dummy;
  out->e1[0] = e1.x; out->e1[1] = e1.y; out->e1[2] = e1.z; out->e1[3] = dummy;
  out->e2[0] = e2.x; out->e2[1] = e2.y; out->e2[2] = e2.z; out->e2[3] = dummy;
  out->fn[0] = fn.x; out->fn[1] = fn.y; out->fn[2] = fn.z; out->fn[3] = dummy;
  out->col[0] = col[0]; out->col[1] = col[1]; out->col[2] = col[2];
  out->emissive = emissive ? 1.0f : 0.0f;
}

/* camera.cpp:64-70 (seed explicit) */
void o_camera_param(float aspect, uint32_t spp, uint32_t seed, o_camera *out) {
  memset(out, 0, sizeof *out);
  out->origin[0] = 278; out->origin[1] = 278; out->origin[2] = -800;
  out->target[0] = 278; out->target[1] = 278; out->target[2] = 0;
  out->aspect = aspect;
  out->fovy = 40.0f;
  out->spp = spp;
  out->seed = seed;
}

/* ------------------------------------------------------------ scene handle */
typedef struct { float lo[3], hi[3]; int left, right, first, count; } obvh_node;

struct o_scene {
  o_quad *lights; int nL;
  o_quad *quads; int nQ;
  o_sphere *spheres; int nS;
  o_tri *tris; int nT;
  float *tbox;       /* 6 floats per tri: padded box (spec) */
  int *tidx;         /* BVH leaf order */
  obvh_node *nodes; int n_nodes;
};

/* Triangle box spec: bounds of v0, v0+e1, v0+e2, then padded. */
static void tri_box(const o_tri *t, float lo[3], float hi[3]) {
  for (int c = 0; c < 3; ++c) {
    float a = t->v0[c];
    float b = a + t->e1[c];
    float d = a + t->e2[c];
    float l = a < b ? a : b;
    l = l < d ? l : d;
    float h = a > b ? a : b;
    h = h > d ? h : d;
    float pad = ((h - l) * 1e-4f + (fabs_w(l) + fabs_w(h)) * 1e-5f) + 1e-6f;
    lo[c] = l - pad;
    hi[c] = h + pad;
  }
}

/* Slab spec: inverse direction with |d| < 1e-30 replaced by
 * copysign(1e-30, d); per plane t = fma(b, inv, -(o*inv)). */
static inline void inv_dir(v3 d, float inv[3]) {
  float dd[3] = {d.x, d.y, d.z};
  for (int c = 0; c < 3; ++c) {
    float x = dd[c];
    if (fabs_w(x) < 1e-30f) x = copysignf(1e-30f, x);
    inv[c] = 1.0f / x;
  }
}
static inline void slab(const float ot[3], const float inv[3], const float lo[3],
                        const float hi[3], float *tnear, float *tfar) {
  float n = -INFINITY, f = INFINITY;
  int first = 1;
  for (int c = 0; c < 3; ++c) {
    float t0 = fmaf(lo[c], inv[c], ot[c]);
    float t1 = fmaf(hi[c], inv[c], ot[c]);
    float a = t0 < t1 ? t0 : t1;
    float b = t0 < t1 ? t1 : t0;
    if (first) { n = a; f = b; first = 0; }
    else { n = a > n ? a : n; f = b < f ? b : f; }
  }
  *tnear = n;
  *tfar = f;
}

/* Moller-Trumbore, two-sided */
static inline int mt_test(v3 o, v3 d, const o_tri *tr, float *tout) {
  v3 v0 = vload(tr->v0), e1 = vload(tr->e1), e2 = vload(tr->e2);
  v3 pvec = vcross(d, e2);
  float det = vdot(e1, pvec);
  if (fabs_w(det) < 1e-12f) return 0;
  float inv_det = 1.0f / det;
  v3 tvec = vsub(o, v0);
  float u = vdot(tvec, pvec) * inv_det;
  if (u < 0.0f || u > 1.0f) return 0;
  v3 qvec = vcross(tvec, e1);
  float v = vdot(d, qvec) * inv_det;
  if (v < 0.0f || u + v > 1.0f) return 0;
  float t = vdot(e2, qvec) * inv_det;
  if (t < kRayMin || kRayMax < t) return 0;
  *tout = t;
  return 1;
}

static inline void tri_candidate(const o_scene *s, int i, v3 o, v3 d, const float ot[3],
                                 const float inv[3], float *best_t, uint32_t *best_i) {
  float t;
  if (!mt_test(o, d, &s->tris[i], &t)) return;
  if (!(t < *best_t || (t == *best_t && (uint32_t)i < *best_i))) return;
  float n, f;
  slab(ot, inv, &s->tbox[6 * i], &s->tbox[6 * i + 3], &n, &f);
  if (!(n <= t && t <= f)) return;
  *best_t = t;
  *best_i = (uint32_t)i;
}

/* min (t, idx) over valid triangles */
static void tris_closest(const o_scene *s, v3 o, v3 d, int brute, float *bt, uint32_t *bi) {
  float best_t = kRayMax;
  uint32_t best_i = kNoHit;
  if (s->nT > 0) {
    float inv[3];
    inv_dir(d, inv);
    float ot[3] = {-(o.x * inv[0]), -(o.y * inv[1]), -(o.z * inv[2])};
    if (brute) {
      for (int i = 0; i < s->nT; ++i) tri_candidate(s, i, o, d, ot, inv, &best_t, &best_i);
    } else {
      int stack[128];
      int sp = 0;
      stack[sp++] = 0;
      while (sp > 0) {
        const obvh_node *nd = &s->nodes[stack[--sp]];
        float n, f;
        slab(ot, inv, nd->lo, nd->hi, &n, &f);
        if (!(n <= f && n <= best_t && f >= kRayMin)) continue;
        if (nd->count > 0) {
          for (int k = 0; k < nd->count; ++k)
            tri_candidate(s, s->tidx[nd->first + k], o, d, ot, inv, &best_t, &best_i);
        } else {
          stack[sp++] = nd->right;
          stack[sp++] = nd->left;
        }
      }
    }
  }
  *bt = best_t;
  *bi = best_i;
}

/* ---- oracle BVH: median split on the longest centroid axis, leaves <= 4 ---- */
static int cmp_axis;
static const float *cmp_cent;
static int cmp_fn(const void *a, const void *b) {
  float fa = cmp_cent[3 * *(const int *)a + cmp_axis], fb = cmp_cent[3 * *(const int *)b + cmp_axis];
  if (fa < fb) return -1;
  if (fa > fb) return 1;
  return (*(const int *)a) - (*(const int *)b);
}
static int build_rec(o_scene *s, const float *cent, int first, int count, int depth) {
  int id = s->n_nodes++;
  obvh_node *nd = &s->nodes[id];
  for (int c = 0; c < 3; ++c) { nd->lo[c] = INFINITY; nd->hi[c] = -INFINITY; }
  float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int k = first; k < first + count; ++k) {
    int i = s->tidx[k];
    for (int c = 0; c < 3; ++c) {
      nd->lo[c] = fminf(nd->lo[c], s->tbox[6 * i + c]);
      nd->hi[c] = fmaxf(nd->hi[c], s->tbox[6 * i + 3 + c]);
      clo[c] = fminf(clo[c], cent[3 * i + c]);
      chi[c] = fmaxf(chi[c], cent[3 * i + c]);
    }
  }
  if (count <= 4 || depth > 100) {
    nd->count = count; nd->first = first; nd->left = nd->right = -1;
    return id;
  }
  int axis = 0;
  float ext = chi[0] - clo[0];
  for (int c = 1; c < 3; ++c) if (chi[c] - clo[c] > ext) { ext = chi[c] - clo[c]; axis = c; }
  cmp_axis = axis; cmp_cent = cent;
  qsort(&s->tidx[first], (size_t)count, sizeof(int), cmp_fn);
  int half = count / 2;
  nd->count = 0; nd->first = -1;
  int l = build_rec(s, cent, first, half, depth + 1);
  int r = build_rec(s, cent, first + half, count - half, depth + 1);
  s->nodes[id].left = l;
  s->nodes[id].right = r;
  return id;
}

o_scene *o_scene_create(const o_quad *lights, int n_lights, const o_quad *quads, int n_quads,
                        const o_sphere *spheres, int n_spheres, const o_tri *tris, int n_tris) {
  o_scene *s = (o_scene *)calloc(1, sizeof *s);
  s->nL = n_lights; s->nQ = n_quads; s->nS = n_spheres; s->nT = n_tris;
  s->lights = (o_quad *)malloc(sizeof(o_quad) * (n_lights > 0 ? n_lights : 1));
  s->quads = (o_quad *)malloc(sizeof(o_quad) * (n_quads > 0 ? n_quads : 1));
  s->spheres = (o_sphere *)malloc(sizeof(o_sphere) * (n_spheres > 0 ? n_spheres : 1));
  s->tris = (o_tri *)malloc(sizeof(o_tri) * (n_tris > 0 ? n_tris : 1));
  if (n_lights) memcpy(s->lights, lights, sizeof(o_quad) * n_lights);
  if (n_quads) memcpy(s->quads, quads, sizeof(o_quad) * n_quads);
  if (n_spheres) memcpy(s->spheres, spheres, sizeof(o_sphere) * n_spheres);
  if (n_tris) memcpy(s->tris, tris, sizeof(o_tri) * n_tris);
  if (n_tris > 0) {
    s->tbox = (float *)malloc(sizeof(float) * 6 * n_tris);
    s->tidx = (int *)malloc(sizeof(int) * n_tris);
    float *cent = (float *)malloc(sizeof(float) * 3 * n_tris);
    for (int i = 0; i < n_tris; ++i) {
      tri_box(&s->tris[i], &s->tbox[6 * i], &s->tbox[6 * i + 3]);
      for (int c = 0; c < 3; ++c) cent[3 * i + c] = 0.5f * (s->tbox[6 * i + c] + s->tbox[6 * i + 3 + c]);
      s->tidx[i] = i;
    }
    s->nodes = (obvh_node *)malloc(sizeof(obvh_node) * 2 * n_tris);
    s->n_nodes = 0;
    build_rec(s, cent, 0, n_tris, 0);
    free(cent);
  }
  return s;
}

void o_scene_destroy(o_scene *s) {
  if (!s) return;
  free(s->lights); free(s->quads); free(s->spheres); free(s->tris);
  free(s->tbox); free(s->tidx); free(s->nodes);
  free(s);
}

/* ------------------------------------------------------------- the shader */
typedef struct { v3 start, dir; } ray;
/* path_tracer.wgsl:27-36 (+ prim id for the hit-ID parity output) */
typedef struct {
  float dist;
  int emissive, front_face;
  uint32_t shape;
  v3 pos, norm, col;
  uint32_t prim;
} hitinfo;
typedef struct { v3 u, v, w; } onb;
typedef struct { ray r; v3 col; int end; } path;

/* path_tracer.wgsl:72-74 */
static inline v3 point_at(ray r, float t) { return vadd(r.start, vscale(t, r.dir)); }

/* path_tracer.wgsl:123-131 */
static inline v3 rand_cos_dir(uint32_t *seed) {
  float r1 = rnd(seed);
  float r2 = rnd(seed);
  float z = sqrtf(1.0f - r2);
  float phi = 2.0f * kPI * r1;
  float x = o_cos(phi) * sqrtf(r2);
  float y = o_sin(phi) * sqrtf(r2);
  return V(x, y, z);
}
/* path_tracer.wgsl:133-140 */
static inline onb build_onb_from_w(v3 w) {
  onb o;
  o.w = vnormalize(w);
  v3 a = (sign_w(o.w.x) * o.w.x) > 0.9f ? V(0, 1, 0) : V(1, 0, 0);
  o.v = vnormalize(vcross(o.w, a));
  o.u = vcross(o.w, o.v);
  return o;
}
/* path_tracer.wgsl:142-144 */
static inline v3 onb_local(onb o, v3 a) {
  return vadd(vadd(vscale(a.x, o.u), vscale(a.y, o.v)), vscale(a.z, o.w));
}
/* path_tracer.wgsl:163-168 */
static inline v3 sample_from_light(const o_scene *s, const hitinfo *hit, uint32_t *seed) {
  const o_quad *L = &s->lights[0];
  float r1 = rnd(seed);
  float r2 = rnd(seed);
  v3 p = vadd(vadd(vload(L->pos), vscale(r1, vload(L->right))), vscale(r2, vload(L->up)));
  return vsub(p, hit->pos);
}
/* path_tracer.wgsl:185-189 */
static inline v3 sample_from_cosine(const hitinfo *hit, uint32_t *seed) {
  onb o = build_onb_from_w(hit->norm);
  v3 a = rand_cos_dir(seed);
  return onb_local(o, a);
}
/* path_tracer.wgsl:146-154 (+ sample_from_bxdf :170-183, bxdf = 0) */
static inline v3 sample_direction(const o_scene *s, const hitinfo *hit, uint32_t *seed) {
  if (rnd(seed) > 0.5f) return sample_from_cosine(hit, seed);
  return sample_from_light(s, hit, seed);
}
/* path_tracer.wgsl:202-209 */
static inline float light_area_pdf(const o_scene *s, v3 to_light) {
  const o_quad *L = &s->lights[0];
  float area = vlength(vcross(vload(L->right), vload(L->up)));
  float distance_squared = vlength(to_light) * vlength(to_light);
  float light_cosine = fabs_w(vnormalize(to_light).y) + kRayMin;
  return distance_squared / (light_cosine * area);
}
/* path_tracer.wgsl:211-215 */
static inline float cosine_pdf(const hitinfo *hit, v3 dir) {
  onb o = build_onb_from_w(hit->norm);
  float c = vdot(vnormalize(dir), o.w);
  return c <= 0.0f ? 0.0f : c * k_1_PI;
}
/* path_tracer.wgsl:191-193 */
static inline float mixture_pdf(const o_scene *s, const hitinfo *hit, v3 dir) {
  return 0.5f * cosine_pdf(hit, dir) + 0.5f * light_area_pdf(s, dir);
}
/* path_tracer.wgsl:217-220 */
static inline float scattering_pdf(const hitinfo *hit, v3 dir) {
  float c = vdot(hit->norm, vnormalize(dir));
  return c < 0.0f ? 0.0f : c * k_1_PI;
}

/* path_tracer.wgsl:314-338 */
static inline void intersect_quad(ray r, const o_quad *q, uint32_t id, hitinfo *closest) {
  v3 qn = vload(q->norm);
  float denom = vdot(qn, r.dir);
  if (fabs_w(denom) < kRayMin) return;
  float t = (q->d - vdot(qn, r.start)) / denom;
  if (t < kRayMin || kRayMax < t) return;
  v3 pos = point_at(r, t);
  float ray_dist = vdistance(pos, r.start);
  if (ray_dist >= closest->dist) return;
  v3 hit_vec = vsub(pos, vload(q->pos));
  v3 qw = vload(q->w);
  float a = vdot(qw, vcross(hit_vec, vload(q->up)));
  float b = vdot(qw, vcross(vload(q->right), hit_vec));
  if ((a < 0.0f) || (1.0f < a) || (b < 0.0f) || (1.0f < b)) return;
  int front_face = vdot(r.dir, qn) < 0.0f;
  closest->dist = ray_dist;
  closest->emissive = q->emissive > 0.0f;
  closest->front_face = front_face;
  closest->shape = 1u;
  closest->pos = pos;
  closest->norm = front_face ? qn : vneg(qn);
  closest->col = vload(q->col);
  closest->prim = id;
}
/* path_tracer.wgsl:340-369 (sphere_uv is dead downstream and omitted) */
static inline void intersect_sphere(ray r, const o_sphere *sp, uint32_t id, hitinfo *closest) {
  v3 center = vload(sp->center);
  v3 oc = vsub(r.start, center);
  v3 dir = r.dir;
  float a = vdot(dir, dir);
  float half_b = vdot(oc, dir);
  float c = vdot(oc, oc) - sp->radius * sp->radius;
  float discriminant = half_b * half_b - a * c;
  if (discriminant < 0.0f) return;
  float sqrt_d = sqrtf(discriminant);
  float root = (-half_b - sqrt_d) / a;
  if (root < kRayMin || kRayMax < root) {
    root = (-half_b + sqrt_d) / a;
    if (root < kRayMin || kRayMax < root) return;
  }
  v3 pos = point_at(r, root);
  float ray_dist = vdistance(pos, r.start);
  if (ray_dist >= closest->dist) return;
  v3 sphere_norm = vdivs(vsub(pos, center), sp->radius);
  int front_face = vdot(r.dir, sphere_norm) < 0.0f;
  closest->dist = ray_dist;
  closest->emissive = sp->emissive > 0.0f;
  closest->front_face = front_face;
  closest->shape = 2u;
  closest->pos = pos;
  closest->norm = front_face ? sphere_norm : vneg(sphere_norm);
  closest->col = vload(sp->col);
  closest->prim = id;
}
/* Triangle extension (NEW semantics), scanned between quads and
 * spheres; shape 0 as declared at path_tracer.wgsl:26. */
static inline void intersect_tris(const o_scene *s, ray r, int brute, hitinfo *closest) {
  float t;
  uint32_t i;
  tris_closest(s, r.start, r.dir, brute, &t, &i);
  if (i == kNoHit) return;
  v3 pos = point_at(r, t);
  float ray_dist = vdistance(pos, r.start);
  if (ray_dist >= closest->dist) return;
  const o_tri *tr = &s->tris[i];
  v3 fn = vload(tr->fn);
  int front_face = vdot(r.dir, fn) < 0.0f;
  closest->dist = ray_dist;
  closest->emissive = tr->emissive > 0.0f;
  closest->front_face = front_face;
  closest->shape = 0u;
  closest->pos = pos;
  closest->norm = front_face ? fn : vneg(fn);
  closest->col = vload(tr->col);
  closest->prim = (uint32_t)(s->nL + s->nQ) + i;
}
/* path_tracer.wgsl:290-310 */
static inline hitinfo sample_hit(const o_scene *s, ray r, int brute) {
  hitinfo hit;
  memset(&hit, 0, sizeof hit);
  hit.dist = kRayMax;
  hit.shape = kNoHit;
  hit.prim = kNoHit;
  uint32_t id = 0;
  for (int k = 0; k < s->nL; ++k) intersect_quad(r, &s->lights[k], id++, &hit);
  for (int k = 0; k < s->nQ; ++k) intersect_quad(r, &s->quads[k], id++, &hit);
  if (s->nT > 0) intersect_tris(s, r, brute, &hit);
  id = (uint32_t)(s->nL + s->nQ + s->nT);
  for (int k = 0; k < s->nS; ++k) intersect_sphere(r, &s->spheres[k], id++, &hit);
  return hit;
}

/* path_tracer.wgsl:264-288 */
static inline path raytrace(const o_scene *s, path p, int depth, uint32_t *seed, hitinfo *hout,
                            uint64_t *cnt) {
  ray r = p.r;
  cnt[O_CNT_QUERIES]++;
  if (visnan(r.start) || visnan(r.dir)) cnt[O_CNT_NAN_RAYS]++;
  else cnt[O_CNT_TRACED]++;
  hitinfo hit = sample_hit(s, r, 0);
  if (hout) *hout = hit;
  path out;
  if (hit.emissive) {
    out.r = r;
    out.end = 1;
    if (depth == 0) {
      out.col = hit.col;
      return out;
    }
    float ff = hit.front_face ? 1.0f : 0.0f;
    out.col = vmul(vscale(ff, hit.col), p.col);
    return out;
  }
  v3 scatter_dir = sample_direction(s, &hit, seed);
  float pdf_val = mixture_pdf(s, &hit, scatter_dir);
  scatter_dir = vnormalize(scatter_dir);
  out.r.start = hit.pos;
  out.r.dir = scatter_dir;
  float spdf = scattering_pdf(&hit, scatter_dir);
  v3 pc = vmul(p.col, hit.col);
  out.col = vdivs(vscale(spdf, pc), pdf_val);
  out.end = 0;
  return out;
}

typedef struct {
  v3 origin, pixel_delta_u, pixel_delta_v, pixel_origin;
  float recip_sqrt_spp;
} camframe;

/* path_tracer.wgsl:232-237 */
static inline v3 pixel_sample_square(float recip, v3 offset, v3 u, v3 v, uint32_t *seed) {
  float px = -0.5f + recip * (offset.x + rnd(seed));
  float py = -0.5f + recip * (offset.y + rnd(seed));
  return vadd(vscale(px, u), vscale(py, v));
}
/* path_tracer.wgsl:239-262 (evaluated per sample, literally) */
static inline ray setup_camera_ray(const o_camera *cam, v3 pos, v3 offset, float sw, float sh,
                                   uint32_t *seed) {
  float theta = o_radians(cam->fovy);
  v3 origin = vload(cam->origin);
  v3 end = vload(cam->target);
  float focal_length = vlength(vsub(origin, end));
  float h = o_tan(theta * 0.5f);
  float viewport_height = 2.0f * h * focal_length;
  float viewport_width = viewport_height * cam->aspect;
  v3 w = vnormalize(vsub(origin, end));
  v3 u = vnormalize(vcross(V(0, 1, 0), w));
  v3 v = vcross(w, u);
  v3 viewport_u = vscale(viewport_width, u);
  v3 viewport_v = vscale(viewport_height, vneg(v));
  v3 pixel_delta_u = vdivs(viewport_u, sw);
  v3 pixel_delta_v = vdivs(viewport_v, sh);
  v3 viewport_upper_left = vsub(vsub(vsub(origin, vscale(focal_length, w)), vscale(0.5f, viewport_u)),
                                vscale(0.5f, viewport_v));
  v3 pixel_origin = vadd(viewport_upper_left, vscale(0.5f, vadd(pixel_delta_u, pixel_delta_v)));
  v3 pixel_center = vadd(vadd(pixel_origin, vscale(pos.x, pixel_delta_u)), vscale(pos.y, pixel_delta_v));
  float recip_sqrt_spp = 1.0f / sqrtf((float)cam->spp);
  v3 pixel_sample = vadd(pixel_center,
                         pixel_sample_square(recip_sqrt_spp, offset, pixel_delta_u, pixel_delta_v, seed));
  ray r;
  r.start = origin;
  r.dir = vsub(pixel_sample, origin);
  return r;
}

/* path_tracer.wgsl:374-398 for one invocation */
static void compute_sample(const o_scene *s, const o_camera *cam, uint32_t x, uint32_t y,
                           uint32_t W, uint32_t H, float out[4], uint32_t *hit_id, uint64_t *cnt) {
  uint32_t seed = x + y * W + cam->seed * W * H;
  v3 col = V(0, 0, 0);
  uint32_t sqrt_spp = (uint32_t)sqrtf((float)cam->spp);
  int first = 1;
  if (hit_id) *hit_id = kNoHit;
  for (uint32_t s_j = 0; s_j < sqrt_spp; ++s_j) {
    for (uint32_t s_i = 0; s_i < sqrt_spp; ++s_i) {
      v3 pos = V((float)x, (float)y, 0);
      v3 offset = V((float)s_i, (float)s_j, 0);
      ray r = setup_camera_ray(cam, pos, offset, (float)W, (float)H, &seed);
      path p;
      p.r = r;
      p.col = V(1, 1, 1);
      p.end = 0;
      cnt[O_CNT_SAMPLES]++;
      for (int i = 0; i < kRayDepth; ++i) {
        hitinfo h;
        p = raytrace(s, p, i, &seed, &h, cnt);
        if (first && i == 0 && hit_id) *hit_id = h.prim;
        if (p.end) break;
      }
      first = 0;
      float fspp = (float)cam->spp;
      col = vadd(col, V(max0(p.col.x) / fspp, max0(p.col.y) / fspp, max0(p.col.z) / fspp));
    }
  }
  out[0] = col.x; out[1] = col.y; out[2] = col.z; out[3] = 1.0f;
}

static inline uint8_t unorm8(float x) {
  float c = x > 0.0f ? x : 0.0f;
  c = c < 1.0f ? c : 1.0f;
  return (uint8_t)floorf(c * 255.0f + 0.5f);
}

int o_render(const o_scene *s, const o_camera *cam, uint32_t W, uint32_t H,
             uint32_t x0, uint32_t y0, uint32_t tw, uint32_t th,
             float *rgba32f, uint8_t *rgba8, uint32_t *hit_id, uint64_t *counters,
             int nthreads) {
  if (!s || !cam) return -1;
  if (s->nL < 1 || s->nS < 1) return -2;
  uint64_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  long long npix = (long long)tw * th;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 8) reduction(+ : c0, c1, c2, c3)
  for (long long p = 0; p < npix; ++p) {
    uint32_t lx = (uint32_t)(p % tw), ly = (uint32_t)(p / tw);
    uint32_t x = x0 + lx, y = y0 + ly;
    if (x >= W || y >= H) continue; /* path_tracer.wgsl:377 */
    uint64_t cnt[O_CNT_N] = {0};
    float out[4];
    uint32_t hid;
    compute_sample(s, cam, x, y, W, H, out, &hid, cnt);
    if (rgba32f) memcpy(&rgba32f[4 * p], out, sizeof out);
    if (rgba8) {
      rgba8[4 * p + 0] = unorm8(out[0]);
      rgba8[4 * p + 1] = unorm8(out[1]);
      rgba8[4 * p + 2] = unorm8(out[2]);
      rgba8[4 * p + 3] = 255;
    }
    if (hit_id) hit_id[p] = hid;
    c0 += cnt[0]; c1 += cnt[1]; c2 += cnt[2]; c3 += cnt[3];
  }
  if (counters) {
    memset(counters, 0, sizeof(uint64_t) * O_CNT_N);
    counters[O_CNT_QUERIES] = c0;
    counters[O_CNT_TRACED] = c1;
    counters[O_CNT_SAMPLES] = c2;
    counters[O_CNT_NAN_RAYS] = c3;
  }
  return 0;
}

void o_trace(const o_scene *s, int n, const float *start, const float *dir,
             uint32_t *prim_id, float *dist, int brute) {
#pragma omp parallel for schedule(dynamic, 64)
  for (int k = 0; k < n; ++k) {
    ray r;
    r.start = vload(&start[3 * k]);
    r.dir = vload(&dir[3 * k]);
    hitinfo h = sample_hit(s, r, brute);
    prim_id[k] = h.prim;
    dist[k] = h.dist;
  }
}

void o_trace_tris(const o_scene *s, int n, const float *start, const float *dir,
                  uint32_t *tri_id, float *t, int brute) {
#pragma omp parallel for schedule(dynamic, 64)
  for (int k = 0; k < n; ++k) {
    tris_closest(s, vload(&start[3 * k]), vload(&dir[3 * k]), brute, &t[k], &tri_id[k]);
  }
}
