// host_fuzz.cpp — the product's host code under AddressSanitizer + UBSan (CPU only; built and
// run by tests/test_host_sanitize.py): the BVH builder over random, degenerate and extreme
// triangle sets and every stack budget, the OBJ parser over valid, malformed and random
// text, the procedural meshes, and the host C-ABI entry points (Cornell scene, triangle
// packing, OBJ and PNG writers).  Exits non-zero on a failed invariant; the sanitizers
// abort on the first finding.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <random>
#include <string>
#include <vector>

#include "../../include/wgt_api.h"
#include "../../webgputracer_amd/csrc/host/bvh.h"
#include "../../webgputracer_amd/csrc/host/obj_loader.h"
#include "../../webgputracer_amd/csrc/host/procedural.h"

// wgt_runtime.cpp's entry points, which need the HIP runtime (Scene::InitBuffers references
// them; nothing here calls them)
namespace wgt {
void set_thread_error(const std::string&) {}
}
extern "C" const char* wgt_last_error(const wgt_ctx*) { return ""; }
extern "C" int wgt_upload_scene(wgt_ctx*, const wgt_quad*, uint32_t, const wgt_quad*, uint32_t, const wgt_sphere*,
                                uint32_t, const wgt_triangle*, uint32_t) {
  return WGT_E_INVALID;
}

static int g_fail = 0;
#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                          \
    }                                                                    \
  } while (0)

static std::vector<wgt_triangle> pack(const std::vector<float>& v) {  // 9 floats per triangle
  const uint32_t n = (uint32_t)(v.size() / 9);
  std::vector<wgt_triangle> t(n);
  const float col[3] = {0.5f, 0.5f, 0.5f};
  CHECK(wgt_make_triangles(v.data(), n, col, 0, nullptr, t.data()) == WGT_OK);
  return t;
}

// The 64-B compact form (WGT_CN64) holds the tree whenever no coordinate is farther from the world
// origin than ~the scene's extent (its origins are 512 K steps with K a signed byte, and the step is
// ~extent / 65504): checked for such triangle sets.
// Returns whether the build succeeded (its output checked).
static bool build(const std::vector<wgt_triangle>& t, uint32_t stack_limit, uint32_t narrow) {
  wgt::BvhOut out;
  std::string err;
  const bool ok = wgt::BuildBvh(t.data(), (uint32_t)t.size(), 24, stack_limit, narrow, 1.03, 1e4, out, err);
  if (!ok) {  // a refusal must say why
    CHECK(!err.empty());
    return false;
  }
  CHECK(out.n_nodes >= 1);
  CHECK(out.nodes.size() == (size_t)out.n_nodes * 32);
  CHECK(out.tris.size() == t.size() * 16);
  CHECK(out.stack_need <= 3u * 24u);
  CHECK(out.max_leaf >= 1 && out.max_leaf <= 8);
  // every triangle index appears once in the leaf-ordered records
  std::vector<int> seen(t.size(), 0);
  for (size_t i = 0; i < t.size(); ++i) {
    uint32_t idx;
    std::memcpy(&idx, &out.tris[i * 16 + 3], 4);
    CHECK(idx < t.size());
    if (idx < t.size()) ++seen[idx];
  }
  for (int s : seen) CHECK(s == 1);
  // the compact form: one record and 4 refs per node
  CHECK(out.cnodes.size() == (size_t)out.n_nodes * 16 && out.crefs.size() == (size_t)out.n_nodes * 4);
  return true;
}

static std::vector<float> soup(std::mt19937& g, uint32_t n, float spread, float size) {
  std::uniform_real_distribution<float> u(0.0f, spread);
  std::normal_distribution<float> e(0.0f, size);
  std::vector<float> v;
  for (uint32_t i = 0; i < n; ++i) {
    const float x = u(g), y = u(g), z = u(g);
    const float p[9] = {x, y, z, x + e(g), y + e(g), z + e(g), x + e(g), y + e(g), z + e(g)};
    v.insert(v.end(), p, p + 9);
  }
  return v;
}

static void fuzz_bvh() {
  std::mt19937 g(7);
  const uint32_t sizes[] = {1, 2, 3, 7, 8, 9, 17, 33, 257, 1000, 5000};
  for (uint32_t n : sizes) {
    for (uint32_t lim : {31u, 24u, 20u, 16u}) build(pack(soup(g, n, 500.0f, 20.0f)), lim, 0);
    build(pack(soup(g, n, 500.0f, 20.0f)), 31, 25);
  }
  // coincident triangles (no SAH split exists), zero-area ones, one plane, one line of centroids
  std::vector<float> same, flat, plane, line;
  for (uint32_t i = 0; i < 300; ++i) {
    const float a[9] = {0, 0, 0, 10, 0, 0, 0, 10, 0};
    same.insert(same.end(), a, a + 9);
    const float f = (float)i;
    const float b[9] = {f, f, f, f, f, f, f, f, f};  // a point
    flat.insert(flat.end(), b, b + 9);
    const float c[9] = {f, 0, 5, f + 1, 0, 5, f, 1, 5};
    plane.insert(plane.end(), c, c + 9);
    const float d[9] = {0, 0, f, 1, 0, f, 0, 1, f};
    line.insert(line.end(), d, d + 9);
  }
  for (auto* v : {&same, &flat, &plane, &line}) build(pack(*v), 31, 0);
  // extreme magnitudes within the scene limits (coordinates up to 2^40, edges up to 2^30)
  for (float s : {1e-30f, 1e-10f, 1.0f, 1e6f, 1e11f}) {
    std::vector<float> v = soup(g, 500, 1.0f, 0.01f);
    for (float& x : v) x *= s;
    build(pack(v), 31, 0);
  }
}

static void fuzz_obj() {
  std::vector<wgt::Vertex> vs;
  std::string err, warn;
  const char* texts[] = {
      "", "\n\n", "# only a comment\n", "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n",
      "v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nvt 0.5 0.5\nvn 0 0 1\nf 1/1/1 2/1/1 3/1/1 4/1/1\n",
      "v 0 0 0\nv 1 0 0\nv 0 1 0\nf -3 -2 -1\n", "v 0 0 0\nf 1 2 3\n", "f 1 2 3\n", "v 1 2\nf 1 1 1\n",
      "v a b c\nf 1 2 3\n", "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1/ 2// 3/x/\n", "v 0 0 0\nf 0 0 0\n",
      "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 4294967296 1 2\n", "v 1e39 -1e39 nan\nv 0 0 0\nv 1 1 1\nf 1 2 3\n",
      "v 0 0 0\r\nv 1 0 0\r\nv 0 1 0\r\nf 1 2 3\r\n", "g a\no b\nusemtl m\ns off\nmtllib x.mtl\n",
      "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2\n", "vt\nvn\nv\nf\n"};
  for (const char* t : texts) {
    vs.clear();
    (void)wgt::obj::ParseTriangulated(t, vs, err, warn);
    CHECK(vs.size() % 3 == 0);
  }
  std::mt19937 g(11);
  const char* tok[] = {"v", "vt", "vn", "f", "g", "o", "#", "1", "-1", "2/3", "4//5", "/", "//", "0.5", "-2.5e3",
                       "nan", "inf", "x", " ", "\t", "7/8/9", "-0", "99999999999", "\\"};
  for (int it = 0; it < 3000; ++it) {
    std::string s;
    const int lines = (int)(g() % 20);
    for (int l = 0; l < lines; ++l) {
      const int nt = (int)(g() % 6);
      for (int k = 0; k < nt; ++k) {
        s += tok[g() % (sizeof(tok) / sizeof(tok[0]))];
        s += ' ';
      }
      s += (g() % 7) ? "\n" : "\r\n";
    }
    vs.clear();
    (void)wgt::obj::ParseTriangulated(s, vs, err, warn);
    CHECK(vs.size() % 3 == 0);
  }
}

static void host_api() {
  wgt_quad l[8], q[64];
  wgt_sphere sp[8];
  uint32_t nl = 8, nq = 64, ns = 8;
  CHECK(wgt_scene_cornell(l, &nl, q, &nq, sp, &ns) == WGT_OK);
  uint32_t z = 0;
  CHECK(wgt_scene_cornell(l, &z, q, &nq, sp, &ns) == WGT_E_INVALID);  // capacity too small
  for (int kind = 0; kind < 2; ++kind) {
    uint32_t n = 0;
    CHECK(wgt_procedural_mesh(kind, kind ? 20000 : 5000, 1, nullptr, &n) == WGT_OK);
    std::vector<wgt_triangle> t(n);
    CHECK(wgt_procedural_mesh(kind, kind ? 20000 : 5000, 1, t.data(), &n) == WGT_OK);
    CHECK(build(t, 31, 0));  // the Cornell-box meshes build
    const char* path = "/tmp/wgt_host_fuzz.obj";
    CHECK(wgt_write_obj(path, t.data(), n) == WGT_OK);
    const float col[3] = {0.2f, 0.4f, 0.6f};
    uint32_t m = 0;
    CHECK(wgt_load_obj(path, col, nullptr, 0, nullptr, &m) == WGT_OK);
    CHECK(m == n);
    std::vector<wgt_triangle> r(m);
    CHECK(wgt_load_obj(path, col, nullptr, 0, r.data(), &m) == WGT_OK);
    uint32_t small = m ? m - 1 : 0;
    if (m) CHECK(wgt_load_obj(path, col, nullptr, 0, r.data(), &small) == WGT_E_INVALID);
    std::remove(path);
  }
  CHECK(wgt_procedural_mesh(2, 10, 1, nullptr, &nl) == WGT_E_INVALID);
  for (uint32_t w : {1u, 3u, 64u}) {
    std::vector<uint8_t> px((size_t)w * 5 * 4, 0x5a);
    CHECK(wgt_write_png("/tmp/wgt_host_fuzz.png", px.data(), w, 5) == WGT_OK);
  }
  std::remove("/tmp/wgt_host_fuzz.png");
  CHECK(wgt_write_png("/tmp/wgt_host_fuzz.png", nullptr, 1, 1) == WGT_E_INVALID);
  uint32_t n = 0;
  const float col[3] = {1, 1, 1};
  CHECK(wgt_load_obj("/nonexistent/wgt.obj", col, nullptr, 0, nullptr, &n) == WGT_E_IO);
}

int main() {
  fuzz_bvh();
  fuzz_obj();
  host_api();
  std::printf("host_fuzz: %s (%d failed checks)\n", g_fail ? "FAIL" : "ok", g_fail);
  return g_fail ? 1 : 0;
}
