// host_api.cpp — host-only entry points of the C-ABI (no GPU needed): the
// reference Cornell scene, triangle construction, OBJ I/O, procedural stand-in
// meshes and PNG output (stb_image_write replacement for save_texture.h).
#include <zlib.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/wgt/scene.h"
#include "../../../include/wgt_api.h"
#include "obj_loader.h"
#include "procedural.h"
#include "../wgt_error.h"

using namespace wgt;

namespace {
int hfail(int code, const std::string& m) {
  wgt::set_thread_error(m);
  return code;
}
}  // namespace

extern "C" int wgt_scene_cornell(wgt_quad* lights, uint32_t* n_lights, wgt_quad* quads,
                                 uint32_t* n_quads, wgt_sphere* spheres, uint32_t* n_spheres) {
  if (!n_lights || !n_quads || !n_spheres) return hfail(WGT_E_INVALID, "null count");
  Scene s(nullptr, false);
  auto l = s.PackQuads(s.lights_);
  auto q = s.PackQuads(s.quads_);
  auto sp = s.PackSpheres();
  if (*n_lights < l.size() || *n_quads < q.size() || *n_spheres < sp.size() || !lights || !quads ||
      !spheres) {
    *n_lights = (uint32_t)l.size();
    *n_quads = (uint32_t)q.size();
    *n_spheres = (uint32_t)sp.size();
    return hfail(WGT_E_INVALID, "capacity too small");
  }
  std::memcpy(lights, l.data(), l.size() * sizeof(wgt_quad));
  std::memcpy(quads, q.data(), q.size() * sizeof(wgt_quad));
  std::memcpy(spheres, sp.data(), sp.size() * sizeof(wgt_sphere));
  *n_lights = (uint32_t)l.size();
  *n_quads = (uint32_t)q.size();
  *n_spheres = (uint32_t)sp.size();
  return WGT_OK;
}

extern "C" int wgt_make_triangles(const float* verts, uint32_t n, const float col[3], int emissive,
                                  const float translation[3], wgt_triangle* out) {
  if ((n > 0 && (!verts || !out)) || !col) return hfail(WGT_E_INVALID, "null argument");
  Scene s;
  vec3 tr = translation ? vec3(translation[0], translation[1], translation[2]) : vec3(0, 0, 0);
  for (uint32_t i = 0; i < n; ++i) {
    const float* v = verts + (size_t)9 * i;
    Vertex a, b, c;
    a.point_ = vec3(v[0], v[1], v[2]);
    b.point_ = vec3(v[3], v[4], v[5]);
    c.point_ = vec3(v[6], v[7], v[8]);
    s.tris_.emplace_back(a.Translate(tr), b.Translate(tr), c.Translate(tr), Color3(col[0], col[1], col[2]),
                         emissive != 0);
  }
  auto packed = s.PackTriangles();
  if (n) std::memcpy(out, packed.data(), packed.size() * sizeof(wgt_triangle));
  return WGT_OK;
}

extern "C" int wgt_load_obj(const char* path, const float col[3], const float translation[3],
                            int emissive, wgt_triangle* out, uint32_t* n_inout) {
  if (!path || !col || !n_inout) return hfail(WGT_E_INVALID, "null argument");
  Scene s;
  vec3 tr = translation ? vec3(translation[0], translation[1], translation[2]) : vec3(0, 0, 0);
  if (!s.LoadObj(path, Color3(col[0], col[1], col[2]), tr, emissive != 0))
    return hfail(WGT_E_IO, std::string("cannot load OBJ ") + path);
  auto packed = s.PackTriangles();
  if (!out) {
    *n_inout = (uint32_t)packed.size();
    return WGT_OK;
  }
  if (*n_inout < packed.size()) {
    *n_inout = (uint32_t)packed.size();
    return hfail(WGT_E_INVALID, "capacity too small");
  }
  std::memcpy(out, packed.data(), packed.size() * sizeof(wgt_triangle));
  *n_inout = (uint32_t)packed.size();
  return WGT_OK;
}

extern "C" int wgt_procedural_mesh(int kind, uint32_t target_tris, uint32_t seed, wgt_triangle* out,
                                   uint32_t* n_inout) {
  if (!n_inout) return hfail(WGT_E_INVALID, "null count");
  std::vector<Triangle> tris;
  if (kind == 0) procedural::Bunny(target_tris, seed, tris);
  else if (kind == 1) procedural::Sponza(target_tris, seed, tris);
  else return hfail(WGT_E_INVALID, "unknown procedural kind");
  Scene s;
  s.tris_ = std::move(tris);
  auto packed = s.PackTriangles();
  if (!out) {
    *n_inout = (uint32_t)packed.size();
    return WGT_OK;
  }
  if (*n_inout < packed.size()) {
    *n_inout = (uint32_t)packed.size();
    return hfail(WGT_E_INVALID, "capacity too small");
  }
  std::memcpy(out, packed.data(), packed.size() * sizeof(wgt_triangle));
  *n_inout = (uint32_t)packed.size();
  return WGT_OK;
}

extern "C" int wgt_write_obj(const char* path, const wgt_triangle* tris, uint32_t n) {
  if (!path || (n && !tris)) return hfail(WGT_E_INVALID, "null argument");
  FILE* f = std::fopen(path, "w");
  if (!f) return hfail(WGT_E_IO, std::string("cannot open ") + path);
  std::fprintf(f, "# wgt procedural mesh, %u triangles\n", n);
  for (uint32_t i = 0; i < n; ++i) {
    const wgt_triangle& t = tris[i];
    // v1 = v0 + e1, v2 = v0 + e2 (exact reconstruction is not required: the OBJ
    // round-trip is re-packed by the Triangle ctor)
    std::fprintf(f, "v %.9g %.9g %.9g\n", t.v0[0], t.v0[1], t.v0[2]);
    std::fprintf(f, "v %.9g %.9g %.9g\n", t.v0[0] + t.e1[0], t.v0[1] + t.e1[1], t.v0[2] + t.e1[2]);
    std::fprintf(f, "v %.9g %.9g %.9g\n", t.v0[0] + t.e2[0], t.v0[1] + t.e2[1], t.v0[2] + t.e2[2]);
  }
  for (uint32_t i = 0; i < n; ++i) std::fprintf(f, "f %u %u %u\n", 3 * i + 1, 3 * i + 2, 3 * i + 3);
  bool ok = std::fclose(f) == 0;
  return ok ? WGT_OK : hfail(WGT_E_IO, "write failed");
}

// PNG (RGBA8, 8-bit, non-interlaced) via zlib; replaces stbi_write_png
// (save_texture.h:63).
extern "C" int wgt_write_png(const char* path, const uint8_t* rgba8, uint32_t w, uint32_t h) {
  if (!path || !rgba8 || w == 0 || h == 0) return hfail(WGT_E_INVALID, "bad argument");
  std::vector<uint8_t> raw((size_t)(w * 4 + 1) * h);
  for (uint32_t y = 0; y < h; ++y) {
    raw[(size_t)y * (w * 4 + 1)] = 0;
    std::memcpy(&raw[(size_t)y * (w * 4 + 1) + 1], rgba8 + (size_t)y * w * 4, (size_t)w * 4);
  }
  uLongf zlen = compressBound((uLong)raw.size());
  std::vector<uint8_t> z(zlen);
  // Z_BEST_SPEED: a path-traced frame's sample noise leaves little for higher levels to find
  // (1080p: 6.74 against 6.73 MB), at 0.6x the time of level 6
  if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), Z_BEST_SPEED) != Z_OK)
    return hfail(WGT_E_IO, "zlib compress failed");
  FILE* f = std::fopen(path, "wb");
  if (!f) return hfail(WGT_E_IO, std::string("cannot open ") + path);
  auto be32 = [](uint32_t v, uint8_t* p) {
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
  };
  auto chunk = [&](const char* type, const uint8_t* data, uint32_t len) {
    uint8_t hdr[8];
    be32(len, hdr);
    std::memcpy(hdr + 4, type, 4);
    std::fwrite(hdr, 1, 8, f);
    if (len) std::fwrite(data, 1, len, f);
    uLong crc = crc32(0L, (const Bytef*)type, 4);
    if (len) crc = crc32(crc, data, len);
    uint8_t c[4];
    be32((uint32_t)crc, c);
    std::fwrite(c, 1, 4, f);
  };
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  std::fwrite(sig, 1, 8, f);
  uint8_t ihdr[13];
  be32(w, ihdr);
  be32(h, ihdr + 4);
  ihdr[8] = 8;   // bit depth
  ihdr[9] = 6;   // RGBA
  ihdr[10] = 0;  // deflate
  ihdr[11] = 0;  // filter
  ihdr[12] = 0;  // no interlace
  chunk("IHDR", ihdr, 13);
  chunk("IDAT", z.data(), (uint32_t)zlen);
  chunk("IEND", nullptr, 0);
  bool ok = std::fclose(f) == 0;
  return ok ? WGT_OK : hfail(WGT_E_IO, "write failed");
}
