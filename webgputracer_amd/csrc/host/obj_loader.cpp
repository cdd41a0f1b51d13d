// obj_loader.cpp — see obj_loader.h.
#include "obj_loader.h"

#include <cstdlib>
#include <fstream>
#include <sstream>

namespace wgt {
namespace obj {

namespace {
struct Corner {
  int v = 0, t = 0, n = 0;  // 1-based after resolution, 0 = absent
};

// Resolve an OBJ index (1-based, or negative = relative to the end).
bool Resolve(long idx, size_t count, int& out) {
  if (idx > 0 && (size_t)idx <= count) { out = (int)idx; return true; }
  if (idx < 0 && (size_t)(-idx) <= count) { out = (int)((long)count + idx + 1); return true; }
  return false;
}

bool ParseCorner(const std::string& tok, size_t nv, size_t nt, size_t nn, Corner& c) {
  long parts[3] = {0, 0, 0};
  bool have[3] = {false, false, false};
  size_t start = 0;
  for (int k = 0; k < 3; ++k) {
    size_t slash = tok.find('/', start);
    std::string s = tok.substr(start, slash == std::string::npos ? std::string::npos : slash - start);
    if (!s.empty()) {
      char* end = nullptr;
      parts[k] = std::strtol(s.c_str(), &end, 10);
      if (end == s.c_str()) return false;
      have[k] = true;
    }
    if (slash == std::string::npos) break;
    start = slash + 1;
  }
  if (!have[0] || !Resolve(parts[0], nv, c.v)) return false;
  if (have[1] && !Resolve(parts[1], nt, c.t)) return false;
  if (have[2] && !Resolve(parts[2], nn, c.n)) return false;
  return true;
}
}  // namespace

bool ParseTriangulated(const std::string& text, std::vector<Vertex>& vertices, std::string& err,
                       std::string& warn) {
  std::vector<float> pos, nrm, tex;
  std::istringstream in(text);
  std::string line;
  size_t lineno = 0, skipped = 0;
  while (std::getline(in, line)) {
    ++lineno;
    if (!line.empty() && line.back() == '\r') line.pop_back();
    std::istringstream ls(line);
    std::string kw;
    if (!(ls >> kw) || kw[0] == '#') continue;
    if (kw == "v") {
      float x = 0, y = 0, z = 0;
      if (!(ls >> x >> y >> z)) { err = "bad vertex at line " + std::to_string(lineno); return false; }
      pos.push_back(x); pos.push_back(y); pos.push_back(z);
    } else if (kw == "vn") {
      float x = 0, y = 0, z = 0;
      if (!(ls >> x >> y >> z)) { err = "bad normal at line " + std::to_string(lineno); return false; }
      nrm.push_back(x); nrm.push_back(y); nrm.push_back(z);
    } else if (kw == "vt") {
      float u = 0, v = 0;
      if (!(ls >> u)) { err = "bad texcoord at line " + std::to_string(lineno); return false; }
      if (!(ls >> v)) v = 0;
      tex.push_back(u); tex.push_back(v);
    } else if (kw == "f") {
      std::vector<Corner> face;
      std::string tok;
      while (ls >> tok) {
        Corner c;
        if (!ParseCorner(tok, pos.size() / 3, tex.size() / 2, nrm.size() / 3, c)) {
          err = "bad face index '" + tok + "' at line " + std::to_string(lineno);
          return false;
        }
        face.push_back(c);
      }
      if (face.size() < 3) { ++skipped; continue; }
      auto emit = [&](const Corner& c) {
        Vertex v;
        v.point_ = vec3(pos[3 * (c.v - 1)], pos[3 * (c.v - 1) + 1], pos[3 * (c.v - 1) + 2]);
        v.normal_ = c.n ? vec3(nrm[3 * (c.n - 1)], nrm[3 * (c.n - 1) + 1], nrm[3 * (c.n - 1) + 2])
                        : vec3(0.0f, 0.0f, 1.0f);
        v.u_ = c.t ? tex[2 * (c.t - 1)] : 0.0f;
        v.v_ = c.t ? tex[2 * (c.t - 1) + 1] : 0.0f;
        vertices.push_back(v);
      };
      for (size_t k = 1; k + 1 < face.size(); ++k) {
        emit(face[0]);
        emit(face[k]);
        emit(face[k + 1]);
      }
    }
    // o, g, s, usemtl, mtllib, l, p: ignored (materials are a constant colour, scene.cpp:56)
  }
  if (skipped) warn = std::to_string(skipped) + " degenerate face(s) skipped";
  return true;
}

bool LoadTriangulated(const char* path, std::vector<Vertex>& vertices, std::string& err,
                      std::string& warn) {
  std::ifstream f(path, std::ios::binary);
  if (!f) { err = std::string("cannot open ") + path; return false; }
  std::stringstream ss;
  ss << f.rdbuf();
  return ParseTriangulated(ss.str(), vertices, err, warn);
}

}  // namespace obj
}  // namespace wgt
