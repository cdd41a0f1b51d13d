// procedural.cpp — see procedural.h.  Everything is a parametric grid surface
// (u, v) -> point, triangulated as two triangles per cell, so triangle counts are
// exact functions of the resolutions; resolutions are solved for the target.
#include "procedural.h"

#include <algorithm>
#include <cmath>
#include <functional>

namespace wgt {
namespace procedural {
namespace {

constexpr float kPi = 3.14159265358979f;

using Surf = std::function<vec3(float u, float v)>;

// nu x nv cells over [0,1]^2; closed_u wraps u.  Emits 2*nu*nv triangles.
void Grid(const Surf& f, int nu, int nv, Color3 col, std::vector<Triangle>& out) {
  std::vector<vec3> p((size_t)(nu + 1) * (nv + 1));
  for (int j = 0; j <= nv; ++j)
    for (int i = 0; i <= nu; ++i) p[(size_t)j * (nu + 1) + i] = f((float)i / nu, (float)j / nv);
  auto P = [&](int i, int j) { return p[(size_t)j * (nu + 1) + i]; };
  for (int j = 0; j < nv; ++j) {
    for (int i = 0; i < nu; ++i) {
      Vertex a(P(i, j), vec3(0, 0, 1), 0, 0), b(P(i + 1, j), vec3(0, 0, 1), 0, 0);
      Vertex c(P(i + 1, j + 1), vec3(0, 0, 1), 0, 0), d(P(i, j + 1), vec3(0, 0, 1), 0, 0);
      out.emplace_back(a, b, c, col);
      out.emplace_back(a, c, d, col);
    }
  }
}

struct Lcg {
  uint32_t s;
  float next() {
    s = s * 1664525u + 1013904223u;
    return (float)(s >> 8) * (1.0f / 16777216.0f);
  }
};

}  // namespace

void Bunny(uint32_t target_tris, uint32_t seed, std::vector<Triangle>& out) {
  // UV sphere: 2 * nu * nv triangles (poles are degenerate cells and are kept
  // so the count is exact; their zero-area triangles are rejected by MT's det test).
  const int n = std::max<int>(8, (int)target_tris);
  int nu = std::max(8, (int)std::lround(std::sqrt(n / 1.0)));
  int nv = std::max(4, (int)std::lround(n / (2.0 * nu)));
  Lcg rng{seed * 2654435761u + 12345u};
  float amp[6], fu[6], fv[6], ph[6];
  for (int k = 0; k < 6; ++k) {
    amp[k] = 0.02f + 0.05f * rng.next();
    fu[k] = (float)(1 + (int)(rng.next() * 5));
    fv[k] = (float)(1 + (int)(rng.next() * 4));
    ph[k] = 2.0f * kPi * rng.next();
  }
  const vec3 center(290.0f, 120.0f, 300.0f);
  const float R = 115.0f;
  Surf f = [&](float u, float v) {
    const float phi = 2.0f * kPi * u;
    const float theta = kPi * v;
    const float st = std::sin(theta), ct = std::cos(theta);
    vec3 dir(st * std::cos(phi), ct, st * std::sin(phi));
    float r = 1.0f;
    for (int k = 0; k < 6; ++k) r += amp[k] * std::sin(fu[k] * phi + ph[k]) * std::sin(fv[k] * theta);
    // two ears: bumps near the top-front
    for (int e = 0; e < 2; ++e) {
      vec3 ear = glm::normalize(vec3(e ? 0.35f : -0.35f, 0.9f, -0.25f));
      float c = glm::dot(dir, ear);
      if (c > 0.9f) r += 0.9f * (c - 0.9f) / 0.1f * (c - 0.9f) / 0.1f;
    }
    // squash: flatter bottom, longer body along x
    return vec3(center.x + R * 1.25f * r * dir.x, center.y + R * r * (dir.y > -0.6f ? dir.y : -0.6f - 0.2f * (dir.y + 0.6f)),
                center.z + R * 0.95f * r * dir.z);
  };
  Grid(f, nu, nv, COL_WHITE, out);
}

namespace {
// All Sponza components at resolution r; returns triangle count.
size_t SponzaAt(int r, uint32_t seed, std::vector<Triangle>* out) {
  std::vector<Triangle> dummy;
  std::vector<Triangle>& o = out ? *out : dummy;
  size_t count = 0;
  auto emit = [&](const Surf& f, int nu, int nv, Color3 col) {
    count += (size_t)2 * nu * nv;
    if (out) Grid(f, nu, nv, col, o);
  };
  Lcg rng{seed * 747796405u + 1u};
  const Color3 stone((float)0.62, (float)0.58, (float)0.5);
  const Color3 cloth_r((float)0.6, (float)0.1, (float)0.08);
  const Color3 cloth_g((float)0.1, (float)0.4, (float)0.15);
  // tiled floor (slightly bumpy), y ~ 1
  {
    const int g = 4 * r;
    float a = 0.3f + 0.3f * rng.next();
    emit([=](float u, float v) {
      return vec3(10.0f + 535.0f * u, 1.0f + a * std::sin(40.0f * u) * std::sin(40.0f * v), 10.0f + 535.0f * v);
    }, g, g, stone);
  }
  // two colonnades: 5 columns each
  const float col_x[2] = {150.0f, 405.0f};
  const int ncol = 5;
  for (int side = 0; side < 2; ++side) {
    for (int k = 0; k < ncol; ++k) {
      const float cx = col_x[side], cz = 90.0f + 95.0f * k;
      // fluted shaft
      emit([=](float u, float v) {
        float phi = 2.0f * kPi * u;
        float rad = 16.0f + 1.2f * std::cos(16.0f * phi);
        return vec3(cx + rad * std::cos(phi), 8.0f + 262.0f * v, cz + rad * std::sin(phi));
      }, 2 * r, r, stone);
      // capital (flared ring)
      emit([=](float u, float v) {
        float phi = 2.0f * kPi * u;
        float rad = 17.0f + 10.0f * v * v;
        return vec3(cx + rad * std::cos(phi), 270.0f + 18.0f * v, cz + rad * std::sin(phi));
      }, 2 * r, std::max(2, r / 4), stone);
      // arch to the next column (half torus swept along z)
      if (k + 1 < ncol) {
        emit([=](float u, float v) {
          float a = kPi * u;          // along the arch
          float b = 2.0f * kPi * v;   // around the cross-section
          float R = 47.5f, rr = 9.0f;
          float x = cx + rr * std::cos(b);
          float yc = 288.0f + R * std::sin(a);
          float zc = cz + 47.5f - R * std::cos(a);
          return vec3(x, yc + rr * std::sin(b) * std::sin(a), zc - rr * std::sin(b) * std::cos(a));
        }, 2 * r, std::max(4, r / 2), stone);
      }
    }
  }
  // gallery slabs above the colonnades (top and bottom faces)
  for (int side = 0; side < 2; ++side) {
    const float x0 = side ? 390.0f : 10.0f, x1 = side ? 545.0f : 165.0f;
    for (int face = 0; face < 2; ++face) {
      const float y = face ? 352.0f : 340.0f;
      emit([=](float u, float v) { return vec3(x0 + (x1 - x0) * u, y, 40.0f + 470.0f * v); },
           r, 2 * r, stone);
    }
  }
  // folded drapes hanging from the galleries
  for (int side = 0; side < 2; ++side) {
    for (int k = 0; k < 4; ++k) {
      const float xb = side ? 392.0f : 163.0f;
      const float z0 = 70.0f + 110.0f * k;
      const float ph = 2.0f * kPi * rng.next();
      emit([=](float u, float v) {
        float fold = 5.0f * std::sin(12.0f * kPi * u + ph) * (0.4f + 0.6f * v);
        return vec3(xb + (side ? -1.0f : 1.0f) * (4.0f + fold), 338.0f - 150.0f * v - 10.0f * std::sin(kPi * u),
                    z0 + 80.0f * u);
      }, 2 * r, 2 * r, side ? cloth_g : cloth_r);
    }
  }
  return count;
}
}  // namespace

void Sponza(uint32_t target_tris, uint32_t seed, std::vector<Triangle>& out) {
  int lo = 4, hi = 4;
  while (SponzaAt(hi, seed, nullptr) < target_tris && hi < (1 << 12)) hi *= 2;
  while (lo < hi) {  // smallest r with count >= target
    int mid = (lo + hi) / 2;
    if (SponzaAt(mid, seed, nullptr) >= target_tris) hi = mid;
    else lo = mid + 1;
  }
  SponzaAt(lo, seed, &out);
}

}  // namespace procedural
}  // namespace wgt
