// bvh.h — host BVH builder (binned SAH) producing the device layout of
// wgt_internal.h / wgt_geom.h.  New component: the reference has no BVH
// (SURVEY §0.2); the build is specified by DESIGN.md §3.4 / §4.2.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../../include/wgt_api.h"

namespace wgt {

struct BvhOut {
  std::vector<float> nodes;   // 16 floats per node (4 x float4)
  std::vector<float> tris;    // kTriRecordFloats per triangle, leaf order (wgt_geom.h)
  std::vector<float> tshade;  // 8 floats per original triangle
  uint32_t n_nodes = 0, n_leaves = 0, max_depth = 0, max_leaf = 0;
  double sah_cost = 0.0;
};

// Builds over n >= 1 triangles.  max_depth_limit bounds the tree depth (the
// traversal stack holds at most depth entries).
bool BuildBvh(const wgt_triangle* tris, uint32_t n, uint32_t max_depth_limit, BvhOut& out,
              std::string& err);

}  // namespace wgt
