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
  std::vector<float> nodes;   // kNode4Floats per BVH4 node (wgt_geom.h layout), root = 0
  std::vector<uint32_t> cnodes;  // kCNodeFloats words per node: the compact form (wgt_geom.h)
  std::vector<int32_t> crefs;    // 4 child refs per node (the compact form's ref records)
  float cstep = 1.0f;            // scene-wide decode step of the compact nodes
  float cbound = 0.0f;           // M: the compact codes are exact for ray origins with |o| <= M
  std::vector<float> tris;    // kTriRecordFloats per triangle, leaf order (wgt_geom.h)
  std::vector<float> tshade;  // 8 floats per original triangle
  uint32_t n_nodes = 0, n_leaves = 0, max_depth = 0, max_leaf = 0;  // BVH4 nodes / depth
  uint32_t n_nodes2 = 0, depth2 = 0;  // the SAH BVH2 the BVH4 was collapsed from
  uint32_t stack_need = 0;            // worst-case traversal stack entries (exact for this tree)
  bool narrow = false;                // collapsed under narrow_limit (BuildBvh)
  double sah_cost = 0.0;
};

// Builds over n >= 1 triangles.  max_depth_limit bounds the BVH2 depth, which
// bounds the BVH4 depth and so the traversal stack (stack_need <= 3 * depth).
// stack_limit bounds stack_need: a greedy collapse over the limit is redone
// two-levels-per-node (stack_need <= 3 * ceil(depth2 / 2)).
// narrow_limit > 0: the BVH2 is also collapsed under that smaller stack bound, and
// that tree is kept (out.narrow) if it has at most narrow_ratio times the nodes.
// origin_bound: an upper bound on |coordinate| of every ray origin the compact nodes
// will see (camera and hit points); the margin of their codes grows with it
// (CompactNode), and a frame whose camera lies beyond out.cbound reads the 128-B
// nodes instead.
constexpr double kNarrowNodeRatio = 1.03;
bool BuildBvh(const wgt_triangle* tris, uint32_t n, uint32_t max_depth_limit, uint32_t stack_limit,
              uint32_t narrow_limit, double narrow_ratio, double origin_bound, BvhOut& out, std::string& err);

}  // namespace wgt
