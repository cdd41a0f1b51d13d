// bvh.cpp — binned-SAH BVH2 builder, collapsed into the 4-wide BVH the kernels
// traverse.  Leaf boxes are unions of the padded triangle boxes of the geometry
// spec (wgt_geom.h tri_box, evaluated on the host with the same fp32 operations),
// so every node box contains, bit for bit, the boxes of all triangles below it:
// the traversal is exact.  The collapse only regroups BVH2 child
// boxes, so the BVH4 child boxes are exactly BVH2 node boxes.
#include "bvh.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>

#include "../wgt_geom.h"

namespace wgt {
namespace {

struct Box {
  float lo[3], hi[3];
  void reset() {
    for (int c = 0; c < 3; ++c) {
      lo[c] = std::numeric_limits<float>::infinity();
      hi[c] = -std::numeric_limits<float>::infinity();
    }
  }
  void grow(const Box& b) {
    for (int c = 0; c < 3; ++c) {
      lo[c] = std::min(lo[c], b.lo[c]);
      hi[c] = std::max(hi[c], b.hi[c]);
    }
  }
  double area() const {
    double dx = (double)hi[0] - lo[0], dy = (double)hi[1] - lo[1], dz = (double)hi[2] - lo[2];
    if (dx < 0 || dy < 0 || dz < 0) return 0.0;
    return 2.0 * (dx * dy + dy * dz + dz * dx);
  }
};

struct Prim {
  Box b;
  float c[3];
  uint32_t idx;
};

constexpr int kMaxBins = 256;
// SAH bins per axis (WGT_SAH_BINS, <= kMaxBins; tuning sweeps)
int SahBins() {
  const char* v = std::getenv("WGT_SAH_BINS");
  const int n = v && *v ? std::atoi(v) : 128;
  return std::max(2, std::min(n, kMaxBins));
}

// Depth of a median-split subtree over `count` primitives (leaves <= leaf_max).
uint32_t MedianDepth(uint32_t count, uint32_t leaf_max = (uint32_t)kLeafMax) {
  uint32_t d = 0;
  while (count > leaf_max) {
    count = (count + 1) / 2;
    ++d;
  }
  return d;
}
// SAH costs of a BVH2 node visit and a triangle test, and the largest leaf the
// SAH may choose (<= kLeafMax, the encoding's limit).  WGT_SAH_TRAV / WGT_SAH_LEAF
// override them for tuning sweeps; the defaults are the measured best.
constexpr double kCostTri = 1.0;
double SahTravCost() {
  const char* v = std::getenv("WGT_SAH_TRAV");
  return v && *v ? std::atof(v) : 1.0;
}
uint32_t SahLeafMax() {
  const char* v = std::getenv("WGT_SAH_LEAF");
  const int n = v && *v ? std::atoi(v) : kLeafMax;
  return (uint32_t)std::max(1, std::min(n, kLeafMax));
}

class Builder {
 public:
  // leaf_max: the largest leaf (kLeafMax, the BVH4 record's limit)
  Builder(std::vector<Prim>& p, BvhOut& o, std::vector<float>& n2, uint32_t limit,
          uint32_t leaf_max = (uint32_t)kLeafMax)
      : prims_(p), out_(o), nodes_(n2), limit_(limit), leaf_max_(leaf_max),
        sah_leaf_(std::min(SahLeafMax(), leaf_max)) {}

  // Returns the child reference of the subtree over prims_[begin, end).
  int Build(uint32_t begin, uint32_t end, uint32_t depth, Box& box) {
    box.reset();
    Box cb;
    cb.reset();
    for (uint32_t i = begin; i < end; ++i) {
      box.grow(prims_[i].b);
      for (int c = 0; c < 3; ++c) {
        cb.lo[c] = std::min(cb.lo[c], prims_[i].c[c]);
        cb.hi[c] = std::max(cb.hi[c], prims_[i].c[c]);
      }
    }
    const uint32_t count = end - begin;
    out_.depth2 = std::max(out_.depth2, depth);
    if (count == 1) return MakeLeaf(begin, count, box);

    uint32_t mid = begin;
    // Depth guarantee: every leaf at depth <= limit_ (the traversal stack holds at
    // most `depth` entries).  Invariant: depth + MedianDepth(count) <= limit_; an SAH
    // split is taken only if both children keep it, otherwise the median split does.
    bool median = false;
    {
      double best = std::numeric_limits<double>::infinity();
      int best_axis = -1, best_bin = -1;
      const double parea = box.area();
      for (int axis = 0; axis < 3; ++axis) {
        const float ext = cb.hi[axis] - cb.lo[axis];
        if (!(ext > 0.0f)) continue;
        Box bb[kMaxBins];
        uint32_t bn[kMaxBins] = {};
        for (int k = 0; k < bins_; ++k) bb[k].reset();
        const double scale = bins_ / (double)ext;
        for (uint32_t i = begin; i < end; ++i) {
          int k = std::min(bins_ - 1, (int)((prims_[i].c[axis] - cb.lo[axis]) * scale));
          bb[k].grow(prims_[i].b);
          bn[k]++;
        }
        double rarea[kMaxBins];
        uint32_t rcount[kMaxBins];
        Box acc;
        acc.reset();
        uint32_t n = 0;
        for (int k = bins_ - 1; k > 0; --k) {
          acc.grow(bb[k]);
          n += bn[k];
          rarea[k] = acc.area();
          rcount[k] = n;
        }
        acc.reset();
        n = 0;
        for (int k = 0; k < bins_ - 1; ++k) {
          acc.grow(bb[k]);
          n += bn[k];
          if (n == 0 || rcount[k + 1] == 0) continue;
          double cost = acc.area() * n + rarea[k + 1] * rcount[k + 1];
          if (cost < best) {
            best = cost;
            best_axis = axis;
            best_bin = k;
          }
        }
      }
      const double split_cost = cost_trav_ + kCostTri * (parea > 0 ? best / parea : 0.0);
      const double leaf_cost = kCostTri * count;
      if (best_axis >= 0 && !(count <= sah_leaf_ && leaf_cost <= split_cost)) {
        const float ext = cb.hi[best_axis] - cb.lo[best_axis];
        const double scale = bins_ / (double)ext;
        auto it = std::partition(prims_.begin() + begin, prims_.begin() + end, [&](const Prim& p) {
          int k = std::min(bins_ - 1, (int)((p.c[best_axis] - cb.lo[best_axis]) * scale));
          return k <= best_bin;
        });
        mid = (uint32_t)(it - prims_.begin());
        if (mid == begin || mid == end) median = true;
        else if (depth + 1 + MedianDepth(std::max(mid - begin, end - mid), leaf_max_) > limit_) median = true;
      } else if (count <= leaf_max_) {
        return MakeLeaf(begin, count, box);
      } else {
        median = true;
      }
    }
    if (median) {
      if (count <= leaf_max_) return MakeLeaf(begin, count, box);
      int axis = 0;
      for (int c = 1; c < 3; ++c)
        if (cb.hi[c] - cb.lo[c] > cb.hi[axis] - cb.lo[axis]) axis = c;
      mid = begin + count / 2;
      std::nth_element(prims_.begin() + begin, prims_.begin() + mid, prims_.begin() + end,
                       [axis](const Prim& a, const Prim& b) {
                         return a.c[axis] < b.c[axis] || (a.c[axis] == b.c[axis] && a.idx < b.idx);
                       });
    }
    const uint32_t id = (uint32_t)(nodes_.size() / 16);
    nodes_.resize(nodes_.size() + 16);
    Box bl, br;
    const int rl = Build(begin, mid, depth + 1, bl);
    const int rr = Build(mid, end, depth + 1, br);
    WriteNode(id, bl, rl, br, rr);
    out_.sah_cost += cost_trav_ * box.area();
    return (int)id;
  }

  void WriteNode(uint32_t id, const Box& b0, int r0, const Box& b1, int r1) {
    float* n = &nodes_[(size_t)id * 16];
    n[0] = b0.lo[0]; n[1] = b0.hi[0]; n[2] = b0.lo[1]; n[3] = b0.hi[1];
    n[4] = b1.lo[0]; n[5] = b1.hi[0]; n[6] = b1.lo[1]; n[7] = b1.hi[1];
    n[8] = b0.lo[2]; n[9] = b0.hi[2]; n[10] = b1.lo[2]; n[11] = b1.hi[2];
    std::memcpy(&n[12], &r0, 4);
    std::memcpy(&n[13], &r1, 4);
    n[14] = 0.0f;
    n[15] = 0.0f;
  }

 private:
  int MakeLeaf(uint32_t begin, uint32_t count, const Box& box) {
    out_.n_leaves++;
    out_.max_leaf = std::max(out_.max_leaf, count);
    out_.sah_cost += kCostTri * count * box.area();
    return leaf_ref(begin, count);
  }

  std::vector<Prim>& prims_;
  BvhOut& out_;
  std::vector<float>& nodes_;
  uint32_t limit_;
  uint32_t leaf_max_;
  uint32_t sah_leaf_;
  double cost_trav_ = SahTravCost();
  int bins_ = SahBins();
};


// BVH2 child `which` (0/1) of node `id`, from the 16-float BVH2 layout.
struct Child {
  Box b;
  int ref;
};
Child Child2(const std::vector<float>& n2, int id, int which) {
  const float* n = &n2[(size_t)id * 16];
  Child c;
  const int o = which ? 4 : 0;
  c.b.lo[0] = n[o + 0]; c.b.hi[0] = n[o + 1]; c.b.lo[1] = n[o + 2]; c.b.hi[1] = n[o + 3];
  c.b.lo[2] = n[8 + 2 * which]; c.b.hi[2] = n[9 + 2 * which];
  std::memcpy(&c.ref, &n[12 + which], 4);
  return c;
}

// Budgeted greedy collapse: a BVH4 node starts from the two children of a BVH2
// node and repeatedly opens its largest-area internal child until it has 4
// slots.  Returns the BVH4 node index; `need` receives the worst-case stack
// entries of the subtree: the traversal pushes at most (children - 1) per node
// on a root-to-node path, so need = (children - 1) + max over internal children.
// The stack is bounded by `budget`: a child is opened only while (children - 1)
// + the least need any child can still reach (its BVH2 height: a 2-wide node
// pushes one entry per level) fits, so only the deep, stack-heavy paths get
// narrower nodes.  Any budget >= the BVH2 height is met.
class Collapser {
 public:
  Collapser(const std::vector<float>& n2, BvhOut& o) : n2_(n2), out_(o), h_(n2.size() / 16, 0u) {
    for (size_t i = h_.size(); i-- > 0;) {  // children follow their parent (preorder)
      uint32_t m = 0;
      for (int w = 0; w < 2; ++w) {
        const Child c = Child2(n2_, (int)i, w);
        if (c.ref >= 0) m = std::max(m, h_[c.ref]);
      }
      h_[i] = 1u + m;
    }
  }
  uint32_t Height(int id2) const { return h_[id2]; }

  int Collapse(int id2, uint32_t depth, uint32_t budget, uint32_t& need) {
    Child ch[kBvhWidth];
    int n = 2;
    ch[0] = Child2(n2_, id2, 0);
    ch[1] = Child2(n2_, id2, 1);
    bool blocked[kBvhWidth] = {false, false, false, false};
    while (n < kBvhWidth) {
      int best = -1;
      double ba = -1.0;
      for (int i = 0; i < n; ++i)
        if (ch[i].ref >= 0 && !blocked[i] && ch[i].b.area() > ba) {
          ba = ch[i].b.area();
          best = i;
        }
      if (best < 0) break;
      // the node after opening `best`: n children, the least subtree need of each
      uint32_t m = 0;
      for (int i = 0; i < n; ++i)
        if (i != best && ch[i].ref >= 0) m = std::max(m, h_[ch[i].ref]);
      const int r = ch[best].ref;
      for (int w = 0; w < 2; ++w) {
        const Child c = Child2(n2_, r, w);
        if (c.ref >= 0) m = std::max(m, h_[c.ref]);
      }
      if ((uint32_t)n + m > budget) {  // (n + 1 children) - 1 + m
        blocked[best] = true;
        continue;
      }
      ch[best] = Child2(n2_, r, 0);
      ch[n++] = Child2(n2_, r, 1);
      blocked[best] = false;
    }
    const uint32_t id = (uint32_t)(out_.nodes.size() / kNode4Floats);
    out_.nodes.resize(out_.nodes.size() + kNode4Floats);
    out_.max_depth = std::max(out_.max_depth, depth + 1);
    int refs[kBvhWidth];
    uint32_t sub = 0;
    for (int i = 0; i < n; ++i) {
      if (ch[i].ref >= 0) {
        uint32_t sn = 0;
        refs[i] = Collapse(ch[i].ref, depth + 1, budget - (uint32_t)(n - 1), sn);
        sub = std::max(sub, sn);
      } else {
        refs[i] = ch[i].ref;
      }
    }
    need = (uint32_t)(n - 1) + sub;
    float* o = &out_.nodes[(size_t)id * kNode4Floats];
    for (int i = 0; i < kBvhWidth; ++i) {
      const bool live = i < n;
      for (int c = 0; c < 3; ++c) {
        o[(2 * c) * 4 + i] = live ? ch[i].b.lo[c] : kEmptySlotCoord;
        o[(2 * c + 1) * 4 + i] = live ? ch[i].b.hi[c] : kEmptySlotCoord;
      }
      const int r = live ? refs[i] : refs[0];
      std::memcpy(&o[24 + i], &r, 4);
      o[28 + i] = 0.0f;
    }
    return (int)id;
  }

 private:
  const std::vector<float>& n2_;
  BvhOut& out_;
  std::vector<uint32_t> h_;  // BVH2 height (internal levels) of every BVH2 node
};

// SAH-optimal collapse under the stack budget (the default; WGT_COLLAPSE=greedy
// selects Collapser).  Every BVH4 node is a frontier of 2..4 descendants of a BVH2
// node; a dynamic program over the BVH2 (children before parents) picks, per node
// and per stack budget B, the frontier minimising the BVH4 SAH cost
//   N(r, B) = c_node * A(r) + min_{k=2..4} Q(r's children -> k slots, B - (k - 1))
//   Q(c -> 1 slot, B) = leaf ? c_tri * count * A(c) : N(c, B)
//   Q(c -> k slots, B) = min_{i + j = k} Q(left(c) -> i, B) + Q(right(c) -> j, B)
// (A = surface area; a node of k slots pushes at most k - 1 entries, so its
// subtree's stack need is (k - 1) + the largest need of its internal slots).
// Like the greedy collapse it only regroups BVH2 boxes: the BVH4 child boxes are
// BVH2 node boxes and the exactness argument is unchanged.
double DpNodeCost() {
  const char* v = std::getenv("WGT_DP_NODE");
  return v && *v ? std::atof(v) : 1.0;
}
double DpTriCost() {
  const char* v = std::getenv("WGT_DP_TRI");
  return v && *v ? std::atof(v) : 1.0;
}
// Largest leaf the collapse may make of a BVH2 subtree (its triangles are one
// contiguous range): 0 keeps the BVH2 leaves (WGT_DP_LEAF, <= kLeafMax).
uint32_t DpLeafMax() {
  const char* v = std::getenv("WGT_DP_LEAF");
  const int n = v && *v ? std::atoi(v) : 0;
  return (uint32_t)std::max(0, std::min(n, kLeafMax));
}
bool UseDpCollapse() {
  const char* v = std::getenv("WGT_COLLAPSE");
  return !(v && std::strcmp(v, "greedy") == 0);
}

class DpCollapser {
 public:
  DpCollapser(const std::vector<float>& n2, BvhOut& o, uint32_t budget)
      : n2_(n2), out_(&o), nb_(budget + 1), n_(n2.size() / 16) {
    const float inf = std::numeric_limits<float>::infinity();
    cost_.assign(n_ * 4 * nb_, inf);  // [node][k-1][B]: k = 1 is N(node, B)
    range_.assign(n_, Range{0u, 0u});
    area_.assign(n_, 0.0);
    for (size_t i = n_; i-- > 0;) {   // preorder: children have larger ids
      const Child a = Child2(n2_, (int)i, 0), b = Child2(n2_, (int)i, 1);
      Box u = a.b;
      u.grow(b.b);
      const double area = u.area();
      area_[i] = area;
      // the node's triangles: one contiguous range (the children's ranges are adjacent)
      const Range ra = Tris(a), rb = Tris(b);
      range_[i] = Range{std::min(ra.first, rb.first), ra.count + rb.count};
      for (uint32_t B = 0; B < nb_; ++B) {
        // k slots of node i's frontier, each with need <= B
        for (int k = 2; k <= 4; ++k) {
          float best = inf;
          for (int ia = 1; ia < k; ++ia) best = std::min(best, Slots(a, ia, B) + Slots(b, k - ia, B));
          Q(i, k, B) = best;
        }
        float best = inf;
        for (int k = 2; k <= 4; ++k)
          if ((uint32_t)(k - 1) <= B) best = std::min(best, Q(i, k, B - (uint32_t)(k - 1)));
        Q(i, 1, B) = (float)(c_node_ * area) + best;
      }
    }
  }
  float Cost(uint32_t budget) const { return budget < nb_ ? Q(0, 1, budget) : std::numeric_limits<float>::infinity(); }
  void Retarget(BvhOut& o) { out_ = &o; }

  // Emit node id2 as a BVH4 node with stack need <= budget (preorder ids).
  int Emit(int id2, uint32_t depth, uint32_t budget, uint32_t& need) {
    const Child a = Child2(n2_, id2, 0), b = Child2(n2_, id2, 1);
    int best_k = 2;
    float best = std::numeric_limits<float>::infinity();
    for (int k = 2; k <= 4; ++k)
      if ((uint32_t)(k - 1) <= budget && Q(id2, k, budget - (uint32_t)(k - 1)) < best) {
        best = Q(id2, k, budget - (uint32_t)(k - 1));
        best_k = k;
      }
    const uint32_t sb = budget - (uint32_t)(best_k - 1);
    std::vector<Child> slots;
    Split(a, b, best_k, sb, slots);
    BvhOut& out = *out_;
    const uint32_t id = (uint32_t)(out.nodes.size() / kNode4Floats);
    out.nodes.resize(out.nodes.size() + kNode4Floats);
    out.max_depth = std::max(out.max_depth, depth + 1);
    const int n = (int)slots.size();
    int refs[kBvhWidth];
    uint32_t sub = 0;
    for (int i = 0; i < n; ++i) {
      if (slots[i].ref >= 0) {
        uint32_t sn = 0;
        refs[i] = Emit(slots[i].ref, depth + 1, sb, sn);
        sub = std::max(sub, sn);
      } else {
        refs[i] = slots[i].ref;
      }
    }
    need = (uint32_t)(n - 1) + sub;
    float* o = &out.nodes[(size_t)id * kNode4Floats];
    for (int i = 0; i < kBvhWidth; ++i) {
      const bool live = i < n;
      for (int c = 0; c < 3; ++c) {
        o[(2 * c) * 4 + i] = live ? slots[i].b.lo[c] : kEmptySlotCoord;
        o[(2 * c + 1) * 4 + i] = live ? slots[i].b.hi[c] : kEmptySlotCoord;
      }
      const int r = live ? refs[i] : refs[0];
      std::memcpy(&o[24 + i], &r, 4);
      o[28 + i] = 0.0f;
    }
    return (int)id;
  }

 private:
  float& Q(size_t node, int k, uint32_t B) { return cost_[(node * 4 + (size_t)(k - 1)) * nb_ + B]; }
  float Q(size_t node, int k, uint32_t B) const { return cost_[(node * 4 + (size_t)(k - 1)) * nb_ + B]; }
  // cost of covering child c with k slots, each of stack need <= B
  float Slots(const Child& c, int k, uint32_t B) const {
    if (c.ref < 0) return k == 1 ? (float)(c_tri_ * leaf_count(c.ref) * c.b.area()) : std::numeric_limits<float>::infinity();
    if (k == 1 && Mergeable(c)) return std::min(Q((size_t)c.ref, 1, B), MergedCost(c));
    return Q((size_t)c.ref, k, B);
  }
  struct Range {
    uint32_t first, count;
  };
  Range Tris(const Child& c) const {
    if (c.ref < 0) return Range{leaf_first(c.ref), leaf_count(c.ref)};
    return range_[(size_t)c.ref];
  }
  // an internal BVH2 child with few enough triangles may become one leaf slot
  bool Mergeable(const Child& c) const {
    if (c.ref < 0 || leaf_max_ == 0) return false;
    const uint32_t n = range_[(size_t)c.ref].count;
    return n != 0 && n <= leaf_max_;
  }
  float MergedCost(const Child& c) const { return (float)(c_tri_ * range_[(size_t)c.ref].count * area_[(size_t)c.ref]); }
  // the slot of child c in a cover by one slot: merged into a leaf when that is cheaper
  Child AsSlot(const Child& c, uint32_t B) const {
    if (Mergeable(c) && MergedCost(c) < Q((size_t)c.ref, 1, B)) {
      const Range r = range_[(size_t)c.ref];
      Child m = c;
      m.ref = leaf_ref(r.first, r.count);
      return m;
    }
    return c;
  }
  // the slots of the cheapest cover of a and b by k slots (budget B each)
  void Split(const Child& a, const Child& b, int k, uint32_t B, std::vector<Child>& out) const {
    int best_i = 1;
    float best = std::numeric_limits<float>::infinity();
    for (int i = 1; i < k; ++i) {
      const float c = Slots(a, i, B) + Slots(b, k - i, B);
      if (c < best) {
        best = c;
        best_i = i;
      }
    }
    Cover(a, best_i, B, out);
    Cover(b, k - best_i, B, out);
  }
  void Cover(const Child& c, int k, uint32_t B, std::vector<Child>& out) const {
    if (k == 1) {
      out.push_back(AsSlot(c, B));
      return;
    }
    Split(Child2(n2_, c.ref, 0), Child2(n2_, c.ref, 1), k, B, out);
  }

  const std::vector<float>& n2_;
  BvhOut* out_;
  uint32_t nb_;
  size_t n_;
  double c_node_ = DpNodeCost(), c_tri_ = DpTriCost();
  uint32_t leaf_max_ = DpLeafMax();
  std::vector<float> cost_;
  std::vector<Range> range_;
  std::vector<double> area_;
};

// Compact form of one node (wgt_geom.h).  The kernel evaluates a child plane's slab
// distance as fma(h, s/d, c) with c = fma(org/s, s/d, ot) per node and axis (one
// fused step instead of decoding the plane first), so the codes keep a margin G
// from the exact child bounds: a lo code's plane org' + h*s (org' = the stored
// org/s times s) lies <= lo - G, a hi code's >= hi + G.  G = 2^-21 * M, with M
// >= |org'| and >= |ray origin| (BuildBvh's origin_bound), covers the rounding of
// c: every decoded interval then contains, bit for bit, the
// slab interval fma(b, 1/d, ot) of every triangle box b below the child.  Codes
// are the tightest binary16 values with the margin (non-negative half bit
// patterns order like their values, so a binary search finds them).
double CDecD(uint32_t h, double s, double orgd) { return orgd + (double)half_bits_to_float(h) * s; }
void CompactNode(const float* n, float s, double G, uint32_t* q) {
  bool live[kBvhWidth];
  for (int i = 0; i < kBvhWidth; ++i) live[i] = !(n[i] == kEmptySlotCoord && n[4 + i] == kEmptySlotCoord);
  float orgs[3];
  for (int a = 0; a < 3; ++a) {
    double ulo = std::numeric_limits<double>::infinity();
    for (int i = 0; i < kBvhWidth; ++i)
      if (live[i]) ulo = std::min(ulo, (double)n[(2 * a) * 4 + i]);
    // org/s as a float whose value times s is <= ulo - G
    const double target = (ulo - G) / (double)s;
    float f = (float)target;
    while ((double)f > target) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
    orgs[a] = f;
    const double orgd = (double)f * (double)s;
    uint32_t lo_h[kBvhWidth], hi_h[kBvhWidth];
    for (int i = 0; i < kBvhWidth; ++i) {
      lo_h[i] = hi_h[i] = 0x7c00u;  // an empty slot: +inf planes on every axis, never entered
      if (!live[i]) continue;
      const double blo = (double)n[(2 * a) * 4 + i] - G, bhi = (double)n[(2 * a + 1) * 4 + i] + G;
      uint32_t l = 0, r = 0x7bffu;  // largest h with plane <= blo (h = 0 is: orgd <= ulo - G)
      while (l < r) {
        const uint32_t m = (l + r + 1) / 2;
        if (CDecD(m, s, orgd) <= blo) l = m; else r = m - 1;
      }
      lo_h[i] = l;
      l = 0; r = 0x7bffu;  // smallest h with plane >= bhi (CompactStep guarantees h = 65504 is)
      while (l < r) {
        const uint32_t m = (l + r) / 2;
        if (CDecD(m, s, orgd) >= bhi) r = m; else l = m + 1;
      }
      hi_h[i] = l;
    }
    q[4 + 4 * a + 0] = lo_h[0] | (lo_h[1] << 16);
    q[4 + 4 * a + 1] = lo_h[2] | (lo_h[3] << 16);
    q[4 + 4 * a + 2] = hi_h[0] | (hi_h[1] << 16);
    q[4 + 4 * a + 3] = hi_h[2] | (hi_h[3] << 16);
  }
  std::memcpy(&q[0], orgs, 12);
  q[3] = 0u;  // reserved
}

// The smallest power-of-two step with which code 65504 reaches every node's upper
// bounds plus the margins (the origin sits up to G + one float step of org/s below
// the lower bound).
float CompactStep(const std::vector<float>& nodes, uint32_t n_nodes, double G) {
  int e = -24;
  for (;;) {
    const float s = std::ldexp(1.0f, e);
    bool ok = true;
    for (uint32_t k = 0; k < n_nodes && ok; ++k) {
      const float* n = &nodes[(size_t)k * kNode4Floats];
      for (int a = 0; a < 3 && ok; ++a) {
        double ulo = std::numeric_limits<double>::infinity(), uhi = -ulo;
        for (int i = 0; i < kBvhWidth; ++i)
          if (!(n[i] == kEmptySlotCoord && n[4 + i] == kEmptySlotCoord)) {
            ulo = std::min(ulo, (double)n[(2 * a) * 4 + i]);
            uhi = std::max(uhi, (double)n[(2 * a + 1) * 4 + i]);
          }
        const double org_low = ulo - G - (std::fabs(ulo - G) * 0x1p-23 + (double)s * 0x1p-126);
        ok = org_low + 65504.0 * (double)s >= uhi + G;
      }
    }
    if (ok) return s;
    ++e;
  }
}

}  // namespace

bool BuildBvh(const wgt_triangle* tris, uint32_t n, uint32_t max_depth_limit, uint32_t stack_limit,
              uint32_t narrow_limit, double narrow_ratio, double origin_bound, BvhOut& out, std::string& err) {
  out = BvhOut{};
  if (n == 0) { err = "BuildBvh: no triangles"; return false; }
  // leaf walks use 32-bit byte offsets into the 64-B records (wgt_geom.h kTriRecordBytes)
  if (n >= (1u << 26)) { err = "BuildBvh: too many triangles (max 2^26-1)"; return false; }
  std::vector<Prim> prims(n);
  for (uint32_t i = 0; i < n; ++i) {
    const wgt_triangle& t = tris[i];
    f3 lo, hi;
    tri_box(f3{t.v0[0], t.v0[1], t.v0[2]}, f3{t.e1[0], t.e1[1], t.e1[2]},
            f3{t.e2[0], t.e2[1], t.e2[2]}, lo, hi);
    Prim& p = prims[i];
    p.b.lo[0] = lo.x; p.b.lo[1] = lo.y; p.b.lo[2] = lo.z;
    p.b.hi[0] = hi.x; p.b.hi[1] = hi.y; p.b.hi[2] = hi.z;
    for (int c = 0; c < 3; ++c) p.c[c] = 0.5f * p.b.lo[c] + 0.5f * p.b.hi[c];
    p.idx = i;
    for (int c = 0; c < 3; ++c) {
      if (!std::isfinite(p.b.lo[c]) || !std::isfinite(p.b.hi[c])) {
        err = "BuildBvh: non-finite triangle " + std::to_string(i);
        return false;
      }
    }
  }
  if (MedianDepth(n) > max_depth_limit) {
    err = "BuildBvh: too many triangles for depth limit " + std::to_string(max_depth_limit);
    return false;
  }
  std::vector<float> n2;
  n2.reserve((size_t)16 * 2 * (n / 2 + 1));
  Builder b(prims, out, n2, max_depth_limit);
  Box root_box;
  const int root = b.Build(0, n, 0, root_box);
  if (root < 0) {
    // single leaf: a root node whose second child is an empty slot (wgt_geom.h)
    n2.assign(16, 0.0f);
    Box empty;
    for (int c = 0; c < 3; ++c) empty.lo[c] = empty.hi[c] = kEmptySlotCoord;
    b.WriteNode(0, root_box, root, empty, root);
    out.depth2 = 1;
  }
  if (out.depth2 > max_depth_limit) {
    err = "BuildBvh: depth " + std::to_string(out.depth2) + " exceeds " + std::to_string(max_depth_limit);
    return false;
  }
  out.n_nodes2 = (uint32_t)(n2.size() / 16);
  const double ra = root_box.area();
  if (ra > 0) out.sah_cost /= ra;
  out.nodes.reserve(n2.size() * 2);
  Collapser greedy(n2, out);
  if (greedy.Height(0) > stack_limit) {
    err = "BuildBvh: BVH2 height " + std::to_string(greedy.Height(0)) + " exceeds the stack limit " +
          std::to_string(stack_limit);
    return false;
  }
  const bool dp = UseDpCollapse();
  std::unique_ptr<DpCollapser> opt;
  if (dp) {
    opt.reset(new DpCollapser(n2, out, stack_limit));
    if (!(opt->Cost(stack_limit) < std::numeric_limits<float>::infinity())) opt.reset();
  }
  if (opt) opt->Emit(0, 0, stack_limit, out.stack_need);
  else greedy.Collapse(0, 0, stack_limit, out.stack_need);
  if (out.stack_need > stack_limit) {
    err = "BuildBvh: traversal stack " + std::to_string(out.stack_need) + " exceeds " +
          std::to_string(stack_limit);
    return false;
  }
  out.n_nodes = (uint32_t)(out.nodes.size() / kNode4Floats);
  if (out.n_nodes >= (1u << 24)) {  // the device copies address nodes by 32-bit byte offsets below kNoRef
    err = "BuildBvh: too many BVH nodes (max 2^24-1)";
    return false;
  }
  if (narrow_limit > 0 && narrow_limit < stack_limit && greedy.Height(0) <= narrow_limit) {
    BvhOut nar;
    if (opt && opt->Cost(narrow_limit) < std::numeric_limits<float>::infinity()) {
      opt->Retarget(nar);
      opt->Emit(0, 0, narrow_limit, nar.stack_need);
    } else {
      Collapser tight(n2, nar);
      tight.Collapse(0, 0, narrow_limit, nar.stack_need);
    }
    const uint32_t nn = (uint32_t)(nar.nodes.size() / kNode4Floats);
    // greedy trees: at most narrow_ratio x the nodes; optimal trees: at most narrow_ratio
    // x the SAH cost of the wide tree
    const bool cheap = opt ? opt->Cost(narrow_limit) <= narrow_ratio * opt->Cost(stack_limit)
                           : nn <= narrow_ratio * out.n_nodes;
    if (nar.stack_need <= narrow_limit && cheap) {
      out.nodes.swap(nar.nodes);
      out.n_nodes = nn;
      out.stack_need = nar.stack_need;
      out.max_depth = nar.max_depth;
      out.narrow = true;
    }
  }
  // The device traversal has no iteration cap: it terminates because every
  // internal ref points forward (preorder), so no node is visited twice.
  for (uint32_t i = 0; i < out.n_nodes; ++i) {
    for (int s = 0; s < 4; ++s) {
      int32_t r;
      std::memcpy(&r, &out.nodes[(size_t)i * kNode4Floats + 24 + s], 4);
      const uint32_t u = ~(uint32_t)r;
      const bool ok = r >= 0 ? ((uint32_t)r > i && (uint32_t)r < out.n_nodes)
                             : ((uint64_t)(u >> 3) + (u & 7u) + 1u <= n);
      if (!ok) {
        err = "BuildBvh: malformed node " + std::to_string(i);
        return false;
      }
    }
  }
  // the compact codes' margin: M bounds |ray origin| (the caller's origin_bound) and
  // every coordinate of the tree (so |org'| <= M as well)
  double M = std::max(origin_bound, 0x1p-60);
  for (uint32_t i = 0; i < out.n_nodes; ++i)
    for (int k = 0; k < 24; ++k) {
      const float v = out.nodes[(size_t)i * kNode4Floats + k];
      if (v != kEmptySlotCoord) M = std::max(M, 2.0 * std::fabs((double)v));
    }
  out.cbound = (float)M;
  const double G = std::ldexp(M, -21);
  out.cstep = CompactStep(out.nodes, out.n_nodes, G);
  out.cnodes.resize((size_t)out.n_nodes * kCNodeFloats);
  out.crefs.resize((size_t)out.n_nodes * 4);
  for (uint32_t i = 0; i < out.n_nodes; ++i) {
    CompactNode(&out.nodes[(size_t)i * kNode4Floats], out.cstep, G, &out.cnodes[(size_t)i * kCNodeFloats]);
    std::memcpy(&out.crefs[(size_t)i * 4], &out.nodes[(size_t)i * kNode4Floats + 24], 16);
  }
  out.tris.resize((size_t)n * kTriRecordFloats);
  for (uint32_t i = 0; i < n; ++i) {
    const wgt_triangle& t = tris[prims[i].idx];
    const Box& b = prims[i].b;
    float* o = &out.tris[(size_t)i * kTriRecordFloats];
    o[0] = t.v0[0]; o[1] = t.v0[1]; o[2] = t.v0[2];
    std::memcpy(&o[3], &prims[i].idx, 4);
    o[4] = t.e1[0]; o[5] = t.e1[1]; o[6] = t.e1[2]; o[7] = b.lo[0];
    o[8] = t.e2[0]; o[9] = t.e2[1]; o[10] = t.e2[2]; o[11] = b.lo[1];
    o[12] = b.lo[2]; o[13] = b.hi[0]; o[14] = b.hi[1]; o[15] = b.hi[2];
  }
  out.tshade.resize((size_t)n * 8);
  for (uint32_t i = 0; i < n; ++i) {
    const wgt_triangle& t = tris[i];
    float* o = &out.tshade[(size_t)i * 8];
    o[0] = t.face_norm[0]; o[1] = t.face_norm[1]; o[2] = t.face_norm[2]; o[3] = t.emissive;
    o[4] = t.col[0]; o[5] = t.col[1]; o[6] = t.col[2]; o[7] = 0.0f;
  }
  return true;
}

}  // namespace wgt
