// Culling hierarchy over reference treelets.
//
// The reference BVH (midpoint split cycling x -> y -> z, HW2/Bounding_volume_hierarchy.cpp:
// 3-29) decides WHICH leaves a ray may test: a leaf is reachable iff every ancestor box
// accepts the ray (BVH.cpp:31-55).  Its shape, though, makes a ray test ~146 boxes on C3.
// Here the reference tree is cut into treelets — a lone leaf, or (K = 2) the two leaf children
// of one reference node, a leaf PAIR — and an 8-wide SAH tree is built over them:
//   * every leaf has a GUARD box, the box of the reference node holding it; the kernels take
//     the exact decision per ray on that box in the leaf batch (accept with a 2^-20 relative
//     margin implies every enclosing reference box accepts too, since the boxes are unions
//     and each computed bound is within 2^-22 of its exact value; inside the band they walk
//     the ancestry with the literal reference test);
//   * the 8-wide nodes only FIND treelets: each slot holds a conservative fp16 box relative to
//     the node's origin (DevNode8), containing every guard box below it with a per-axis
//     margin (HostScene::cull_margin) that covers the rounding of the kernels' slab test, so
//     a plain slab test never culls a treelet the reference would enter.
// The wide nodes are appended to HostScene::nodes after the reference nodes; the leaves of
// the culling tree are DevLeaf records in HostScene::leaves (each wide node's leaves
// contiguous), the reference's leaf order and tie-break are untouched.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <stdexcept>
#include <vector>

#include "host_scene.h"

namespace rt {
namespace {

struct Box {
  float lo[3] = {std::numeric_limits<float>::infinity(), std::numeric_limits<float>::infinity(),
                 std::numeric_limits<float>::infinity()};
  float hi[3] = {-std::numeric_limits<float>::infinity(), -std::numeric_limits<float>::infinity(),
                 -std::numeric_limits<float>::infinity()};
  void grow(const float* b) {
    for (int a = 0; a < 3; a++) {
      lo[a] = std::min(lo[a], b[a]);
      hi[a] = std::max(hi[a], b[a + 3]);
    }
  }
  void grow(const Box& b) {
    for (int a = 0; a < 3; a++) {
      lo[a] = std::min(lo[a], b.lo[a]);
      hi[a] = std::max(hi[a], b.hi[a]);
    }
  }
  double area() const {
    const double dx = std::max(0.0, (double)hi[0] - lo[0]), dy = std::max(0.0, (double)hi[1] - lo[1]),
                 dz = std::max(0.0, (double)hi[2] - lo[2]);
    return dx * dy + dy * dz + dz * dx;
  }
};

struct Item {   // one treelet
  int leaf;     // first DFS leaf
  bool pair;    // with leaf + 1 (the two leaf children of one reference node)
  float box[6]; // guard box (the holder's box)
  float c[3];   // centroid (SAH binning)
};

// Binary SAH node: child >= 0 another node, < 0 ~item.
struct BNode {
  int child[2];
  Box box[2];
};

struct SahBuilder {
  std::vector<Item>& items;
  std::vector<BNode> nodes;
  static constexpr int kBins = 32;

  // Splits items[b, e) (e - b >= 2); returns the split point.
  int split(int b, int e) {
    Box cb;
    for (int i = b; i < e; i++) {
      const float p[6] = {items[i].c[0], items[i].c[1], items[i].c[2],
                          items[i].c[0], items[i].c[1], items[i].c[2]};
      cb.grow(p);
    }
    double best = std::numeric_limits<double>::infinity();
    int best_axis = -1, best_bin = 0;
    for (int a = 0; a < 3; a++) {
      const float ext = cb.hi[a] - cb.lo[a];
      if (!(ext > 0.0f)) continue;
      Box bins[kBins];
      int cnt[kBins] = {};
      const float scale = kBins / ext;
      for (int i = b; i < e; i++) {
        int k = (int)((items[i].c[a] - cb.lo[a]) * scale);
        k = std::min(std::max(k, 0), kBins - 1);
        cnt[k]++;
        bins[k].grow(items[i].box);
      }
      double right_area[kBins];
      int right_cnt[kBins];
      Box acc;
      int n = 0;
      for (int k = kBins - 1; k > 0; k--) {
        acc.grow(bins[k]);
        n += cnt[k];
        right_area[k] = acc.area();
        right_cnt[k] = n;
      }
      Box left;
      int nl = 0;
      for (int k = 1; k < kBins; k++) {  // split between bins k-1 and k
        left.grow(bins[k - 1]);
        nl += cnt[k - 1];
        if (nl == 0 || right_cnt[k] == 0) continue;
        const double cost = left.area() * nl + right_area[k] * right_cnt[k];
        if (cost < best) {
          best = cost;
          best_axis = a;
          best_bin = k;
        }
      }
    }
    if (best_axis < 0) return b + (e - b) / 2;  // coincident centroids: halve by position
    const int a = best_axis;
    const float scale = kBins / (cb.hi[a] - cb.lo[a]);
    auto goes_left = [&](const Item& it) {
      int k = (int)((it.c[a] - cb.lo[a]) * scale);
      k = std::min(std::max(k, 0), kBins - 1);
      return k < best_bin;
    };
    const int m = (int)(std::partition(items.begin() + b, items.begin() + e, goes_left) -
                        items.begin());
    return (m == b || m == e) ? b + (e - b) / 2 : m;
  }

  // The SAH tree over items[b0, e0) (>= 2 items); returns its root.
  int build(int b0, int e0) {
    struct Task {
      int b, e, parent, side;
    };
    std::vector<Task> todo{{b0, e0, -1, 0}};
    int root = -1;
    while (!todo.empty()) {
      const Task t = todo.back();
      todo.pop_back();
      const int idx = (int)nodes.size();
      nodes.push_back(BNode{});
      if (t.parent >= 0)
        nodes[t.parent].child[t.side] = idx;
      else
        root = idx;
      const int m = split(t.b, t.e);
      const int ranges[2][2] = {{t.b, m}, {m, t.e}};
      for (int side = 0; side < 2; side++) {
        const int b = ranges[side][0], e = ranges[side][1];
        Box u;
        for (int i = b; i < e; i++) u.grow(items[i].box);
        nodes[idx].box[side] = u;
        if (e - b == 1) nodes[idx].child[side] = ~b;
      }
      for (int side = 1; side >= 0; side--)
        if (ranges[side][1] - ranges[side][0] >= 2)
          todo.push_back({ranges[side][0], ranges[side][1], idx, side});
    }
    return root;
  }
};

// fp16 bits of the largest half <= x (up = false) or the smallest half >= x (up = true), for
// 0 <= x <= 32768; never a subnormal (a value below 2^-14 becomes 0 going down, 2^-14 going up).
uint16_t half_dir(double x, bool up) {
  if (!(x > 0.0)) return 0;
  if (x < 0x1p-14) return up ? 0x0400 : 0;
  int e;
  std::frexp(x, &e);
  int E = e - 1;  // x in [2^E, 2^(E + 1))
  const double m = std::ldexp(x, 10 - E);  // in [1024, 2048)
  double mi = up ? std::ceil(m) : std::floor(m);
  if (mi >= 2048.0) {
    mi = 1024.0;
    E++;
  }
  return (uint16_t)(((E + 15) << 10) | ((int)mi - 1024));
}

double half_value(uint16_t h) {
  const int E = (h >> 10) & 31, M = h & 1023;
  if (E == 0) return std::ldexp((double)M, -24);
  return std::ldexp(1.0 + M / 1024.0, E - 15);
}

constexpr uint16_t kHalfNaN = 0x7e00;

// Largest float <= x.
float float_down(double x) {
  float f = (float)x;
  if ((double)f > x) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
  return f;
}

struct Slot {
  int ref;  // BNode index (inner) or ~item (treelet)
  Box box;  // exact union of the guard boxes below (a treelet's guard box)
};

// Writes one wide node's header and slot boxes: origin = the inflated union's lower corner
// (rounded down to fp32), per-axis power-of-two scale with the largest offset <= 32768, each
// plane rounded outward to fp16 after the margin is applied.
void encode_node(DevNode8& W, const Slot* sl, int n, const double* margin) {
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int k = 0; k < n; k++)
    for (int a = 0; a < 3; a++) {
      lo[a] = std::min(lo[a], (double)sl[k].box.lo[a] - margin[a]);
      hi[a] = std::max(hi[a], (double)sl[k].box.hi[a] + margin[a]);
    }
  W.scale = 0;
  int ka[3];
  for (int a = 0; a < 3; a++) {
    W.origin[a] = float_down(lo[a]);
    const double ext = hi[a] - (double)W.origin[a];
    int k = (int)std::ceil(std::log2(std::max(ext, 1e-300) / 32768.0));
    k = std::min(std::max(k, -120), 120);
    while (std::ldexp(ext, -k) > 32768.0) k++;  // (log2 rounding)
    if (k > 127) throw std::runtime_error("culling node extent beyond the fp16 scale range");
    ka[a] = k;
    W.scale |= (uint32_t)(uint8_t)(int8_t)k << (8 * a);  // signed byte: one s_bfe_i32 in the kernel
  }
  for (int c = 0; c < kWideSlots; c++)
    for (int a = 0; a < 3; a++) {
      if (c >= n) {
        W.box[c][a] = (uint32_t)kHalfNaN | ((uint32_t)kHalfNaN << 16);
        continue;
      }
      const double o = (double)W.origin[a];
      const uint16_t l = half_dir(std::ldexp((double)sl[c].box.lo[a] - margin[a] - o, -ka[a]), false);
      const uint16_t h = half_dir(std::ldexp((double)sl[c].box.hi[a] + margin[a] - o, -ka[a]), true);
      W.box[c][a] = (uint32_t)l | ((uint32_t)h << 16);
    }
}

// The decoded box of slot c (for the invariant check).
void decode_slot(const DevNode8& W, int c, double* lo, double* hi) {
  for (int a = 0; a < 3; a++) {
    const int k = (int)(int8_t)(uint8_t)((W.scale >> (8 * a)) & 255);
    lo[a] = (double)W.origin[a] + std::ldexp(half_value((uint16_t)(W.box[c][a] & 0xffff)), k);
    hi[a] = (double)W.origin[a] + std::ldexp(half_value((uint16_t)(W.box[c][a] >> 16)), k);
  }
}

// SAH cost model of the wide collapse: visiting a wide node costs kNodeCost (one scalar fetch
// and eight slot tests per packet, whatever its fill), a treelet's leaf tests kLeafCost per
// leaf (they run in full-wave batches), each weighted by the surface area of the box that
// leads there (the chance a ray reaches it).
#ifndef RT_WIDE_NODE_COST  // (A/B builds: make exp EXTRA=-DRT_WIDE_LEAF_COST=...)
#define RT_WIDE_NODE_COST 1.0
#endif
#ifndef RT_WIDE_LEAF_COST
#define RT_WIDE_LEAF_COST 0.3
#endif
#ifndef RT_WIDE_SLOT_COST  // per valid slot of a visit (the kernel tests only the valid slots)
#define RT_WIDE_SLOT_COST 0.0
#endif
constexpr double kNodeCost = RT_WIDE_NODE_COST, kLeafCost = RT_WIDE_LEAF_COST,
                 kSlotCost = RT_WIDE_SLOT_COST;

// Optimal 8-wide collapse of the binary SAH tree (dynamic programme over (binary node, slots)):
// F[n][k] = least cost of covering n's subtree with k slots (a slot is a treelet, or an inner
// binary node that becomes a wide node of its own), T[n] = cost of n as a wide node.
struct WideCollapse {
  const SahBuilder& B;
  std::vector<std::array<double, kWideSlots + 1>> F;
  std::vector<std::array<signed char, kWideSlots + 1>> split;  // k of the left side
  std::vector<double> T;
  std::vector<signed char> tk;  // slots of n as a wide node

  explicit WideCollapse(const SahBuilder& b, int root) : B(b) {
    const size_t n = B.nodes.size();
    F.assign(n, {});
    split.assign(n, {});
    T.assign(n, 0.0);
    tk.assign(n, 2);
    // children after parents in B.nodes (preorder emission): a reverse sweep is post-order
    (void)root;
    for (size_t i = n; i-- > 0;) solve((int)i);
  }
  // cost of one side of binary node n as k slots
  double side(int n, int s, int k) const {
    const int c = B.nodes[n].child[s];
    if (c < 0) {
      if (k != 1) return INFINITY;
      return B.nodes[n].box[s].area() * kLeafCost * (B.items[~c].pair ? 2 : 1);
    }
    if (k == 1) return B.nodes[n].box[s].area() * kNodeCost + T[c];
    return F[c][k];
  }
  void solve(int n) {
    // F[n][k]: n's two sides covered by k slots together (k >= 2)
    for (int k = 0; k <= kWideSlots; k++) F[n][k] = INFINITY;
    for (int k = 2; k <= kWideSlots; k++)
      for (int k1 = 1; k1 < k; k1++) {
        const double c = side(n, 0, k1) + side(n, 1, k - k1);
        if (c < F[n][k]) {
          F[n][k] = c;
          split[n][k] = (signed char)k1;
        }
      }
    T[n] = INFINITY;
    Box bn = B.nodes[n].box[0];
    bn.grow(B.nodes[n].box[1]);
    const double slot = kSlotCost * bn.area();
    for (int k = 2; k <= kWideSlots; k++)
      if (F[n][k] + slot * k < T[n]) {
        T[n] = F[n][k] + slot * k;
        tk[n] = (signed char)k;
      }
  }
  // the slots of binary node n's side s covered by k slots
  void emit_side(int n, int s, int k, std::vector<Slot>& out) const {
    const int c = B.nodes[n].child[s];
    if (k == 1 || c < 0) {
      out.push_back(Slot{c, B.nodes[n].box[s]});
      return;
    }
    emit(c, k, out);
  }
  void emit(int n, int k, std::vector<Slot>& out) const {
    const int k1 = split[n][k];
    emit_side(n, 0, k1, out);
    emit_side(n, 1, k - k1, out);
  }
};

// Collapses the binary SAH tree into 8-wide nodes appended to s.nodes (WideCollapse), with
// every node's inner children allocated contiguously and its treelets' leaves appended to
// s.leaves in slot order.  Returns the tagged root; s.accel_depth receives the
// traversal-stack bound.
int collapse_wide(HostScene& s, const SahBuilder& B, int broot, const std::vector<int>& holder,
                  const std::vector<float>& ref_box) {
  const std::vector<Item>& items = B.items;
  const WideCollapse W8(B, broot);
  struct Job {
    int bnode, wide;
  };
  const int w0 = (int)s.nodes.size();
  s.nodes.resize(w0 + 2);
  std::vector<Job> todo{{broot, w0}};
  std::vector<int> order;           // wide nodes as processed (parents before children)
  std::vector<std::vector<int>> kids;  // per processed node: its inner children (wide indices)
  std::vector<Slot> slots;
  while (!todo.empty()) {
    const Job j = todo.back();
    todo.pop_back();
    slots.clear();
    W8.emit(j.bnode, W8.tk[j.bnode], slots);
    const int n = (int)slots.size();
    const Slot* sl = slots.data();
    DevNode8 W;
    std::memset(&W, 0, sizeof W);
    encode_node(W, sl, n, s.cull_margin);
    int inner = 0;
    for (int k = 0; k < n; k++) inner += sl[k].ref >= 0;
    W.inner_base = inner ? (int)s.nodes.size() : 0;
    s.nodes.resize(s.nodes.size() + 2 * (size_t)inner);
    W.leaf_base = (int)s.leaves.size();
    std::vector<int> mine;
    int off = 0, r = 0;
    for (int k = 0; k < n; k++) {
      W.kinds |= kSlotValid << k;
      if (sl[k].ref >= 0) {
        mine.push_back(W.inner_base + 2 * r++);
        continue;
      }
      const Item& it = items[~sl[k].ref];
      W.kinds |= kSlotLeafy << k;
      if (it.pair) W.kinds |= kSlotPair << k;
      W.offs |= (uint32_t)off << (4 * k);  // <= 14: at most 7 pairs before the last slot
      for (int q = 0; q < (it.pair ? 2 : 1); q++) {
        const int l = it.leaf + q;
        const DevPrim& p = s.prims[l];
        DevLeaf L;
        std::memcpy(L.v0, p.v0, sizeof L.v0);
        std::memcpy(L.a1, p.a1, sizeof L.a1);
        std::memcpy(L.a2, p.a2, sizeof L.a2);
        L.dfs = l | (p.kind == kPrimSphere ? kLeafSphere : 0);
        const float* g = &ref_box[(size_t)holder[l] * 6];
        L.g0 = g[0], L.g1 = g[1], L.g2 = g[2], L.g3 = g[3], L.g4 = g[4], L.g5 = g[5];
        s.leaves.push_back(L);
        off++;
      }
    }
    std::memcpy(&s.nodes[j.wide], &W, sizeof W);
    order.push_back(j.wide);
    kids.push_back(mine);
    r = 0;
    std::vector<Job> next;
    for (int k = 0; k < n; k++)
      if (sl[k].ref >= 0) next.push_back({sl[k].ref, mine[r++]});
    for (auto it = next.rbegin(); it != next.rend(); ++it) todo.push_back(*it);
  }
  // stack bound, children before parents: a visit keeps one entered inner slot and pushes the
  // others, then the deepest requirement below
  std::vector<int> need(s.nodes.size(), 0);
  for (size_t i = order.size(); i-- > 0;) {
    int deepest = 0;
    for (int c : kids[i]) deepest = std::max(deepest, need[c]);
    need[order[i]] = kids[i].empty() ? 0 : (int)kids[i].size() - 1 + deepest;
  }
  s.accel_depth = need[w0] + 1;
  return w0 | kWideTag;
}

}  // namespace

void build_accel(HostScene& s, int K) {
  if (s.accel_root >= 0) s.nodes.resize(s.accel_root & ~kWideTag);  // drop an earlier culling tree
  s.accel_root = -1;
  s.accel_depth = 0;
  s.accel_items = 0;
  s.ancestry.clear();
  s.leaves.clear();
  K = std::min(K, 2);
  if (K <= 0 || s.root_kind != kRootNode) return;
  const int nn = (int)s.nodes.size();
  std::vector<int> leaves(nn, 0);
  std::vector<int> parent(nn, -1), holder(s.prims.size(), -1);
  std::vector<float> ref_box((size_t)nn * 6, 0.0f);
  std::memcpy(&ref_box[0], s.root_box, sizeof s.root_box);
  for (int n = 0; n < nn; n++) {  // preorder: a parent precedes its children
    const DevNode& N = s.nodes[n];
    for (int side = 0; side < 2; side++) {
      const int c = N.child[side];
      if (c >= 0) {
        parent[c] = n;
        float* b = &ref_box[(size_t)c * 6];
        for (int a = 0; a < 3; a++) {
          b[a] = N.lo[a][side];
          b[a + 3] = N.hi[a][side];
        }
      } else {
        holder[~c] = n;
      }
    }
  }
  for (int n = nn - 1; n >= 0; n--)
    for (int side = 0; side < 2; side++) {
      const int c = s.nodes[n].child[side];
      leaves[n] += c >= 0 ? leaves[c] : 1;
    }
  if (leaves[0] <= K) return;  // the whole tree is one treelet: nothing to cull
  s.ancestry.assign(std::max<size_t>(nn, holder.size()), DevAncestry{});
  for (size_t i = 0; i < s.ancestry.size(); i++) {
    DevAncestry& A = s.ancestry[i];
    if (i < (size_t)nn) {
      std::memcpy(A.box, &ref_box[i * 6], sizeof A.box);
      A.parent = parent[i];
    }
    A.leaf_parent = i < holder.size() ? holder[i] : -1;
  }
  // culling margin: 2^-18 of the largest scene coordinate magnitude per axis
  // (the kernels add the ray origin's share per ray)
  for (int a = 0; a < 3; a++) {
    const double m = std::max(std::fabs((double)s.root_box[a]), std::fabs((double)s.root_box[a + 3]));
    s.cull_margin[a] = std::ldexp(m, -18) + 0x1p-100;
  }
  std::vector<Item> items;
  auto push_item = [&](int leaf, bool pair, int hold) {
    Item it;
    it.leaf = leaf;
    it.pair = pair;
    std::memcpy(it.box, &ref_box[(size_t)hold * 6], sizeof it.box);
    for (int a = 0; a < 3; a++) it.c[a] = 0.5f * (it.box[a] + it.box[a + 3]);
    items.push_back(it);
  };
  std::vector<int> todo{0};
  while (!todo.empty()) {
    const int n = todo.back();
    todo.pop_back();
    const DevNode& N = s.nodes[n];
    if (K == 2 && N.child[0] < 0 && N.child[1] < 0) {  // both children leaves: a pair
      if (~N.child[1] != ~N.child[0] + 1) throw std::logic_error("leaf children not consecutive");
      push_item(~N.child[0], true, n);
      continue;
    }
    for (int side = 0; side < 2; side++) {
      const int c = N.child[side];
      if (c < 0)
        push_item(~c, false, n);  // lone leaf: guarded by its holder's box
      else
        todo.push_back(c);
    }
  }
  SahBuilder B{items, {}};
  const int broot = B.build(0, (int)items.size());
  Box u;
  for (const Item& it : items) u.grow(it.box);
  for (int a = 0; a < 3; a++) {  // root box: outward by a few ulps, tested with the band
    s.accel_box[a] = u.lo[a] - std::fabs(u.lo[a]) * 0x1p-20f - 0x1p-100f;
    s.accel_box[a + 3] = u.hi[a] + std::fabs(u.hi[a]) * 0x1p-20f + 0x1p-100f;
  }
  s.accel_items = (int)items.size();
  s.accel_root = collapse_wide(s, B, broot, holder, ref_box);
  if (s.nodes.size() >= kMaxNodeSlots) {  // the kernels address wide nodes by 32-bit byte offset
    s.nodes.resize(s.accel_root & ~kWideTag);
    s.accel_root = -1;  // (the reference traversal has no such limit)
    s.accel_depth = 0;
    s.accel_items = 0;
    s.leaves.clear();
  }
}

// Structural invariants of the culling tree the kernels' exactness argument relies on
// (DESIGN.md §4.2).  Returns "" when they hold, else a description of the first violation.
std::string check_accel(const HostScene& s, int K, long long stats[4]) {
  for (int i = 0; i < 4; i++) stats[i] = 0;
  if (s.accel_root < 0) return "";
  K = std::min(K, 2);
  const int nref = s.accel_root & ~kWideTag;  // culling nodes follow the reference's
  const size_t nleaf = s.prims.size();
  // ancestry: each reference node's box is its parent's child slot; leaves point at holders
  for (int n = 0; n < nref; n++) {
    const DevNode& N = s.nodes[n];
    if (N.pad != 0) return "reference node " + std::to_string(n) + " is flagged";
    for (int side = 0; side < 2; side++) {
      const int c = N.child[side];
      if (c >= 0) {
        if (c >= nref || s.ancestry[c].parent != n) return "bad parent of node " + std::to_string(c);
        for (int a = 0; a < 3; a++)
          if (s.ancestry[c].box[a] != N.lo[a][side] || s.ancestry[c].box[a + 3] != N.hi[a][side])
            return "ancestry box of node " + std::to_string(c) + " differs from its slot";
      } else if ((size_t)~c >= nleaf || s.ancestry[~c].leaf_parent != n) {
        return "bad holder of leaf " + std::to_string(~c);
      }
    }
  }
  for (int a = 0; a < 6; a++)
    if (s.ancestry[0].box[a] != s.root_box[a]) return "root box differs from ancestry";
  if (s.leaves.size() != nleaf) return "culling leaves do not cover the leaves once";
  std::vector<int> seen(nleaf, 0);
  long long lone = 0, items = 0, nodes = 0;
  const double* mg = s.cull_margin;
  // returns the union of the guard boxes below `node` (tagged) through lo/hi, or an error
  struct Frame {
    int node, depth;
  };
  std::vector<Frame> todo{{s.accel_root, 1}};
  std::vector<int> order;
  std::vector<double> ulo(s.nodes.size() * 3, INFINITY), uhi(s.nodes.size() * 3, -INFINITY);
  while (!todo.empty()) {
    const Frame f = todo.back();
    todo.pop_back();
    if (!(f.node & kWideTag)) return "culling child is not a wide node";
    const int idx = f.node & ~kWideTag;
    if (idx < nref || (size_t)idx + 1 >= s.nodes.size()) return "wide node index out of range";
    DevNode8 W;
    std::memcpy(&W, &s.nodes[idx], sizeof W);
    nodes++;
    order.push_back(idx);
    stats[2] = std::max<long long>(stats[2], f.depth);
    int valid = 0, r = 0;
    const unsigned vbits = (unsigned)W.kinds & 0xffu;
    if (vbits & (vbits + 1)) return "valid slots not first";  // the kernel stops at the first invalid
    for (int c = 0; c < kWideSlots; c++) {
      if (!(W.kinds & (kSlotValid << c))) {
        if (W.box[c][0] != (0x7e00u | 0x7e000000u)) return "invalid slot without NaN planes";
        continue;
      }
      valid++;
      double lo[3], hi[3];
      decode_slot(W, c, lo, hi);
      if (!(W.kinds & (kSlotLeafy << c))) {
        if (W.kinds & (kSlotPair << c)) return "pair flag on an inner slot";
        const int child = W.inner_base + 2 * r++;
        todo.push_back({child | kWideTag, f.depth + 1});
        continue;  // containment checked bottom-up below
      }
      items++;
      const bool pair = (W.kinds & (kSlotPair << c)) != 0;
      const int first = W.leaf_base + (int)((W.offs >> (4 * c)) & 15);
      if (first < 0 || (size_t)first + (pair ? 2 : 1) > s.leaves.size()) return "leaf range out of bounds";
      if (!pair) lone++;
      if (pair && K < 2) return "leaf pair with K = 1";
      int hold = -1;
      for (int q = 0; q < (pair ? 2 : 1); q++) {
        const DevLeaf& L = s.leaves[first + q];
        const int l = L.dfs & ~kLeafSphere;
        if (l < 0 || (size_t)l >= nleaf) return "leaf index out of range";
        if (seen[l]++) return "leaf " + std::to_string(l) + " in two treelets";
        const DevPrim& p = s.prims[l];
        if ((p.kind == kPrimSphere) != ((L.dfs & kLeafSphere) != 0) ||
            std::memcmp(L.v0, p.v0, 12) || std::memcmp(L.a1, p.a1, 12) || std::memcmp(L.a2, p.a2, 12))
          return "leaf record differs from its primitive";
        const int h = s.ancestry[l].leaf_parent;
        const float g[6] = {L.g0, L.g1, L.g2, L.g3, L.g4, L.g5};
        if (std::memcmp(g, s.ancestry[h].box, sizeof g)) return "guard box is not the holder's box";
        if (q == 0) hold = h;
        if (q == 1 && (h != hold || l != (s.leaves[first].dfs & ~kLeafSphere) + 1 ||
                       s.nodes[h].child[0] != ~(l - 1) || s.nodes[h].child[1] != ~l))
          return "leaf pair " + std::to_string(l - 1) + " is not one node's two leaves";
        if (q == 0 && pair && s.nodes[h].child[0] != ~l) return "leaf pair does not start its holder";
        for (int a = 0; a < 3; a++)  // the slot box holds the guard box with the margin
          if (!(lo[a] <= (double)g[a] - mg[a] && hi[a] >= (double)g[a + 3] + mg[a]))
            return "slot box does not hold its guard box with the margin";
      }
    }
    if (valid < 2) return "wide node with fewer than two slots";
  }
  for (size_t l = 0; l < nleaf; l++)
    if (!seen[l]) return "leaf " + std::to_string(l) + " in no treelet";
  // containment, bottom-up: every inner slot box holds every guard box below it, with the margin
  for (auto it = order.rbegin(); it != order.rend(); ++it) {
    DevNode8 W;
    std::memcpy(&W, &s.nodes[*it], sizeof W);
    double nlo[3] = {INFINITY, INFINITY, INFINITY}, nhi[3] = {-INFINITY, -INFINITY, -INFINITY};
    int r = 0;
    for (int c = 0; c < kWideSlots; c++) {
      if (!(W.kinds & (kSlotValid << c))) continue;
      double lo[3], hi[3];
      decode_slot(W, c, lo, hi);
      double glo[3], ghi[3];
      if (W.kinds & (kSlotLeafy << c)) {
        const DevLeaf& L = s.leaves[W.leaf_base + ((W.offs >> (4 * c)) & 15)];
        const float g[6] = {L.g0, L.g1, L.g2, L.g3, L.g4, L.g5};
        for (int a = 0; a < 3; a++) glo[a] = g[a], ghi[a] = g[a + 3];
      } else {
        const size_t ci = (size_t)(W.inner_base + 2 * r++) * 3;
        for (int a = 0; a < 3; a++) {
          glo[a] = ulo[ci + a];
          ghi[a] = uhi[ci + a];
          if (!(lo[a] <= glo[a] - mg[a] && hi[a] >= ghi[a] + mg[a]))
            return "culling box does not hold the guard boxes below it with the margin";
        }
      }
      for (int a = 0; a < 3; a++) {
        nlo[a] = std::min(nlo[a], glo[a]);
        nhi[a] = std::max(nhi[a], ghi[a]);
      }
    }
    for (int a = 0; a < 3; a++) {
      ulo[(size_t)*it * 3 + a] = nlo[a];
      uhi[(size_t)*it * 3 + a] = nhi[a];
    }
  }
  const size_t r0 = (size_t)nref * 3;
  for (int a = 0; a < 3; a++)
    if (s.accel_box[a] > ulo[r0 + a] || s.accel_box[a + 3] < uhi[r0 + a])
      return "culling root box does not contain the tree";
  stats[0] = items;
  stats[1] = nodes;
  stats[3] = lone;
  return "";
}

}  // namespace rt
