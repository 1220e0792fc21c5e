// Culling hierarchy over reference treelets.
//
// The reference BVH (midpoint split cycling x -> y -> z, HW2/Bounding_volume_hierarchy.cpp:
// 3-29) decides WHICH leaves a ray may test: a leaf is reachable iff every ancestor box
// accepts the ray (BVH.cpp:31-55).  Its shape, though, makes a ray test ~146 boxes on C3.
// Here the reference tree is cut into treelets (maximal subtrees with <= K leaves; a lone leaf
// child of a larger node is a treelet of its own) and a binned-SAH tree is built over the
// treelets.  The kernels walk the SAH tree to find treelets, then walk each treelet with the
// reference's own semantics.  Reachability is preserved by a per-treelet guard:
//   * the guard box is the innermost reference ancestor box a ray must pass to enter the
//     treelet (the treelet root's own box, or for a lone leaf its parent's box);
//   * the fast slab test decides "accept" only with a 2^-20 relative margin, and an accept
//     with that margin implies every enclosing reference box accepts too (the boxes are
//     unions, so the exact t-intervals nest; each computed bound is within 2^-22 of its exact
//     value) — no need to test the ancestors;
//   * inside the margin band the kernel walks the ancestor chain with the literal reference
//     test (ref_parent / ref_box below).
// SAH inner boxes are only culling bounds: they contain every guard box below them, and the
// kernel tests them conservatively (only a sure reject culls), so a treelet the reference would
// enter is never culled.  The SAH tree's nodes are appended to HostScene::nodes after the
// reference nodes; DevNode::pad marks them (kAccelNode | guard bits per child).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <stdexcept>
#include <vector>

#include "host_scene.h"

namespace rt {
namespace {

struct Item {
  int ref;        // treelet root: reference node index, or ~leaf
  float box[6];   // guard box
  float c[3];     // centroid (SAH binning)
  int height;     // internal-node levels of the treelet (stack use inside it)
};

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

// outward by a few ulps: a culling bound only, never compared with the reference's boxes
float widen_down(float x) { return x - std::fabs(x) * 0x1p-20f - 0x1p-100f; }
float widen_up(float x) { return x + std::fabs(x) * 0x1p-20f + 0x1p-100f; }

struct SahBuilder {
  std::vector<Item>& items;
  std::vector<DevNode>& nodes;
  bool pairs = true;  // two-leaf treelets as leaf pairs (kAccelPair*)
  int depth = 0;  // max over leaves of (SAH levels + treelet height)

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

  // Emits the SAH tree over items[b0, e0) (>= 2 items) in DFS preorder; returns its root.
  int build(int b0, int e0) {
    struct Task {
      int b, e, parent, side, depth;
    };
    std::vector<Task> todo{{b0, e0, -1, 0, 0}};
    int root = -1;
    while (!todo.empty()) {
      const Task t = todo.back();
      todo.pop_back();
      const int idx = (int)nodes.size();
      nodes.push_back(DevNode{});
      if (t.parent >= 0)
        nodes[t.parent].child[t.side] = idx;
      else
        root = idx;
      DevNode& N = nodes[idx];
      N.pad = kAccelNode;
      const int m = split(t.b, t.e);
      const int ranges[2][2] = {{t.b, m}, {m, t.e}};
      for (int side = 0; side < 2; side++) {
        const int b = ranges[side][0], e = ranges[side][1];
        if (e - b == 1) {
          const Item& it = items[b];
          int ref = it.ref;
          if (pairs && ref >= 0) {  // a reference node whose children are two consecutive leaves
            const DevNode& R = nodes[ref];
            if (R.pad == 0 && R.child[0] < 0 && R.child[1] < 0 && ~R.child[1] == ~R.child[0] + 1) {
              ref = R.child[0];
              N.pad |= side ? kAccelPair1 : kAccelPair0;
            }
          }
          N.child[side] = ref;
          N.pad |= side ? kAccelGuard1 : kAccelGuard0;
          for (int a = 0; a < 3; a++) {
            N.lo[a][side] = it.box[a];
            N.hi[a][side] = it.box[a + 3];
          }
          depth = std::max(depth, t.depth + 1 + it.height);
        } else {
          Box u;
          for (int i = b; i < e; i++) u.grow(items[i].box);
          for (int a = 0; a < 3; a++) {
            N.lo[a][side] = widen_down(u.lo[a]);
            N.hi[a][side] = widen_up(u.hi[a]);
          }
        }
      }
      // right pushed first: the left subtree is emitted first (preorder)
      for (int side = 1; side >= 0; side--)
        if (ranges[side][1] - ranges[side][0] >= 2)
          todo.push_back({ranges[side][0], ranges[side][1], idx, side, t.depth + 1});
    }
    return root;
  }
};

// Reference subtree height (internal-node levels): the stack a guarded treelet of more than
// two leaves can need.
int ref_height(const std::vector<DevNode>& nodes, int n) {
  int h = 0;
  for (int side = 0; side < 2; side++)
    if (nodes[n].child[side] >= 0) h = std::max(h, ref_height(nodes, nodes[n].child[side]));
  return h + 1;
}

// Collapses the binary culling tree (nodes[nref..], rooted at `root`) into 4-wide nodes that
// replace it: each wide node takes a binary node's two slots and repeatedly opens the inner
// slot with the largest box (surface area) into its two children, up to four slots.  Every
// slot keeps its box, guard and pair flags, so the acceptance tests are the binary tree's.
// Returns the tagged wide root; `stack` receives a bound on the traversal stack.
int collapse_wide(std::vector<DevNode>& nodes, int nref, int root, int& stack) {
  const std::vector<DevNode> bin(nodes.begin() + nref, nodes.end());
  nodes.resize(nref);
  struct Slot {
    int ref;
    bool guard, pair;
    float box[6];
  };
  auto slot_of = [&](int bnode, int side) {
    const DevNode& N = bin[bnode - nref];
    Slot sl;
    sl.ref = N.child[side];
    sl.guard = (N.pad & (side ? kAccelGuard1 : kAccelGuard0)) != 0;
    sl.pair = (N.pad & (side ? kAccelPair1 : kAccelPair0)) != 0;
    for (int a = 0; a < 3; a++) {
      sl.box[a] = N.lo[a][side];
      sl.box[a + 3] = N.hi[a][side];
    }
    return sl;
  };
  auto area = [](const float* b) {
    const double dx = (double)b[3] - b[0], dy = (double)b[4] - b[1], dz = (double)b[5] - b[2];
    return dx * dy + dy * dz + dz * dx;
  };
  struct Job {
    int bnode, parent, slot, depth;
  };
  std::vector<Job> todo{{root, -1, 0, 0}};
  int wroot = -1;
  std::vector<int> order;  // wide nodes in preorder
  while (!todo.empty()) {
    const Job j = todo.back();
    todo.pop_back();
    Slot sl[4];
    int n = 2;
    sl[0] = slot_of(j.bnode, 0);
    sl[1] = slot_of(j.bnode, 1);
    while (n < 4) {
      int best = -1;
      double ba = -1.0;
      for (int k = 0; k < n; k++)
        if (!sl[k].guard && area(sl[k].box) > ba) {
          ba = area(sl[k].box);
          best = k;
        }
      if (best < 0) break;
      const int bn = sl[best].ref;
      sl[best] = slot_of(bn, 0);
      sl[n++] = slot_of(bn, 1);
    }
    const int w = (int)nodes.size();
    nodes.resize(w + 2);
    DevNode4 W;
    std::memset(&W, 0, sizeof W);
    if (j.depth < kWideTopLevels) W.flags |= kWideTop;
    for (int k = 0; k < 4; k++) {
      for (int a = 0; a < 3; a++) {  // (empty slots: an inverted box, never read)
        W.lo[a][k] = k < n ? sl[k].box[a] : 1.0f;
        W.hi[a][k] = k < n ? sl[k].box[a + 3] : -1.0f;
      }
      if (k >= n) continue;
      W.flags |= kWideValid << k;
      if (sl[k].guard) {
        W.child[k] = sl[k].ref;
        W.flags |= kWideGuard << k;
        if (sl[k].pair) W.flags |= kWidePair << k;
      }
    }
    std::memcpy(&nodes[w], &W, sizeof W);
    if (j.parent >= 0) {
      DevNode4 P;
      std::memcpy(&P, &nodes[j.parent], sizeof P);
      P.child[j.slot] = w | kWideTag;
      std::memcpy(&nodes[j.parent], &P, sizeof P);
    } else {
      wroot = w;
    }
    order.push_back(w);
    for (int k = n - 1; k >= 0; k--)
      if (!sl[k].guard) todo.push_back({sl[k].ref, w, k, j.depth + 1});
  }
  // stack bound, bottom-up: a visit pushes at most (slots - 1) entries
  std::vector<int> need(nodes.size(), 0);
  for (auto it = order.rbegin(); it != order.rend(); ++it) {
    DevNode4 W;
    std::memcpy(&W, &nodes[*it], sizeof W);
    int slots = 0, deepest = 0;
    for (int k = 0; k < 4; k++) {
      if (!(W.flags & (kWideValid << k))) continue;
      slots++;
      const int c = W.child[k];
      if (!(W.flags & (kWideGuard << k)))
        deepest = std::max(deepest, need[c & ~kWideTag]);
      else if (c >= 0)
        deepest = std::max(deepest, ref_height(nodes, c));
    }
    need[*it] = slots - 1 + deepest;
  }
  stack = need[wroot] + 1;
  return wroot | kWideTag;
}

}  // namespace


void build_accel(HostScene& s, int K) {
  if (s.accel_root >= 0) s.nodes.resize(s.accel_root & ~kWideTag);  // drop an earlier culling tree
  s.accel_root = -1;
  s.accel_depth = 0;
  s.accel_items = 0;
  s.ancestry.clear();
  if (K <= 0 || s.root_kind != kRootNode) return;
  const int nn = (int)s.nodes.size();
  std::vector<int> leaves(nn, 0), height(nn, 1);
  std::vector<int> parent(nn, -1), leaf_parent(s.prims.size(), -1);
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
        leaf_parent[~c] = n;
      }
    }
  }
  for (int n = nn - 1; n >= 0; n--) {
    const DevNode& N = s.nodes[n];
    int h = 0;
    for (int side = 0; side < 2; side++) {
      const int c = N.child[side];
      if (c >= 0) {
        leaves[n] += leaves[c];
        h = std::max(h, height[c]);
      } else {
        leaves[n] += 1;
      }
    }
    height[n] = h + 1;
  }
  if (leaves[0] <= K) return;  // the whole tree is one treelet: nothing to cull
  s.ancestry.assign(std::max<size_t>(nn, leaf_parent.size()), DevAncestry{});
  for (size_t i = 0; i < s.ancestry.size(); i++) {
    DevAncestry& A = s.ancestry[i];
    if (i < (size_t)nn) {
      std::memcpy(A.box, &ref_box[i * 6], sizeof A.box);
      A.parent = parent[i];
    }
    A.leaf_parent = i < leaf_parent.size() ? leaf_parent[i] : -1;
  }
  std::vector<Item> items;
  std::vector<int> todo{0};
  auto push_item = [&](int ref, const float* box, int h) {
    Item it;
    it.ref = ref;
    std::memcpy(it.box, box, sizeof it.box);
    for (int a = 0; a < 3; a++) it.c[a] = 0.5f * (box[a] + box[a + 3]);
    it.height = h;
    items.push_back(it);
  };
  while (!todo.empty()) {
    const int n = todo.back();
    todo.pop_back();
    const DevNode& N = s.nodes[n];
    for (int side = 0; side < 2; side++) {
      const int c = N.child[side];
      if (c < 0)
        push_item(c, &ref_box[(size_t)n * 6], 0);  // lone leaf: guarded by the parent's box
      else if (leaves[c] <= K)
        push_item(c, &ref_box[(size_t)c * 6], height[c]);
      else
        todo.push_back(c);
    }
  }
  // The node array is appended to; nothing else refers to the indices past the reference's.
  SahBuilder B{items, s.nodes};
  const char* pe = std::getenv("CENG795_RT_PAIRS");  // =0: visit two-leaf treelets (A/B)
  B.pairs = !(pe && pe[0] == '0');
  const int root = B.build(0, (int)items.size());
  Box u;
  for (const Item& it : items) u.grow(it.box);
  for (int a = 0; a < 3; a++) {
    s.accel_box[a] = widen_down(u.lo[a]);
    s.accel_box[a + 3] = widen_up(u.hi[a]);
  }
  s.accel_root = root;
  s.accel_depth = B.depth + 1;
  s.accel_items = (int)items.size();
  const char* we = std::getenv("CENG795_RT_WIDE");  // =0: keep the binary culling tree (A/B)
  if (!(we && we[0] == '0')) {
    int stack = 0;
    s.accel_root = collapse_wide(s.nodes, nn, root, stack);
    s.accel_depth = stack;
  }
}

int accel_treelet_leaves() {
  const char* e = std::getenv("CENG795_RT_TREELET");
  if (e && *e) return std::atoi(e);
  return kDefaultTreeletLeaves;
}

}  // namespace rt

namespace rt {

// Structural invariants of the culling tree the kernels' exactness argument relies on
// (DESIGN.md §4.2).  Returns "" when they hold, else a description of the first violation.
std::string check_accel(const HostScene& s, int K, long long stats[4]) {
  for (int i = 0; i < 4; i++) stats[i] = 0;
  if (s.accel_root < 0) return "";
  const int nref = s.accel_root & ~kWideTag;  // culling nodes follow the reference's
  const size_t nleaf = s.prims.size();
  auto box_of = [&](int ref_node) { return s.ancestry[ref_node].box; };
  // ancestry: each reference node's box is its parent's child slot; leaves point at holders
  for (int n = 0; n < nref; n++) {
    const DevNode& N = s.nodes[n];
    if (N.pad != 0) return "reference node " + std::to_string(n) + " is flagged as culling";
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
  // the slots of a culling node, binary (DevNode, kAccelNode) or wide (DevNode4, tagged)
  struct Slot {
    int ref;
    bool guard, pair;
    float box[6];
  };
  auto slots_of = [&](int node, std::vector<Slot>& out, std::string& err) {
    out.clear();
    const int idx = node & ~kWideTag;
    if (idx < nref || (size_t)idx >= s.nodes.size()) {
      err = "culling child is not a culling node";
      return;
    }
    if (node & kWideTag) {
      if ((size_t)idx + 1 >= s.nodes.size()) {
        err = "wide node past the end";
        return;
      }
      DevNode4 W;
      std::memcpy(&W, &s.nodes[idx], sizeof W);
      for (int k = 0; k < 4; k++) {
        if (!(W.flags & (kWideValid << k))) continue;
        Slot sl{W.child[k], (W.flags & (kWideGuard << k)) != 0, (W.flags & (kWidePair << k)) != 0, {}};
        for (int a = 0; a < 3; a++) {
          sl.box[a] = W.lo[a][k];
          sl.box[a + 3] = W.hi[a][k];
        }
        if (!sl.guard && !(sl.ref & kWideTag)) err = "inner slot of a wide node is not wide";
        out.push_back(sl);
      }
      if (out.size() < 2) err = "wide node with fewer than two slots";
    } else {
      const DevNode& N = s.nodes[idx];
      if (!(N.pad & kAccelNode)) {
        err = "culling child is not a culling node";
        return;
      }
      for (int side = 0; side < 2; side++) {
        Slot sl{N.child[side], (N.pad & (side ? kAccelGuard1 : kAccelGuard0)) != 0,
                (N.pad & (side ? kAccelPair1 : kAccelPair0)) != 0, {}};
        for (int a = 0; a < 3; a++) {
          sl.box[a] = N.lo[a][side];
          sl.box[a + 3] = N.hi[a][side];
        }
        out.push_back(sl);
      }
    }
  };
  std::vector<int> seen(nleaf, 0);
  long long lone = 0, items = 0;
  struct Frame {
    int node, depth;
  };
  std::vector<Frame> todo{{s.accel_root, 1}};
  // leaves of a reference subtree, and the union of guard boxes under a culling node
  auto ref_leaves = [&](int root, std::vector<int>& out) {
    std::vector<int> st{root};
    while (!st.empty()) {
      const int n = st.back();
      st.pop_back();
      for (int side = 0; side < 2; side++) {
        const int c = s.nodes[n].child[side];
        if (c >= 0) st.push_back(c); else out.push_back(~c);
      }
    }
  };
  std::vector<float> lo(s.nodes.size() * 3), hi(s.nodes.size() * 3);
  std::vector<int> order;  // culling nodes in preorder, for the bottom-up union pass
  std::vector<Slot> sl;
  std::string err;
  while (!todo.empty()) {
    const Frame f = todo.back();
    todo.pop_back();
    slots_of(f.node, sl, err);
    if (!err.empty()) return err;
    order.push_back(f.node);
    stats[2] = std::max<long long>(stats[2], f.depth);
    for (const Slot& x : sl) {
      const int c = x.ref;
      if (!x.guard) {
        if (x.pair) return "pair flag on an inner slot";
        todo.push_back({c, f.depth + 1});
        continue;
      }
      items++;
      const float* g = c >= 0 ? box_of(c) : box_of(s.ancestry[~c].leaf_parent);
      for (int a = 0; a < 6; a++)
        if (x.box[a] != g[a]) return "guard box differs from the reference box it stands for";
      std::vector<int> lv;
      if (c >= 0) {
        if (x.pair) return "leaf pair stored as a node";
        if (c >= nref) return "guarded child is not a reference node";
        ref_leaves(c, lv);
        if ((int)lv.size() > K) return "treelet larger than K";
      } else if (x.pair) {  // the two leaf children, in DFS order, of the guard's reference node
        if ((size_t)~c + 1 >= nleaf) return "leaf pair past the last leaf";
        const int holder = s.ancestry[~c].leaf_parent;
        if (holder < 0 || s.ancestry[~c + 1].leaf_parent != holder ||
            s.nodes[holder].child[0] != c || s.nodes[holder].child[1] != ~(~c + 1))
          return "leaf pair " + std::to_string(~c) + " is not one node's two leaves";
        lv.push_back(~c);
        lv.push_back(~c + 1);
      } else {
        lv.push_back(~c);
        lone++;
      }
      for (int l : lv)
        if (seen[l]++) return "leaf " + std::to_string(l) + " in two treelets";
    }
  }
  for (size_t l = 0; l < nleaf; l++)
    if (!seen[l]) return "leaf " + std::to_string(l) + " in no treelet";
  // containment: every inner slot box contains every guard box below it
  for (auto it = order.rbegin(); it != order.rend(); ++it) {
    slots_of(*it, sl, err);
    float ulo[3] = {INFINITY, INFINITY, INFINITY}, uhi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (const Slot& x : sl) {
      const size_t ci = (size_t)(x.ref & ~kWideTag) * 3;
      for (int a = 0; a < 3; a++) {
        const float l = x.guard ? x.box[a] : lo[ci + a], h = x.guard ? x.box[a + 3] : hi[ci + a];
        if (!x.guard && (x.box[a] > l || x.box[a + 3] < h))
          return "culling box does not contain the guard boxes below it";
        ulo[a] = std::min(ulo[a], l);
        uhi[a] = std::max(uhi[a], h);
      }
    }
    const size_t me = (size_t)(*it & ~kWideTag) * 3;
    for (int a = 0; a < 3; a++) {
      lo[me + a] = ulo[a];
      hi[me + a] = uhi[a];
    }
  }
  const size_t r0 = (size_t)nref * 3;
  for (int a = 0; a < 3; a++)
    if (s.accel_box[a] > lo[r0 + a] || s.accel_box[a + 3] < hi[r0 + a])
      return "culling root box does not contain the tree";
  stats[0] = items;
  stats[1] = (long long)order.size();
  stats[3] = lone;
  return "";
}

}  // namespace rt
