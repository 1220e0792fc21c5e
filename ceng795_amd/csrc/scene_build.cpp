// Host scene construction: the reference's object list and BVH, flattened for the GPU.
//
//   object list order  HW2/Scene.cpp:380-449 (meshes, loose triangles, spheres)
//   triangle ctor      HW2/Triangle.cpp:4-34 (flat normal, fmin/fmax box)
//   sphere box         HW2/Sphere.h:17-20
//   BVH build          HW2/Bounding_volume_hierarchy.cpp:3-29, create_bvh (.h:9-18)
//   box union          HW2/bounding_box.cpp:2-13
//
// The build must reproduce the reference's topology exactly: the leaf order it produces is
// the closest-hit tie-break order, and the set of boxes on each root-to-leaf path decides
// which leaves a ray may test at all.  Compiled with -ffp-contract=off (no FMA) so every
// fp32 expression rounds as on the reference's x86-64 SSE build.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <sstream>
#include <stdexcept>
#include <thread>
#include <utility>

#include "host_scene.h"

namespace rt {
namespace {

constexpr float kInf = std::numeric_limits<float>::infinity();

struct F3 {
  float x, y, z;
  float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
inline F3 operator+(F3 a, F3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline F3 operator-(F3 a, F3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline F3 operator*(F3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline F3 operator/(F3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline F3 cross(F3 a, F3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline F3 unit(F3 a) { return a / std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
inline F3 fmin3(F3 a, F3 b) { return {std::fmin(a.x, b.x), std::fmin(a.y, b.y), std::fmin(a.z, b.z)}; }
inline F3 fmax3(F3 a, F3 b) { return {std::fmax(a.x, b.x), std::fmax(a.y, b.y), std::fmax(a.z, b.z)}; }

struct Aabb {
  F3 lo{kInf, kInf, kInf};
  F3 hi{-kInf, -kInf, -kInf};
  F3 mid{0, 0, 0};  // (max + min) / 2, as Bounding_box::center
  static Aabb of(F3 lo, F3 hi) {
    Aabb b;
    b.lo = lo;
    b.hi = hi;
    b.mid = (hi + lo) / 2.0f;
    return b;
  }
  void grow(const Aabb& o) {  // bounding_box.cpp:2-13 (center recomputed on every expand)
    lo = fmin3(lo, o.lo);
    hi = fmax3(hi, o.hi);
    mid = (hi + lo) / 2.0f;
  }
  // n expands in a row: only the last center survives, so compute it once.
  void grow_all(const std::vector<int>& ids, int b, int e, const std::vector<struct Obj>& objs);
};

// The reference's Shape hierarchy as a tagged list.
enum ObjKind { kObjBvh, kObjMesh, kObjTri, kObjSphere };
struct Obj {
  ObjKind kind;
  Aabb box;
  int a = -1, b = -1;  // BVH children; Mesh: a = bvh root
  int axis = 0;        // BVH split dimension
  int leaf = -1;       // index into `leaves`
};

void Aabb::grow_all(const std::vector<int>& ids, int b, int e, const std::vector<Obj>& objs) {
  for (int i = b; i < e; i++) {
    lo = fmin3(lo, objs[ids[i]].box.lo);
    hi = fmax3(hi, objs[ids[i]].box.hi);
  }
  if (e > b) mid = (hi + lo) / 2.0f;
}

struct Builder {
  std::vector<Obj> objs;
  std::vector<LeafSource> leaves;
  std::vector<F3> normals;

  // BVH::BVH over ids[begin, end) (HW2/Bounding_volume_hierarchy.cpp:3-29), iteratively,
  // appending its nodes to `out`.  Leaf refs are object ids; refs to nodes of `out` are
  // encoded as node_ref(local index) and resolved by the caller.  Reads only leaf boxes.
  static int node_ref(int local) { return -2 - local; }
  void build_range(std::vector<int>& ids, int begin, int end, int axis, std::vector<Obj>& out) const {
    struct Range {
      int begin, end, axis, node;
    };
    std::vector<Range> todo;
    auto open = [&](int b, int e, int ax) {
      Obj o;
      o.kind = kObjBvh;
      o.axis = ax;
      o.box.grow_all(ids, b, e, objs);
      out.push_back(o);
      todo.push_back({b, e, ax, (int)out.size() - 1});
      return node_ref((int)out.size() - 1);
    };
    open(begin, end, axis);
    while (!todo.empty()) {
      const Range r = todo.back();
      todo.pop_back();
      const float split = out[r.node].box.mid[r.axis];
      int m = r.begin;
      for (int i = r.begin; i < r.end; i++)
        if (objs[ids[i]].box.mid[r.axis] < split) std::swap(ids[i], ids[m++]);
      if (m == r.begin || m == r.end) m = r.begin + (r.end - r.begin) / 2;
      const int next = (r.axis + 1) % 3;
      const int left = (r.begin + 1 == m) ? ids[r.begin] : open(r.begin, m, next);
      const int right = (m + 1 == r.end) ? ids[m] : open(m, r.end, next);
      out[r.node].a = left;
      out[r.node].b = right;
    }
  }

  // create_bvh + BVH::BVH over the object ids in `ids` (permuted in place like the reference).
  // The top levels are split on this thread; below them the independent subtrees are built
  // on worker threads (each writes its own node list), then spliced in.  Same topology and
  // boxes as a serial build: every node depends only on its own id range.
  int build(std::vector<int>& ids) {
    const int n = (int)ids.size();
    if (n == 0) return -1;
    if (n == 1) return ids[0];
    constexpr int kParallelDepth = 5, kParallelMin = 1 << 12;
    struct Task {
      int begin, end, axis, parent, side;
    };
    std::vector<Task> tasks;
    std::vector<Obj> top;
    // top levels, serially, into `top` (local refs), deferring deep ranges to tasks
    struct Range {
      int begin, end, axis, node, depth;
    };
    std::vector<Range> todo;
    auto open = [&](int b, int e, int ax, int depth) {
      Obj o;
      o.kind = kObjBvh;
      o.axis = ax;
      o.box.grow_all(ids, b, e, objs);
      top.push_back(o);
      todo.push_back({b, e, ax, (int)top.size() - 1, depth});
      return node_ref((int)top.size() - 1);
    };
    open(0, n, 0, 0);
    while (!todo.empty()) {
      const Range r = todo.back();
      todo.pop_back();
      const float split = top[r.node].box.mid[r.axis];
      int m = r.begin;
      for (int i = r.begin; i < r.end; i++)
        if (objs[ids[i]].box.mid[r.axis] < split) std::swap(ids[i], ids[m++]);
      if (m == r.begin || m == r.end) m = r.begin + (r.end - r.begin) / 2;
      const int next = (r.axis + 1) % 3;
      const int bounds[2][2] = {{r.begin, m}, {m, r.end}};
      for (int side = 0; side < 2; side++) {
        const int b = bounds[side][0], e = bounds[side][1];
        int ref;
        if (b + 1 == e) {
          ref = ids[b];
        } else if (r.depth + 1 >= kParallelDepth || e - b < kParallelMin) {
          tasks.push_back({b, e, next, r.node, side});
          ref = -1;  // patched below
        } else {
          ref = open(b, e, next, r.depth + 1);
        }
        (side == 0 ? top[r.node].a : top[r.node].b) = ref;
      }
    }
    std::vector<std::vector<Obj>> sub(tasks.size());
    {
      std::vector<std::thread> pool;
      const unsigned workers = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
      std::atomic<size_t> next_task{0};
      for (unsigned w = 0; w < workers && w < tasks.size(); w++)
        pool.emplace_back([&] {
          for (size_t t; (t = next_task++) < tasks.size();)
            build_range(ids, tasks[t].begin, tasks[t].end, tasks[t].axis, sub[t]);
        });
      for (auto& t : pool) t.join();
    }
    // splice: top nodes, then each task's nodes; resolve local refs to object ids
    auto splice = [&](std::vector<Obj>& nodes) {
      const int base = (int)objs.size();
      for (Obj& o : nodes) {
        if (o.a <= -2) o.a = base + (-2 - o.a);
        if (o.b <= -2) o.b = base + (-2 - o.b);
        objs.push_back(o);
      }
      return base;
    };
    const int top_base = splice(top);
    for (size_t t = 0; t < tasks.size(); t++) {
      const int root = splice(sub[t]);  // a task's first node is its root
      Obj& parent = objs[top_base + tasks[t].parent];
      (tasks[t].side == 0 ? parent.a : parent.b) = root;
    }
    return top_base;
  }
};

void fail(const std::string& m) { throw std::invalid_argument(m); }

}  // namespace

void camera_from_view(const float pos[3], const float gaze[3], const float up[3],
                      const float np[4], float dist, int w, int h, int ns, rt_camera& c) {
  // HW2/Camera.h:19-28
  const F3 e{pos[0], pos[1], pos[2]};
  const F3 g{gaze[0], gaze[1], gaze[2]};
  const F3 u0{up[0], up[1], up[2]};
  const F3 gn = unit(g);
  const F3 W{-gn.x, -gn.y, -gn.z};  // w = -(gaze.normalize())
  const F3 U = unit(cross(unit(u0), W));
  const F3 V = unit(cross(W, U));
  const float l = np[0], r = np[1], b = np[2], t = np[3];
  const F3 tl = ((e - W * dist) + U * l) + V * t;  // e - w*d + l*u + t*v, left to right
  const F3 su = U * ((r - l) / (float)w);
  const F3 sv = V * ((t - b) / (float)h);
  const F3* src[4] = {&e, &tl, &su, &sv};
  float* dst[4] = {c.e, c.top_left, c.s_u, c.s_v};
  for (int k = 0; k < 4; k++) {
    dst[k][0] = src[k]->x;
    dst[k][1] = src[k]->y;
    dst[k][2] = src[k]->z;
  }
  c.width = w;
  c.height = h;
  c.num_samples = ns;
}

namespace {

// One leaf of the flattened scene (DevPrim + normal/material record + its source), appended in
// leaf order; returns its leaf index.  Triangle: v0, a1 = v0 - v1, a2 = v0 - v2 as
// HW2/Triangle.cpp:43-44 computes them.
template <typename Vtx>
int append_leaf(HostScene& s, const LeafSource& ls, F3 n, Vtx vtx) {
  DevPrim p{};
  p.kind = ls.kind;
  p.material = ls.material;
  if (ls.kind == kPrimTriangle) {
    const F3 v0 = vtx(ls.i0), v1 = vtx(ls.i1), v2 = vtx(ls.i2);
    const F3 a1 = v0 - v1, a2 = v0 - v2;
    const float rec[9] = {v0.x, v0.y, v0.z, a1.x, a1.y, a1.z, a2.x, a2.y, a2.z};
    std::memcpy(p.v0, rec, sizeof rec);
    p.cx = a1.y * a2.z - a2.y * a1.z;  // c1.y*c2.z - c2.y*c1.z with c1 = a1, c2 = a2
    s.quot_ok &= quot_coord_ok(v0.x) & quot_coord_ok(v0.y) & quot_coord_ok(v0.z);
  } else {
    std::memcpy(p.v0, ls.center, 12);
    p.a1[0] = ls.radius;
  }
  const int index = (int)s.prims.size();
  s.prims.push_back(p);
  int mat_bits = ls.material;
  float mat_f;
  std::memcpy(&mat_f, &mat_bits, 4);
  s.normals.insert(s.normals.end(), {n.x, n.y, n.z, mat_f});
  s.leaf_src.push_back(ls);
  return index;
}

// rt_scene_desc with the caller's own BVH (bvh_*, ABI 7): adopted as given.  The walk checks
// that nodes are numbered in DFS preorder and leaves in DFS (left-first) order, each exactly
// once, and that every primitive of the object lists is exactly one leaf.
template <typename Vtx>
void adopt_tree(const rt_scene_desc& d, HostScene& s, const std::vector<LeafSource>& objects,
                const std::vector<F3>& normals, Vtx vtx) {
  const int nn = d.bvh_num_nodes, nl = d.bvh_num_leaves;
  if (nn < 0 || nl <= 0) fail("bvh_num_nodes < 0 or bvh_num_leaves <= 0");
  if (!d.bvh_leaf_object) fail("bvh_leaf_object == NULL");
  if (nn > 0 && (!d.bvh_children || !d.bvh_boxes)) fail("bvh_children / bvh_boxes == NULL");
  if ((size_t)nl != objects.size())
    fail("bvh_num_leaves (" + std::to_string(nl) + ") is not the number of primitives (" +
         std::to_string(objects.size()) + ")");
  if (nn != nl - 1) fail("a binary tree of " + std::to_string(nl) + " leaves has " +
                         std::to_string(nl - 1) + " internal nodes, not " + std::to_string(nn));
  std::vector<char> used(objects.size(), 0);
  for (int k = 0; k < nl; k++) {
    const int o = d.bvh_leaf_object[k];
    if (o < 0 || (size_t)o >= objects.size()) fail("bvh_leaf_object out of range");
    if (used[o]++) fail("primitive " + std::to_string(o) + " is two leaves");
    F3 n = normals[o];
    if (d.bvh_leaf_normals && objects[o].kind == kPrimTriangle)
      n = {d.bvh_leaf_normals[3 * k], d.bvh_leaf_normals[3 * k + 1], d.bvh_leaf_normals[3 * k + 2]};
    append_leaf(s, objects[o], n, vtx);
  }
  if (nn == 0) {  // the root is the one primitive (BVH::create_bvh, .h:13-14)
    s.root_kind = s.prims[0].kind == kPrimTriangle ? kRootTriangle : kRootSphere;
    s.root_ref = 0;
    s.depth = 0;
    return;
  }
  s.root_kind = kRootNode;
  s.root_ref = 0;
  std::memcpy(s.root_box, d.bvh_boxes, sizeof s.root_box);
  s.nodes.assign((size_t)nn, DevNode{});
  const float kAll[6] = {-1e30f, -1e30f, -1e30f, 1e30f, 1e30f, 1e30f};  // a leaf's slot
  int next_node = 1, next_leaf = 0;
  s.depth = 1;
  struct Frame {
    int node, side, depth;
  };
  std::vector<Frame> st{{0, 0, 1}};
  while (!st.empty()) {
    Frame& f = st.back();
    if (f.side == 2) {
      st.pop_back();
      continue;
    }
    const int side = f.side++, node = f.node, depth = f.depth;
    const int c = d.bvh_children[2 * node + side];
    DevNode& dn = s.nodes[node];
    dn.axis = (depth - 1) % 3;
    const float* b = kAll;
    if (c >= 0) {
      if (c != next_node) fail("bvh nodes are not numbered in DFS preorder (node " +
                               std::to_string(node) + " child " + std::to_string(c) + ")");
      next_node++;
      b = d.bvh_boxes + 6 * (size_t)c;
      dn.child[side] = c;
      s.depth = std::max(s.depth, depth + 1);
      st.push_back({c, 0, depth + 1});  // invalidates f
    } else {
      if (~c != next_leaf) fail("bvh leaves are not numbered in DFS order (leaf " +
                                std::to_string(~c) + ")");
      next_leaf++;
      dn.child[side] = c;
    }
    for (int a = 0; a < 3; a++) {
      s.nodes[node].lo[a][side] = b[a];
      s.nodes[node].hi[a][side] = b[a + 3];
    }
  }
  if (next_node != nn || next_leaf != nl) fail("bvh tree does not reach every node and leaf");
}

}  // namespace

void build_host_scene(const rt_scene_desc& d, HostScene& s) {
  if (d.num_vertices < 0 || d.num_materials < 0 || d.num_lights < 0 || d.num_cameras < 0 ||
      d.num_meshes < 0 || d.num_triangles < 0 || d.num_spheres < 0)
    fail("negative count in scene description");
  if (d.num_vertices && !d.vertices) fail("vertices == NULL");
  std::memcpy(s.background, d.background, sizeof s.background);
  std::memcpy(s.ambient, d.ambient_light, sizeof s.ambient);
  s.eps = d.shadow_ray_epsilon;
  s.max_depth = d.max_recursion_depth;
  if (s.max_depth < 0) fail("MaxRecursionDepth < 0");
  s.materials.clear();
  for (int i = 0; i < d.num_materials; i++) {
    const rt_material& m = d.materials[i];
    DevMaterial dm{};
    std::memcpy(dm.ambient, m.ambient, 12);
    std::memcpy(dm.diffuse, m.diffuse, 12);
    std::memcpy(dm.specular, m.specular, 12);
    std::memcpy(dm.mirror, m.mirror, 12);
    std::memcpy(dm.transparency, m.transparency, 12);
    dm.refraction_index = m.refraction_index;
    dm.phong_exponent = m.phong_exponent;
    s.materials.push_back(dm);
  }
  s.lights.clear();
  for (int i = 0; i < d.num_lights; i++) {
    DevLight L{};
    std::memcpy(L.position, d.lights[i].position, 12);
    std::memcpy(L.intensity, d.lights[i].intensity, 12);
    s.lights.push_back(L);
  }
  s.cameras.assign(d.cameras, d.cameras + d.num_cameras);
  for (const rt_camera& c : s.cameras)
    if (c.width <= 0 || c.height <= 0 || c.num_samples <= 0) fail("bad camera resolution");
  if (s.image_names.size() != s.cameras.size()) s.image_names.assign(s.cameras.size(), "");

  auto vtx = [&](int i) -> F3 {
    if (i < 0 || i >= d.num_vertices) fail("vertex index out of range");
    return {d.vertices[3 * i], d.vertices[3 * i + 1], d.vertices[3 * i + 2]};
  };
  auto check_material = [&](int m) {
    if (m < 0 || m >= d.num_materials) fail("material id out of range");
  };

  if (d.bvh_num_leaves > 0 || d.bvh_num_nodes > 0) {
    // the caller's own tree: the primitives in object-list order, then adopt_tree
    std::vector<LeafSource> objects;
    std::vector<F3> normals;
    auto tri = [&](int i0, int i1, int i2, int mat) {
      check_material(mat);
      const F3 v0 = vtx(i0), v1 = vtx(i1), v2 = vtx(i2);
      LeafSource ls{};
      ls.kind = kPrimTriangle;
      ls.i0 = i0;
      ls.i1 = i1;
      ls.i2 = i2;
      ls.material = mat;
      objects.push_back(ls);
      normals.push_back(unit(cross(v1 - v0, v2 - v0)));  // Triangle.cpp:14
    };
    long long fb = 0;
    for (int m = 0; m < d.num_meshes; m++) {
      const int nf = d.mesh_face_count[m];
      if (nf <= 0) fail("mesh without faces (the reference dereferences a NULL bvh)");
      for (int f = 0; f < nf; f++) {
        const int* idx = d.mesh_faces + 3 * (fb + f);
        tri(idx[0], idx[1], idx[2], d.mesh_material[m]);
      }
      fb += nf;
    }
    for (int t = 0; t < d.num_triangles; t++) {
      const int* idx = d.triangle_indices + 3 * t;
      tri(idx[0], idx[1], idx[2], d.triangle_material[t]);
    }
    for (int k = 0; k < d.num_spheres; k++) {
      check_material(d.sphere_material[k]);
      const F3 c = vtx(d.sphere_center[k]);
      LeafSource ls{};
      ls.kind = kPrimSphere;
      ls.center[0] = c.x;
      ls.center[1] = c.y;
      ls.center[2] = c.z;
      ls.radius = d.sphere_radius[k];
      ls.material = d.sphere_material[k];
      objects.push_back(ls);
      normals.push_back({0, 0, 0});
    }
    s.nodes.clear();
    s.prims.clear();
    s.normals.clear();
    s.leaf_src.clear();
    s.quot_ok = 1;
    adopt_tree(d, s, objects, normals, vtx);
    return;
  }

  Builder B;
  auto add_triangle = [&](int i0, int i1, int i2, int mat) {
    check_material(mat);
    const F3 v0 = vtx(i0), v1 = vtx(i1), v2 = vtx(i2);
    Obj o;
    o.kind = kObjTri;
    o.box = Aabb::of(fmin3(fmin3(v0, v1), v2), fmax3(fmax3(v0, v1), v2));
    o.leaf = (int)B.leaves.size();
    LeafSource ls{};
    ls.kind = kPrimTriangle;
    ls.i0 = i0;
    ls.i1 = i1;
    ls.i2 = i2;
    ls.material = mat;
    B.leaves.push_back(ls);
    B.normals.push_back(unit(cross(v1 - v0, v2 - v0)));
    B.objs.push_back(o);
    return (int)B.objs.size() - 1;
  };

  std::vector<int> top;
  long long face_base = 0;
  for (int m = 0; m < d.num_meshes; m++) {
    const int nf = d.mesh_face_count[m];
    if (nf <= 0) fail("mesh without faces (the reference dereferences a NULL bvh)");
    std::vector<int> tris;
    tris.reserve(nf);
    for (int f = 0; f < nf; f++) {
      const int* idx = d.mesh_faces + 3 * (face_base + f);
      tris.push_back(add_triangle(idx[0], idx[1], idx[2], d.mesh_material[m]));
    }
    face_base += nf;
    const int root = B.build(tris);
    Obj mo;
    mo.kind = kObjMesh;
    mo.a = root;
    mo.box = B.objs[root].box;
    B.objs.push_back(mo);
    top.push_back((int)B.objs.size() - 1);
  }
  for (int t = 0; t < d.num_triangles; t++) {
    const int* idx = d.triangle_indices + 3 * t;
    top.push_back(add_triangle(idx[0], idx[1], idx[2], d.triangle_material[t]));
  }
  for (int k = 0; k < d.num_spheres; k++) {
    check_material(d.sphere_material[k]);
    const F3 c = vtx(d.sphere_center[k]);
    const float r = d.sphere_radius[k];
    const F3 rr{r, r, r};
    Obj o;
    o.kind = kObjSphere;
    o.box = Aabb::of(c - rr, c + rr);
    o.leaf = (int)B.leaves.size();
    LeafSource ls{};
    ls.kind = kPrimSphere;
    ls.center[0] = c.x;
    ls.center[1] = c.y;
    ls.center[2] = c.z;
    ls.radius = r;
    ls.material = d.sphere_material[k];
    B.leaves.push_back(ls);
    B.normals.push_back({0, 0, 0});
    B.objs.push_back(o);
    top.push_back((int)B.objs.size() - 1);
  }
  if (top.empty()) fail("scene has no objects (the reference dereferences a NULL bvh)");
  int root = B.build(top);
  while (B.objs[root].kind == kObjMesh) root = B.objs[root].a;  // Mesh::intersect delegates

  // ---- flatten: DFS preorder nodes, DFS-order leaves, meshes spliced out.
  s.nodes.clear();
  s.prims.clear();
  s.normals.clear();
  s.leaf_src.clear();
  s.quot_ok = 1;
  auto resolve = [&](int id) {
    while (B.objs[id].kind == kObjMesh) id = B.objs[id].a;
    return id;
  };
  auto emit_leaf = [&](int id) {
    const Obj& o = B.objs[id];
    return ~append_leaf(s, B.leaves[o.leaf], B.normals[o.leaf], vtx);
  };
  auto put_box = [](float* dst, const Aabb& b) {
    dst[0] = b.lo.x;
    dst[1] = b.lo.y;
    dst[2] = b.lo.z;
    dst[3] = b.hi.x;
    dst[4] = b.hi.y;
    dst[5] = b.hi.z;
  };
  auto put_child_box = [](DevNode& n, int side, const Aabb& b) {
    for (int a = 0; a < 3; a++) {
      n.lo[a][side] = b.lo[a];
      n.hi[a][side] = b.hi[a];
    }
  };
  if (B.objs[root].kind != kObjBvh) {
    s.root_kind = B.objs[root].kind == kObjTri ? kRootTriangle : kRootSphere;
    s.root_ref = ~emit_leaf(root);
    s.depth = 0;
  } else {
    s.root_kind = kRootNode;
    s.root_ref = 0;
    put_box(s.root_box, B.objs[root].box);
    struct Frame {
      int obj, node, stage, depth;
    };
    std::vector<Frame> st;
    s.nodes.push_back(DevNode{});
    st.push_back({root, 0, 0, 1});
    s.depth = 1;
    while (!st.empty()) {
      Frame& f = st.back();
      if (f.stage == 2) {
        st.pop_back();
        continue;
      }
      const int side = f.stage++;
      const int child = resolve(side == 0 ? B.objs[f.obj].a : B.objs[f.obj].b);
      const int node = f.node, depth = f.depth;
      s.nodes[node].axis = B.objs[f.obj].axis;
      if (B.objs[child].kind == kObjBvh) {
        const int idx = (int)s.nodes.size();
        s.nodes.push_back(DevNode{});
        put_child_box(s.nodes[node], side, B.objs[child].box);
        s.nodes[node].child[side] = idx;
        if (depth + 1 > s.depth) s.depth = depth + 1;
        st.push_back({child, idx, 0, depth + 1});  // invalidates f
      } else {
        const int ref = emit_leaf(child);
        s.nodes[node].child[side] = ref;
        // A leaf has no box in the reference (every ray in the node tests it).  Its slot gets
        // a +-1e30 box that every ray with a normalised direction accepts by a wide margin in
        // the kernels' slab test, so leaf and inner children share one decision path.
        Aabb all;
        all.lo = {-1e30f, -1e30f, -1e30f};
        all.hi = {1e30f, 1e30f, 1e30f};
        put_child_box(s.nodes[node], side, all);
      }
    }
  }
}

std::string dump_bvh(const HostScene& s) {
  std::ostringstream os;
  auto hex = [](float f) {
    unsigned u;
    std::memcpy(&u, &f, 4);
    char b[16];
    std::snprintf(b, sizeof b, "%08x", u);
    return std::string(b);
  };
  auto leaf = [&](int li) {
    const LeafSource& l = s.leaf_src[li];
    if (l.kind == kPrimTriangle)
      os << "T " << l.i0 << " " << l.i1 << " " << l.i2 << " " << l.material << "\n";
    else
      os << "S " << hex(l.center[0]) << " " << hex(l.center[1]) << " " << hex(l.center[2])
         << " " << hex(l.radius) << " " << l.material << "\n";
  };
  if (s.root_kind != kRootNode) {
    leaf(s.root_ref);
    return os.str();
  }
  struct Item {
    int ref;
    float box[6];
  };
  std::vector<Item> st{{0, {s.root_box[0], s.root_box[1], s.root_box[2], s.root_box[3],
                            s.root_box[4], s.root_box[5]}}};
  while (!st.empty()) {
    Item it = st.back();
    st.pop_back();
    if (it.ref < 0) {
      leaf(~it.ref);
      continue;
    }
    os << "N";
    for (int k = 0; k < 6; k++) os << " " << hex(it.box[k]);
    os << "\n";
    const DevNode& n = s.nodes[it.ref];
    for (int side = 1; side >= 0; side--)
      st.push_back({n.child[side], {n.lo[0][side], n.lo[1][side], n.lo[2][side], n.hi[0][side],
                                    n.hi[1][side], n.hi[2][side]}});
  }
  return os.str();
}

}  // namespace rt
