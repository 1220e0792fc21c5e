// Host-side scene: validation, the reference-identical BVH build and its flattening into the
// device layout of rt_internal.h.  Untimed, like the reference's Scene constructor.
#ifndef CENG795_HOST_SCENE_H_
#define CENG795_HOST_SCENE_H_

#include <string>
#include <vector>

#include "../../include/ceng795_rt.h"
#include "rt_internal.h"

namespace rt {

struct LeafSource {  // what the leaf was in the reference object list (for BVH dumps)
  int kind;          // kPrimTriangle / kPrimSphere
  int i0, i1, i2;    // triangle vertex ids (0-based)
  float center[3], radius;
  int material;
};

struct HostScene {
  // scalars / lists copied from the description
  float background[3] = {0, 0, 0};
  float ambient[3] = {0, 0, 0};
  float eps = 0.001f;
  int max_depth = 0;
  std::vector<DevMaterial> materials;
  std::vector<DevLight> lights;
  std::vector<rt_camera> cameras;
  std::vector<std::string> image_names;
  // flattened acceleration structure
  std::vector<DevNode> nodes;
  std::vector<DevPrim> prims;
  std::vector<float> normals;  // 4 per leaf
  std::vector<LeafSource> leaf_src;
  int root_kind = kRootNode;
  int root_ref = 0;
  float root_box[6] = {0, 0, 0, 0, 0, 0};
  int depth = 0;  // internal-node levels
  // culling tree over reference treelets (accel_build.cpp), FAST traversal only
  int accel_root = -1;   // tagged index into nodes (8-wide nodes follow the reference's), -1 = none
  int accel_depth = 0;   // stack entries a traversal from accel_root can need
  int accel_items = 0;   // treelets
  float accel_box[6] = {0, 0, 0, 0, 0, 0};
  // per-axis outward margin of every culling box: 2^-18 * the largest coordinate magnitude of
  // the scene, its cameras and every ray origin; it lets the kernels cull on
  // a plain slab test
  double cull_margin[3] = {0, 0, 0};
  std::vector<DevLeaf> leaves;        // culling-tree order (DevLeaf)
  std::vector<DevAncestry> ancestry;  // max(nodes, leaves) entries, see DevAncestry
  int quot_ok = 0;  // every triangle v0 coordinate passes quot_coord_ok (rt_internal.h)
};

// Cuts the reference tree into treelets of <= K leaves (K = 1: lone leaves; 2: also leaf
// pairs; K <= 0: no culling tree) and appends an 8-wide SAH tree over them.  Leaves the
// reference nodes, leaves and tie-break order untouched.
void build_accel(HostScene& s, int K);
// Invariants of the culling tree (coverage, guard boxes, conservative containment with the
// margin, child layout, ancestry); "" if they hold.  stats: treelets, culling nodes, culling
// depth, lone-leaf treelets.
std::string check_accel(const HostScene& s, int K, long long stats[4]);

// Builds `out` from `desc`; throws std::invalid_argument on a bad description.
void build_host_scene(const rt_scene_desc& desc, HostScene& out);

// Preorder dump in oracle/ref/ref_harness.cpp's format (without the Mesh "M" markers, which
// the flattened layout splices away).
std::string dump_bvh(const HostScene& s);

// XML ingest (HW2/Scene.cpp:198-451) into a description whose arrays live in `storage`.
struct XmlSceneStorage {
  std::vector<float> vertices;
  std::vector<rt_material> materials;
  std::vector<rt_point_light> lights;
  std::vector<rt_camera> cameras;
  std::vector<std::string> image_names;
  std::vector<int> mesh_material, mesh_face_count, mesh_faces;
  std::vector<int> triangle_indices, triangle_material;
  std::vector<int> sphere_center, sphere_material;
  std::vector<float> sphere_radius;
};
void load_scene_xml(const std::string& path, XmlSceneStorage& st, rt_scene_desc& desc);

void camera_from_view(const float pos[3], const float gaze[3], const float up[3],
                      const float np[4], float dist, int w, int h, int ns, rt_camera& c);

}  // namespace rt

#endif
