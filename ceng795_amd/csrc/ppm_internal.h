// Device-side layout of the photon-mapping (PPM) path, shared by the host builder
// (ppm_scene.cpp) and the kernels (ppm_kernels.hip).  Reference: /root/reference/PPM.
#ifndef CENG795_PPM_INTERNAL_H_
#define CENG795_PPM_INTERNAL_H_

#include <cstdint>

namespace ppm {

constexpr int kMatDiffuse = 0, kMatMirror = 1, kMatRefractive = 2;  // Material.h:7
constexpr int kObjSphere = 0, kObjInstance = 1;
constexpr int kTopStack = 48;   // per-lane traversal stacks (host checks the BVH depths)
constexpr int kMeshStack = 64;
constexpr int kLdsStack = 12;   // ... in LDS when both BVHs fit this many levels (PScene::lds_stack)
constexpr int kPpmThreads = 256;  // workgroup size of the eye and photon kernels
constexpr int kEyeStack = 24;   // eye-ray tree: <= MaxRecursionDepth (<= 20) + 1 pending
constexpr int kStatSlots = 36;  // device counter words (ppm_collect_stats)
constexpr int kMaxCells = 27;
constexpr int kGroupBits = 27;  // expansion keys: group | multiplicity << kGroupBits
constexpr int kRepBits = 5;  // multiplicity bits next to a deposit index (kMaxCells < 32)
constexpr unsigned kRepMask = (1u << kRepBits) - 1u;
constexpr long long kMaxBatchDeposits = 1ll << (32 - kRepBits);   // hash cells a hit point's radius box can touch (3 per axis)

// PPM/include/Material.h (+ type resolved as Material.cpp:57-63)
struct PMaterial {
  float diffuse[3], specular[3], mirror[3], transparency[3];
  int type, brdf_id;
  float refraction_index, phong;
};

// BVH node of either level (top-level over objects, or one mesh's triangles); DFS preorder.
// child >= 0: node index; child < 0: leaf ~index (object or triangle).
struct PNode {
  float lo[3], hi[3];
  int child[2];
};

// Top-level object: a Sphere (Sphere.cpp) or a Mesh_instance (Mesh.h:61-117), with the
// inverse and inverse-transpose of its transformation (3x4 / 3x3, row-major).
struct PObject {
  int kind, material, mesh, refractive;
  float lo[3], hi[3];  // world bounding box (Mesh_instance::intersect tests it first)
  float inv[12];
  float nrm[9];
  float center[3], radius;
};

struct PTriangle {  // Mesh_triangle: absolute vertex ids, flat normal, shading mode
  int v[3];
  int smooth;
  float normal[3];
  float pad;
};

struct PMesh {
  int root;  // >= 0 mesh node, < 0 ~triangle (a one-triangle mesh)
};

// One eye-pass hit point (PPM/include/Hit_point.h), written in the single-threaded reference
// order: pixels row-major, each pixel's eye-ray tree depth first.
struct PHitPoint {
  float pos[3], normal[3], w_o[3], att[3];
  int material, pixel;
  float weight, pad;
};

// Hash-grid parameters of build_hash_grid (PPM/src/Scene.cpp:53-93).
struct PGrid {
  float bmin[3], bmax[3];  // hit_point_bbox after the radius padding
  float radius;            // initial radius
  float hash_scale;
  unsigned num_hash;
  unsigned pad;
};

// Diffuse photon hit (photon_trace, Scene.cpp:122-170): what a hit point update needs.
struct PDeposit {
  float x[3], normal[3], w_i[3], flux[3];
};

struct PScene {  // device pointers + scalars, passed by value to every kernel
  const PNode* top_nodes;
  const PObject* objects;
  const PNode* mesh_nodes;
  const PTriangle* triangles;
  const PMesh* meshes;
  const float* vpos;
  const float* vnormal;
  const PMaterial* materials;
  int top_root;  // >= 0 node, < 0 ~object, INT_MIN = empty scene
  int max_depth;
  float eps;
  float light_pos[3], light_intensity[3];
  int diag;  // timing experiments only (CENG795_PPM_DIAG): 1 = skip the update recurrence
  int compact_seg;  // update pass: deposits per compaction segment (ppm_set_update_segment)
  int lds_stack;    // 1: both BVHs fit kLdsStack levels, the traversal stacks live in LDS
};

struct PCamera {
  float e[3], top_left[3], s_u[3], s_v[3];
  int width, height, samples;
};

}  // namespace ppm

#endif
