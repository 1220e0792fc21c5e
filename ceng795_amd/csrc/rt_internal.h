// Internal layouts shared by the host scene builder and the HIP kernels.
//
// HBM layout (see DESIGN.md §Data layout):
//   nodes   : DevNode[num_nodes]    64 B, BVH2 internal nodes in DFS preorder; each holds
//                                    both CHILD boxes, so one s_load_dwordx16 per visit tests
//                                    both children (the reference tests a node's own box on
//                                    entry, HW2/Bounding_volume_hierarchy.cpp:32-35 — same set).
//   prims   : DevPrim[num_leaves]   48 B, leaves in DFS order: leaf index == the reference's
//                                    DFS leaf order, which is the closest-hit tie-break key.
//   normals : float4[num_leaves]     flat normal (Triangle.cpp:14) + material id, read once
//                                    per pixel for the winning leaf only.
#ifndef CENG795_RT_INTERNAL_H_
#define CENG795_RT_INTERNAL_H_

#include <stdint.h>

namespace rt {

constexpr int kTile = 8;          // one wavefront = one 8x8 pixel packet
constexpr int kWavesPerBlock = 4; // 256-thread workgroups
constexpr int kLaneStack = 64;    // per-wave traversal stack held one entry per VGPR lane
constexpr int kCounterRows = 64;  // ray-counter rows (spread atomics)
constexpr int kCounterWidth = 16; // u64 counters per row
// counter columns
enum : int {
  kCntPrimary = 0, kCntShadow = 1, kCntSecondary = 2, kCntHits = 3,
  // RT_DIAG builds only: packet-level traversal work
  kCntPrimNodes = 4, kCntPrimNodeLanes = 5, kCntPrimLeaves = 6, kCntPrimLeafLanes = 7,
  kCntShadNodes = 8, kCntShadNodeLanes = 9, kCntShadLeaves = 10, kCntShadLeafLanes = 11,
  kCntExactBox = 12,
  kCntPrimTopWide = 13,  // RT_DIAG: primary visits of wide nodes in the top kWideTopLevels levels
  // RT_DIAG builds: the node visits above that were 4-wide culling nodes (128 B each)
  kCntPrimWide = 14, kCntShadWide = 15
};

// DevNode::pad of the culling-tree nodes (accel_build.cpp); reference nodes have pad == 0.
// Guard bit set: that child is a treelet root (node index or ~leaf) behind a reachability
// guard; clear: an inner culling node tested conservatively.
// culling nodes (accel_build.cpp): pad = kAccelNode | guard bits | leaf-pair bits.  A guarded
// child with its pair bit set is a treelet of two leaves, stored as ~first leaf (its second
// leaf is the next one in DFS order): the kernels queue both leaf tests at once instead of
// visiting the treelet's root, whose own box is the guard already tested.
enum : int32_t { kAccelGuard0 = 1, kAccelGuard1 = 2, kAccelNode = 4, kAccelPair0 = 8, kAccelPair1 = 16 };
constexpr int kDefaultTreeletLeaves = 2;

struct alignas(16) DevNode {
  // Both CHILD boxes, interleaved per coordinate ([axis][child]) so one packed-fp32 op
  // (v_pk_add_f32 / v_pk_mul_f32) works on both children.  Unused for a leaf child.
  float lo[3][2];
  float hi[3][2];
  int32_t child[2];  // >= 0: internal node index; < 0: leaf index ~child
  int32_t axis;      // split dimension of THIS node (Bounding_volume_hierarchy.cpp:8)
  int32_t pad;       // 0: reference node; else kAccelNode | guard bits | pair bits
};
static_assert(sizeof(DevNode) == 64, "node must be one 64-byte scalar load");

// 4-wide culling node (accel_build.cpp, collapse of the binary SAH tree): two consecutive
// DevNode slots of `nodes`, referred to as (index of the first slot) | kWideTag, so a stack
// entry says which kind it holds before the fetch.  Slot c of a wide node is valid when
// flags bit kWideValid << c is set; it is then either a guarded treelet (bit kWideGuard << c:
// child = ~leaf, with kWidePair << c the leaf pair ~child, ~child + 1, or a reference node
// for treelets of more than two leaves) tested with the guard rule, or an inner wide node
// (child = its tagged index) tested conservatively.
constexpr int32_t kWideTag = 1 << 30;
enum : int32_t { kWideGuard = 1, kWidePair = 16, kWideValid = 256 };
// a wide node in the top kWideTopLevels levels of the tree (the RT_DIAG build counts the visits;
// would those nodes pay for LDS residency?)
constexpr int32_t kWideTop = 1 << 12;
constexpr int kWideTopLevels = 3;
struct alignas(16) DevNode4 {
  float lo[3][4];
  float hi[3][4];
  int32_t child[4];
  int32_t flags;  // kWideGuard << c | kWidePair << c | kWideValid << c
  int32_t pad[3];
};
static_assert(sizeof(DevNode4) == 2 * sizeof(DevNode), "a wide node is two node slots");

enum PrimKind : int32_t { kPrimTriangle = 0, kPrimSphere = 1 };

struct alignas(16) DevPrim {
  // triangle: v0, a1 = v0 - v1, a2 = v0 - v2 (Triangle.cpp:43-44, same fp32 rounding)
  // sphere:   v0 = center, a1[0] = radius
  float v0[3];
  float a1[3];
  float a2[3];
  int32_t kind;
  int32_t material;
  float cx;  // triangle: a1.y*a2.z - a2.y*a1.z (the d-free minor of Triangle.h:35-37)
};
static_assert(sizeof(DevPrim) == 48, "prim record is three 16-byte loads");

// Range in which the triangle test's three divisions (v0 - o) / det may share one reciprocal
// (tri_quotients in rt_kernels.hip): a coordinate is 0 or 2^-26 <= |x| <= 2^48, so every
// difference v0 - o is 0 or 2^-49 <= |v0 - o| <= 2^49.
inline bool quot_coord_ok(float x) {
  const float a = x < 0 ? -x : x;
  return a == 0.0f || (a >= 0x1p-26f && a <= 0x1p48f);
}

// Reference ancestry for the culling tree's exact guard (accel_build.cpp): entry i holds
// reference node i's own box and parent (-1 at the root), and the node holding leaf i.
struct alignas(16) DevAncestry {
  float box[6];
  int32_t parent;
  int32_t leaf_parent;
};
static_assert(sizeof(DevAncestry) == 32, "");

struct DevMaterial {  // HW2/Material.h
  float ambient[3], diffuse[3], specular[3], mirror[3], transparency[3];
  float refraction_index, phong_exponent;
  float pad[3];
};
static_assert(sizeof(DevMaterial) == 80, "");

struct DevLight {
  float position[3];
  float intensity[3];
  float pad[2];
};

// Primary-hit record, 8 B per pixel: x = DFS leaf index (-1 miss, -2 outside the image),
// y = the bits of t.  As one little-endian u64 it is the key (t bits << 32) | leaf whose
// minimum is the reference's (t, DFS leaf) rule (rt_kernels.hip, batch_flush).
struct alignas(8) int2_t {
  int32_t x, y;
};


enum RootKind : int32_t { kRootNode = 0, kRootTriangle = 1, kRootSphere = 2 };

constexpr unsigned kMinstdM = 2147483647u;  // minstd_rand0 modulus (std::default_random_engine)
constexpr unsigned kMinstdA = 16807u;

// Resolve of the Gaussian MSAA splat: samples[s][h][w][3] -> out[h][w][3] = color / weight.
struct MsaaResolveParams {
  const float* samples;
  float* out;
  int width, height, n;
  unsigned long long seed;
  int row_lo, row_hi;  // the rows resolved: [row_lo, row_hi) (a multi-device band)
};

// Untile of a multi-device frame (rt_api.hip render_multi): the frame's tiles were dealt
// round-robin over `devices` (tile t -> device t mod devices, slot position t / devices) and
// gathered as recv[devices][slot][64 pixels][3]; writes the selected rows of the row-major
// frame out[h][w][3] (logical row k = image row row0 + k*row_stride).
struct UntileParams {
  const float* recv;
  float* out;
  int width, row0, row_stride, rows, tiles_x, tiles_total, devices, slot;
};

// Words of the per-stream schedule buffer for a launch of `tiles` selected tiles: tile costs
// + the unit order lists (order_layout in rt_kernels.hip stays within this).
inline unsigned long long sched_words_for(unsigned long long tiles) { return 10 * tiles + 64; }

struct RenderParams {
  const DevNode* nodes;
  // the wide nodes again with every slot box relative to this camera's origin, RN(b - e) per
  // coordinate (upload_replica), indexed like `nodes`; null when unavailable.  The primary
  // kernel's wide visits read them: the slab test's b - o is then precomputed (same bits).
  const DevNode* rel_nodes;
  const DevPrim* prims;
  const float* normals;  // float4 per leaf: nx ny nz material(bits)
  const DevMaterial* materials;
  const DevLight* lights;
  int num_lights;
  int max_depth;
  float background[3];
  float ambient[3];
  float eps;
  int root_kind;
  int root_ref;           // kRootNode: node index; else leaf index
  float root_box[6];
  // culling tree (FAST traversal): root node index or -1, its conservative box, and the
  // reference ancestry a guard walks when its fast test cannot decide
  int accel_root;
  float accel_box[6];
  // every triangle's v0 coordinate is 0 or in [2^-26, 2^48] (quot_coord_ok): the triangle
  // test may take the shared-reciprocal quotient path (rt_kernels.hip, tri_quotients)
  int quot_ok;
  const struct DevAncestry* anc;
  // camera (rt_camera)
  float cam_e[3], cam_tl[3], cam_su[3], cam_sv[3];
  int width, height;
  // row subset: image row of logical row k = row0 + k*row_stride
  int row0, row_stride, rows;
  // tiles over (rows x width), row-major; this launch does tile_begin + i*tile_step
  int tiles_x, tiles_total, tile_begin, tile_step, num_sel_tiles;
  int tile_major;
  int tile_block;  // traversal kernels: workgroups take 2-D blocks of tiles (rt_kernels.hip)
  // jittered MSAA (HW2/Scene.cpp:32-69): 0 = pixel centres; else this launch traces sample
  // msaa_s = x*n + y of every pixel, whose minstd_rand0 draws 2s+1, 2s+2 are
  // u0 * msaa_mul[0], u0 * msaa_mul[1] (mod 2^31-1), u0 the pixel's seeded state.
  int msaa_n, msaa_s;
  unsigned msaa_mul[2];
  unsigned long long msaa_seed;
  float* out;
  int2_t* hits;   // num_sel_tiles * 64 records {t bits, leaf}: trace_primary -> shadow, shade
  unsigned* occ;  // num_sel_tiles * 64 * occ_words light-occlusion bits: trace_shadow -> shade
  int occ_words;  // ceil(num_lights / 32)
  // heavy-first dispatch (null: off).  tile_cost[sel] holds each selected
  // tile's cost: the probe kernel's estimate before the primary kernel, the primary kernel's
  // measured time (100 MHz ticks) before the shadow kernel.  order_kernel sorts the traversal
  // workgroups' units (kTraceWaves packets each) heaviest first within each of order_regions
  // regions into unit_order[region * order_stride + i] (-1 pads); region r holds the chunks of
  // order_chunk consecutive units c with c mod order_regions == r, and block b of an ordered
  // launch takes unit_order[(b mod regions) * stride + b / regions] — with 8 regions, the
  // blocks the hardware deals to one XCD walk one spatially coherent part of the frame,
  // heaviest first, so its L2 serves neighbouring packets.  use_order: this launch reads it.
  unsigned* tile_cost;
  int* unit_order;
  int order_regions, order_chunk, order_stride, order_units;
  int order_probe;  // estimate the primary kernel's tile costs with probe_kernel first
  int probe_depth, probe_visits;  // probe_kernel: levels walked, visits per ray
  int use_order;
  float* frames;  // recursive scenes only: (max_depth+1) * 28 * lanes ray-tree frames, else null
  // kCounterRows rows of kCounterWidth u64 (columns: kCnt*)
  unsigned long long* counters;
};

}  // namespace rt

#endif
