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
  kCntGuardTests = 13,  // RT_DIAG: leaf-batch guard tests (primary + shadow)
  // RT_DIAG builds: the node visits above that were 8-wide culling nodes (128 B each)
  kCntPrimWide = 14, kCntShadWide = 15
};

// RT_DIAG per-phase attribution (rt_debug_phases, tools/phases.py): per traversal kind (primary,
// shadow) the visit loop's events, then shader-clock cycle sums.
enum : int {
  kPhVisits = 0, kPhSlotsTested = 1, kPhSlotHits = 2, kPhLeafyHits = 3, kPhPairHits = 4,
  kPhInnerHits = 5, kPhPushes = 6, kPhPops = 7, kPhFlushes = 8, kPhFlushIters = 9,
  kPhaseEvents = 10
};
enum : int {
  kPhCycPrimTotal = 2 * kPhaseEvents, kPhCycPrimVisit, kPhCycPrimLoad, kPhCycPrimFlush,
  kPhCycShadTotal, kPhCycShadVisit, kPhCycShadLoad, kPhCycShadFlush, kPhCycShade,
  kPhCycFrame, kPhWaves, kPhaseSlots
};

constexpr int kDefaultTreeletLeaves = 2;  // culling-tree treelets: lone leaves and leaf pairs

struct alignas(16) DevNode {
  // Both CHILD boxes, interleaved per coordinate ([axis][child]).  Unused for a leaf child (a
  // +-1e30 box every normalised ray accepts, scene_build.cpp).
  float lo[3][2];
  float hi[3][2];
  int32_t child[2];  // >= 0: internal node index; < 0: leaf index ~child
  int32_t axis;      // split dimension of THIS node (Bounding_volume_hierarchy.cpp:8)
  int32_t pad;       // 0 (reference nodes; the culling tree has its own record, DevNode8)
};
static_assert(sizeof(DevNode) == 64, "node must be one 64-byte scalar load");

// 8-wide culling node (accel_build.cpp): two consecutive DevNode slots of
// `nodes`, referred to as (index of the first slot) | kWideTag.  Slot c is valid when bit c of
// `kinds` is set; it is then either LEAFY (bit 8 + c: one treelet = a lone leaf, or with bit
// 16 + c a leaf pair; its leaves are DevLeaf records leaf_base + (offs >> 4c & 15) and the next
// one) or INNER (a child node: inner_base + 2 * (number of inner slots before c)).  Every slot
// carries a CONSERVATIVE box in fp16, relative to `origin` and scaled by 2^k per axis:
//   plane = origin[a] + h * 2^(scale byte a, signed)
// rounded outward and inflated by the scene's culling margin (HostScene::cull_margin), so a
// plain slab test (no decision band) never culls a treelet the reference would enter; the
// exact decision (the treelet's guard box) is taken per ray in the leaf batch.  An invalid
// slot holds NaN planes, which every slab test rejects.
constexpr int32_t kWideTag = 1 << 30;
// node slots a scene may have with a culling tree: the traversal loads a wide node at the 32-bit
// byte offset (ref << 6) (rt_kernels.hip load_node8); larger scenes walk the reference tree
constexpr size_t kMaxNodeSlots = size_t(1) << 26;
constexpr int kWideSlots = 8;
enum : int32_t { kSlotValid = 1, kSlotLeafy = 1 << 8, kSlotPair = 1 << 16 };
struct alignas(16) DevNode8 {
  float origin[3];
  uint32_t scale;      // byte a: k_a as a signed byte
  int32_t inner_base;  // DevNode index of the first inner child (children contiguous, 2 slots each)
  int32_t leaf_base;   // DevLeaf index of the first leafy slot's first leaf
  int32_t kinds;       // kSlotValid << c | kSlotLeafy << c | kSlotPair << c
  uint32_t offs;       // 4 bits per slot: its first leaf's offset from leaf_base (leafy slots)
  uint32_t box[kWideSlots][3];  // per slot and axis: lo fp16 (bits 0-15), hi fp16 (16-31)
};
static_assert(sizeof(DevNode8) == 128, "a wide node is two s_load_dwordx16");
static_assert(sizeof(DevNode8) == 2 * 64, "a wide node is two node slots");

// A leaf as the fast traversal tests it, in culling-tree order (each wide node's leaves
// contiguous): the primitive (as DevPrim), its DFS leaf index — the reference's tie-break key
// and the index of every per-leaf array — and the GUARD box, the box of the reference node
// holding the leaf.  A ray may test the leaf iff every reference ancestor box accepts it
// (HW2/Bounding_volume_hierarchy.cpp:31-55); the guard accepting with margin implies that
// (DESIGN.md §4.1), else the kernel walks the ancestry (guard_exact).
//   q[0] = v0.xyz, dfs | kLeafSphere      q[1] = a1.xyz (sphere: radius, 0, 0), guard lo.x
//   q[2] = a2.xyz, guard lo.y              q[3] = guard lo.z, hi.xyz
constexpr int32_t kLeafSphere = 1 << 30;
struct alignas(16) DevLeaf {
  float v0[3];
  int32_t dfs;  // | kLeafSphere for a sphere
  float a1[3];
  float g0;
  float a2[3];
  float g1;
  float g2, g3, g4, g5;
};
static_assert(sizeof(DevLeaf) == 64, "leaf record is four 16-byte loads");

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
#if defined(__HIPCC__)
#define RT_HD __host__ __device__
#else
#define RT_HD
#endif

// Pixel record (rt_render_device with RT_TILE_RECORDS; rt_resolve_device): what a share of a
// multi-GPU frame sends to the gathering rank instead of 12 B of colour — the primary hit's DFS
// leaf index (bits 0..25) and the shadow bits of lights 0..3 (bits 26..29); or a miss (the
// background) or a pixel outside the image.  The gathering rank re-derives the hit's t with the
// same intersection arithmetic (bit for bit) and shades it there.
constexpr unsigned kRecLeafMask = (1u << 26) - 1u;
constexpr int kRecLightShift = 26;
constexpr unsigned kRecLightMask = 15u;  // lights 0..3
constexpr int kRecMaxLights = 4;
constexpr unsigned kRecMiss = 1u << 30;
constexpr unsigned kRecOutside = 2u << 30;

// Block deal (rt_render_device with RT_TILE_BLOCKS, multi-device frames): the unit dealt over
// devices is a 2x2 block of tiles (the traversal workgroup's unit, so a share keeps the
// in-place frame's coherence), numbered with each block row rotated by its row index —
// d = by * nbx + (bx - by) mod nbx — so that a deal d = r (mod N) takes diagonal stripes of
// blocks rather than the same columns in every row (nbx is often a multiple of N).  Selected
// block k holds tiles 4k .. 4k + 3 of the selection (w = 2 * (ty & 1) + (tx & 1)).
RT_HD inline int deal_blocks_x(int tiles_x) { return (tiles_x + 1) >> 1; }
RT_HD inline int deal_blocks(int tiles_x, int tiles_y) {
  return deal_blocks_x(tiles_x) * ((tiles_y + 1) >> 1);
}
RT_HD inline void deal_block_tile(int tiles_x, int d, int w, int& tx, int& ty) {
  const int nbx = deal_blocks_x(tiles_x), by = d / nbx;
  int bx = d - by * nbx + by % nbx;
  if (bx >= nbx) bx -= nbx;
  tx = 2 * bx + (w & 1);
  ty = 2 * by + (w >> 1);
}
RT_HD inline int deal_block_index(int tiles_x, int tx, int ty, int& w) {
  const int nbx = deal_blocks_x(tiles_x), bx = tx >> 1, by = ty >> 1;
  w = ((ty & 1) << 1) | (tx & 1);
  int c = bx - by % nbx;
  if (c < 0) c += nbx;
  return by * nbx + c;
}

struct UntileParams {
  const float* recv;
  float* out;
  int width, row0, row_stride, rows, tiles_x, tiles_total, devices, slot;
  int tile_offset;  // deal unit u went to rank (u + tile_offset) mod devices (rt_untile_device)
  int blocks;       // 1: the units are 2x2 blocks in deal order (deal_block_index), else tiles
  int vec;          // 1: rows and buffers 16-B aligned (untile by 16-B chunks)
  int skip_root;    // 1: rank 0's units are left alone (it rendered them in place)
};

// Words of the per-stream schedule buffer for a launch of `tiles` selected tiles: tile costs
// + the unit order lists (order_layout in rt_kernels.hip stays below sched_snap_offset), then
// the snapshot of the tile costs the order kernel read (rt_tile_costs) in the last `tiles` words.
constexpr unsigned long long sched_words_for(unsigned long long tiles) { return 10 * tiles + 64; }
constexpr unsigned long long sched_snap_offset(unsigned long long tiles) { return 9 * tiles + 64; }

struct RenderParams {
  const DevNode* nodes;
  const DevLeaf* leaves;  // culling-tree order (DevLeaf), FAST traversal
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
  int block_deal;  // the selection counts 2x2 blocks in deal order (deal_block_tile)
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
  // tile's cost: the primary kernel's measured time (100 MHz ticks), read before the shadow
  // kernel.  order_kernel sorts the traversal
  // workgroups' units (kTraceWaves packets each) heaviest first within each of order_regions
  // regions into unit_order[region * order_stride + i] (-1 pads); region r holds the chunks of
  // order_chunk consecutive units c with c mod order_regions == r, and block b of an ordered
  // launch takes unit_order[(b mod regions) * stride + b / regions] — with 8 regions, the
  // blocks the hardware deals to one XCD walk one spatially coherent part of the frame,
  // heaviest first, so its L2 serves neighbouring packets.  use_order: this launch reads it.
  unsigned* tile_cost;
  int* unit_order;
  int order_regions, order_chunk, order_stride, order_units;
  int order_split;  // units per region the order kernel may split into quadrant waves per tile
  int use_order;
  // cold_order: the camera's whole-frame unit order seeded at scene creation from estimated tile
  // costs (rt_api.hip seed_cold_orders), for a frame without a previous one (no split entries);
  // used when the launch selects cold_tiles tiles (the whole frame), else nullptr
  const int* cold_order;
  int cold_tiles;
  // pair_rows: a row-major frame in host memory written over PCIe (rt_render, pinned): the two
  // tiles of a workgroup are written together as whole rows of 16 pixels (launch_variant
  // checks the layout; 0 = each wave writes its own tile)
  int pair_rows;
  int primary_order;  // the primary kernel too dispatches by unit_order: the order the previous
                      // frame of the same selection left on this stream (rt_api.hip warm order)
  int records;    // RT_TILE_RECORDS: the shading phase writes 32-bit pixel records, not RGB
  float* frames;  // recursive scenes only: (max_depth+1) * 28 * lanes ray-tree frames, else null
  // kCounterRows rows of kCounterWidth u64 (columns: kCnt*)
  unsigned long long* counters;
};

}  // namespace rt

#endif
