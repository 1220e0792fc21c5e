/* ceng795_rt — MI355X (gfx950) ray-trace hot path behind a C ABI.
 *
 * This is the drop-in boundary for the reference's render seam:
 *
 *   void Scene::render_image(int camera_index, Pixel* result, int starting_row,
 *                            int height_increase = 1) const;      HW2/Scene.h:34-35
 *                                                                 HW2/Scene.cpp:16-70
 *
 * The reference calls it from T host threads on a shared const Scene, each thread with a
 * disjoint row set (HW2/main.cpp:33-36).  Here the whole row set runs as one HIP launch
 * (or several callers on disjoint rows — rt_render is reentrant).  Everything up to the
 * seam stays on the host, as in the reference: XML ingest (HW2/Scene.cpp:198-451), the
 * Camera basis (HW2/Camera.h:10-29) and the BVH build (HW2/Bounding_volume_hierarchy.cpp:3-29)
 * happen in rt_scene_create / rt_scene_load_xml, untimed like the reference's Scene ctor.
 * rt_scene_create_multi spreads one scene's frames over several GPUs of the process.
 *
 * Plain C types only: no torch, no HIP types in signatures (streams are void*).
 * Every function returns 0 on success or a negative RT_E* code; the message of the last
 * failure on the calling thread is in rt_last_error().  No C++ exception crosses the ABI.
 */
#ifndef CENG795_RT_H_
#define CENG795_RT_H_
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

#define CENG795_RT_ABI_VERSION 7  /* 2: MSAA cameras + rt_set_msaa_seed; 3: tile ranges,
                                      kernel timing; 4: multi-device scenes, stream scratch
                                      release, no CULL mode; 5: pixel records
                                      (RT_TILE_RECORDS, rt_resolve_device); 6: rt_tile_costs,
                                      row-major records + rt_resolve_rows; 7: the caller's own
                                      BVH in rt_scene_desc (bvh_*), rt_host_dump_bvh_desc,
                                      rt_host_alloc / rt_host_free */

enum {
  RT_OK = 0,
  RT_E_INVALID = -1,  /* bad argument or scene description            */
  RT_E_HIP = -2,      /* HIP runtime error (message has the HIP text)   */
  RT_E_IO = -3,       /* file could not be read / written                */
  RT_E_PARSE = -4,    /* scene XML malformed (reference would throw/crash) */
  RT_E_UNSUPPORTED = -5
};

/* HW2/Material.h:5-13 (field order kept). */
typedef struct rt_material {
  float ambient[3];
  float diffuse[3];
  float specular[3];
  float mirror[3];
  float transparency[3];
  float refraction_index;
  float phong_exponent;
} rt_material;

/* HW2/Point_light.h:5-8 */
typedef struct rt_point_light {
  float position[3];
  float intensity[3];
} rt_point_light;

/* A camera after HW2/Camera.h:10-29's precompute: primary ray for pixel (x, y) is
 *   o = e,  d = normalize((top_left + (x+0.5)*s_u) - (y+0.5)*s_v - e).          Camera.h:30-35
 * num_samples is the per-axis sample count n = (int)sqrt(<NumSamples>) (Scene.cpp:275-276). */
typedef struct rt_camera {
  float e[3];
  float top_left[3];
  float s_u[3];
  float s_v[3];
  int width, height;
  int num_samples;
} rt_camera;

/* Scene description, flattened, 0-based, host-owned (copied by rt_scene_create).
 * Objects enter the top-level BVH in the reference's parse order: meshes, then loose
 * triangles, then spheres (HW2/Scene.cpp:380-449). */
typedef struct rt_scene_desc {
  float background[3];          /* <BackgroundColor>, default 0 0 0      */
  float shadow_ray_epsilon;     /* <ShadowRayEpsilon>, default 0.001     */
  int max_recursion_depth;      /* <MaxRecursionDepth>, default 0        */
  float ambient_light[3];       /* <Lights><AmbientLight>                */

  const float* vertices;        /* fp32[3*num_vertices]  <VertexData>    */
  int num_vertices;
  const rt_material* materials;
  int num_materials;
  const rt_point_light* lights;
  int num_lights;
  const rt_camera* cameras;
  int num_cameras;

  int num_meshes;               /* <Mesh>: material + faces              */
  const int* mesh_material;     /* int32[num_meshes]                     */
  const int* mesh_face_count;   /* int32[num_meshes]                     */
  const int* mesh_faces;        /* int32[3*sum(face_count)], vertex ids  */

  int num_triangles;            /* <Triangle>                            */
  const int* triangle_indices;  /* int32[3*num_triangles]                */
  const int* triangle_material; /* int32[num_triangles]                  */

  int num_spheres;              /* <Sphere>                              */
  const int* sphere_center;     /* int32[num_spheres], vertex id         */
  const float* sphere_radius;   /* fp32[num_spheres]                     */
  const int* sphere_material;   /* int32[num_spheres]                    */

  /* Optional (ABI 7): the caller's own BVH — e.g. the reference's Scene::bvh walked through
   * its public members (BVH::left / right / bounding_box, Mesh::bvh, Triangle::index_* /
   * normal, Sphere::center / radius; HW2/Bounding_volume_hierarchy.h:39-41, Mesh.h:12,
   * Triangle.h:12-14).  bvh_num_leaves == 0 (zero-initialised desc): the library builds the
   * reference's tree itself from the object lists (HW2/Bounding_volume_hierarchy.cpp:3-29).
   * Otherwise the library adopts this tree as given, Mesh wrappers spliced out (Mesh::intersect
   * delegates to its BVH with no box test of its own, Mesh.h:13-15):
   *   internal nodes in DFS preorder, node 0 the root (none when the root is one primitive);
   *   bvh_children[2 i + s] = child s (0 left, 1 right) of node i: >= 0 an internal node
   *     (> i), < 0 ~k for leaf k;  leaves numbered in DFS (left-first) order, which is the
   *     closest-hit tie-break order (appendix A.5 of SURVEY.md);
   *   bvh_boxes[6 i ..] = node i's Bounding_box (min xyz, max xyz) exactly as the caller holds
   *     it — these are the boxes the slab tests see;
   *   bvh_leaf_object[k] = leaf k's primitive: an index into the triangles of the object lists
   *     (mesh faces in mesh order, then loose triangles) or, past them, into the spheres;
   *   bvh_leaf_normals: NULL, or fp32[3 bvh_num_leaves] = each triangle leaf's flat normal as
   *     the caller computed it (Triangle.cpp:14; sphere leaves: ignored).
   * Every leaf index and every primitive must occur exactly once. */
  int bvh_num_nodes;
  const int* bvh_children;      /* int32[2*bvh_num_nodes]                */
  const float* bvh_boxes;       /* fp32[6*bvh_num_nodes]                 */
  int bvh_num_leaves;
  const int* bvh_leaf_object;   /* int32[bvh_num_leaves]                 */
  const float* bvh_leaf_normals;/* fp32[3*bvh_num_leaves] or NULL        */
} rt_scene_desc;

/* Work counters for one render call. */
typedef struct rt_stats {
  long long primary_rays;
  long long shadow_rays;
  long long secondary_rays;
  long long primary_hits;
  double kernel_ms;             /* HIP-event time of the render kernel(s)  */
} rt_stats;

/* Traversal modes.  Both give the reference's result on every input. */
enum {
  RT_TRAVERSAL_FAST = 0,        /* culling tree over reference treelets, near-first order,
                                   batched leaf tests (default)                               */
  RT_TRAVERSAL_REFERENCE = 1    /* visits every box the reference visits, in its order        */
};
typedef struct rt_scene rt_scene;

/* Replaces Scene::Scene's object + BVH construction (HW2/Scene.cpp:378-449 and
 * Bounding_volume_hierarchy.cpp:3-29).  `device` < 0 = the calling thread's current HIP
 * device.  Uploads the flattened scene to that device. */
int rt_scene_create(const rt_scene_desc* desc, int device, rt_scene** out);
void rt_scene_destroy(rt_scene* scene);

/* Host convenience: HW2/Scene.cpp:198-451's XML ingest, then rt_scene_create. */
int rt_scene_load_xml(const char* xml_path, int device, rt_scene** out);

/* One scene over several GPUs of this process (the reference's T render
 * threads, HW2/main.cpp:33-36, become the devices of one node).  The scene is built once on
 * the host and replicated on devices[0 .. device_count-1] (NULL: devices 0 .. device_count-1);
 * devices[0] holds the output.  rt_render / rt_render_device on such a scene deal the frame's
 * 8x8 tiles round-robin over the devices (tile t -> device t mod device_count), render every
 * share on its own device, gather the shares onto devices[0] with RCCL (one communicator per
 * device, ncclCommInitAll; send / receive pairs in one group, over xGMI) and untile them there.
 * Pixels are the single-device ones bit for bit.  MSAA cameras (whose 3x3 splat crosses tile
 * borders, HW2/Scene.cpp:51-63) split by bands of rows instead: device d owns rows
 * [H*d/n, H*(d+1)/n), renders every sample pass over its band plus a one-row halo each side,
 * resolves its band, and the bands are gathered the same way.
 * Frames of one multi-device scene are serialised (its RCCL communicators are shared). */
int rt_scene_create_multi(const rt_scene_desc* desc, int device_count, const int* devices,
                          rt_scene** out);
int rt_scene_load_xml_multi(const char* xml_path, int device_count, const int* devices,
                            rt_scene** out);
int rt_scene_device_count(const rt_scene* scene);

int rt_scene_num_cameras(const rt_scene* scene);
int rt_scene_camera(const rt_scene* scene, int camera_index, rt_camera* out);
/* Output file name of a camera's <ImageName> (loaded scenes only; "" otherwise). */
const char* rt_scene_image_name(const rt_scene* scene, int camera_index);
int rt_scene_num_lights(const rt_scene* scene);
/* Preorder BVH dump (oracle/ref/ref_harness.cpp `bvh` format) for topology parity. */
int rt_scene_dump_bvh(const rt_scene* scene, const char* path);
/* Host-only variant for tests without a GPU: XML ingest + BVH build + flatten, then the
 * same dump.  Touches no HIP API. */
int rt_host_dump_bvh_xml(const char* xml_path, const char* out_path);
/* Host-only, for tests without a GPU: the same dump for a scene description (with or without
 * the caller's own BVH, bvh_*).  Touches no HIP API. */
int rt_host_dump_bvh_desc(const rt_scene_desc* desc, const char* out_path);
/* Host-only, for tests: XML ingest + BVH build + the culling tree over reference treelets of
 * <= treelet_leaves leaves, then a check of the invariants the kernels'
 * exactness rests on (every leaf in exactly one treelet, guard boxes = the reference boxes
 * they stand for, culling boxes contain every guard box below them, ancestry links).
 * stats4: treelets, culling nodes, culling-tree depth, lone-leaf treelets (zeros when the
 * tree is a single treelet).  RT_E_INVALID with the violation in rt_last_error(). */
int rt_host_check_accel_xml(const char* xml_path, int treelet_leaves, long long* stats4);
/* Height of the flattened BVH (levels of internal nodes). */
int rt_scene_bvh_depth(const rt_scene* scene);

int rt_set_traversal(rt_scene* scene, int mode);

/* Scene::render_image(camera_index, result, starting_row, row_stride) with NumSamples == 1
 * (HW2/Scene.cpp:24-31).  Writes fp32 RGB radiance — exactly Pixel::color after the
 * reference's add_color(color, 1) — for rows j = starting_row + k*row_stride into
 * out_rgb[3*(j*width + i)] (w*h*3 floats, row-major, top row first).  Other rows are left
 * untouched.  Synchronous; safe to call concurrently on one scene from several threads.
 *
 * NumSamples > 1 (jittered MSAA + 3x3 Gaussian splat, HW2/Scene.cpp:32-69): whole frames
 * only (starting_row 0, row_stride 1, else RT_E_UNSUPPORTED).  out_rgb is then
 * Pixel::color / Pixel::weight, the value Pixel::get_color truncates (HW2/Pixel.h:17-27),
 * with the splat summed in the single-threaded reference order.  The reference seeds each
 * pixel's std::default_random_engine from the wall clock; here it is seeded with
 * splitmix64(msaa_seed, j*width + i) (rt_set_msaa_seed, default 0), so frames are
 * reproducible.  rt_stats counts every sample's rays. */
int rt_render(rt_scene* scene, int camera_index, int starting_row, int row_stride,
              float* out_rgb, rt_stats* stats);

/* Page-locked host memory for rt_render's out_rgb (ABI 7): the frame kernel writes such a buffer
 * directly through its device-visible address, with no device-to-host copy afterwards (any
 * pinned buffer, e.g. torch's pin_memory, gets the same path).  NULL on failure
 * (rt_last_error). */
void* rt_host_alloc(size_t bytes);
void rt_host_free(void* ptr);

/* tile_major flags of rt_render_device / rt_render_device_range */
enum { RT_TILE_MAJOR = 1, RT_TILE_BLOCKS = 2,
       RT_TILE_RECORDS = 4  /* each pixel as one 32-bit pixel record (the primary hit's
                               primitive and the shadow bits) instead of 3 floats — a third of the
                               bytes for the framebuffer exchange; the gathering rank shades the
                               records: tile-major shares with rt_resolve_device, row-major ones
                               (no RT_TILE_MAJOR: a 4-B word per pixel at py * width + px) with
                               rt_resolve_rows.  Only where rt_scene_records_ok. */ };

/* Device-resident variant (the building block of the one-process-per-GPU image tiling, and
 * of frames kept in HBM).  The image (rows starting_row +
 * k*row_stride) is cut into 8x8 tiles; this call renders the deal units
 * tile_begin, tile_begin + tile_step, ... into d_out (device memory).  A deal unit is
 *   one tile, tiles numbered row-major (tile_major without RT_TILE_BLOCKS), or
 *   with RT_TILE_BLOCKS one 2x2 block of tiles, blocks numbered row-major with block row by
 *   rotated left by by (unit d = by*nbx + (bx - by) mod nbx, nbx = ceil(tiles_x / 2)); a
 *   block's tiles are taken in the order (0,0) (1,0) (0,1) (1,1).  This is the deal the
 *   multi-GPU paths use: a share keeps whole blocks (the traversal workgroup's unit, so the
 *   rays of a workgroup stay neighbours) and a deal d = r (mod N) takes diagonal stripes.
 * Output (tile_major & RT_TILE_MAJOR):
 *   0: d_out is a full w*h*3 frame, written in place;
 *   1: d_out holds the selected units' tiles back to back, 8*8*3 floats each (pixels or
 *      block tiles outside the image are written as 0).
 * MSAA cameras: only the whole frame, row-major (tile_begin 0, tile_step 1, tile_major 0).
 * Asynchronous on `hip_stream` (a hipStream_t, NULL = default stream).  Ray counts
 * accumulate on the device until rt_collect_stats.  Calls on one stream run in order and share
 * that stream's scratch buffers (hit records, occlusion bits, tile schedule); each further
 * stream a scene renders on gets scratch of its own, so frames on different streams may be
 * in flight at the same time (their outputs must not overlap); host threads may enqueue
 * concurrently.  A stream's scratch lives until rt_release_stream_scratch or the scene's
 * destruction.  Multi-device scenes: whole frames only (tile_begin 0, tile_step 1,
 * tile_major 0; row subsets allowed), d_out and hip_stream on devices[0]; every caller stream
 * gets a context (device stream + buffers) of its own on each device, kept until
 * rt_release_stream_scratch, so frames on different caller streams overlap on every device. */
int rt_render_device(rt_scene* scene, int camera_index, int starting_row, int row_stride,
                     int tile_begin, int tile_step, int tile_major, float* d_out,
                     void* hip_stream);
/* rt_render_device restricted to the first `tile_count` selected deal units (tile_count < 0:
 * all): units tile_begin + k*tile_step for k < tile_count.  With RT_TILE_MAJOR the k-th tile
 * rendered lands at d_out + k*192 floats (4 tiles per unit with RT_TILE_BLOCKS).  Lets a rank render its share of a frame in chunks and hand each
 * chunk to the framebuffer gather while the next one renders (multi-GPU).
 * MSAA cameras: whole frames only. */
int rt_render_device_range(rt_scene* scene, int camera_index, int starting_row, int row_stride,
                           int tile_begin, int tile_step, int tile_count, int tile_major,
                           float* d_out, void* hip_stream);
/* The other half of the process-per-GPU tile deal: rank 0 holds every rank's share as
 * d_gathered[devices][slot][8*8*3] (rank r rendered the frame's deal units u with
 * (u + tile_offset) mod devices == r, tile-major, in order, into its slot of `slot` tiles — what
 * one equal-size gather of rt_render_device(tile_begin, tile_step = devices, RT_TILE_MAJOR
 * [| RT_TILE_BLOCKS with RT_UNTILE_BLOCKS]) outputs leaves; with blocks, slot is a multiple of
 * 4);
 * this writes them into the row-major frame d_out (rows starting_row + k*row_stride of
 * camera_index), one wave per tile, on hip_stream (device devices[0] of the scene).  Replaces
 * nothing in the reference (its threads share one Pixel array, HW2/main.cpp:33-36): it is the
 * gather's inverse. */
int rt_untile_device(rt_scene* scene, int camera_index, int starting_row, int row_stride,
                     int devices, int slot, int tile_offset, int flags, const float* d_gathered,
                     float* d_out, void* hip_stream);
/* rt_untile_device flags */
enum { RT_UNTILE_BLOCKS = 1,    /* the units are 2x2 blocks (shares rendered with RT_TILE_BLOCKS) */
       RT_UNTILE_SKIP_ROOT = 2  /* rank 0's units are not touched: the gathering rank rendered its
                                   own share in place into d_out (tile_major without
                                   RT_TILE_MAJOR), so its slot need not be gathered */ };
/* 1 when camera_index of the scene can exchange pixel records (RT_TILE_RECORDS): a pixel-centre
 * camera, no mirror/dielectric recursion, at most 4 point lights; else 0. */
int rt_scene_records_ok(const rt_scene* scene, int camera_index);
/* rt_untile_device for shares rendered with RT_TILE_RECORDS: d_gathered holds
 * [devices][slot][8*8] 32-bit pixel records; each is shaded into its pixel of the row-major
 * frame d_out — the colour the rank that traced it would have written, bit for bit (the hit's
 * distance is re-derived by the same intersection arithmetic).  Same layout and flags as
 * rt_untile_device.  This is the shading step of Scene::trace_ray (HW2/Scene.cpp:101-138)
 * moved to the gathering GPU. */
int rt_resolve_device(rt_scene* scene, int camera_index, int starting_row, int row_stride,
                      int devices, int slot, int tile_offset, int flags,
                      const unsigned* d_gathered, float* d_out, void* hip_stream);
/* The measured cost of every tile of the last frame rt_render_device enqueued on `hip_stream`
 * (single-device scenes, pixel-centre cameras without recursion): each 8x8 packet's time from
 * its first traversal step to its shading, in ticks of the 100 MHz device clock, in the order
 * of that call's tile selection (row-major tiles for a whole frame).  Waits for the stream;
 * writes at most `capacity` values to host memory and returns how many it wrote.  The row bands
 * of the multi-GPU frame split are cut from these (dist_tiles.BandPlan).  Nothing in the
 * reference measures work; its threads take interleaved rows (HW2/main.cpp:33-36). */
int rt_tile_costs(rt_scene* scene, void* hip_stream, unsigned* host_out, int capacity);
/* Row-major pixel records (rt_render_device with RT_TILE_RECORDS and no RT_TILE_MAJOR: one
 * 32-bit word per pixel at py * width + px of d_records) shaded into rows [row_begin, row_end)
 * of the row-major frame d_out — bit for bit the colours the tracing rank would have written.
 * The band split's rank 0 runs it over the rows the other ranks sent (dist_tiles.BandPlan). */
int rt_resolve_rows(rt_scene* scene, int camera_index, int row_begin, int row_end,
                    const unsigned* d_records, float* d_out, void* hip_stream);
/* Waits for `hip_stream` and frees the scratch rt_render_device keeps for it (no-op for a
 * stream the scene never rendered on).  Streams that come and go should release theirs. */
int rt_release_stream_scratch(rt_scene* scene, void* hip_stream);
/* Per-kernel timing of render launches: while enabled, every launch records HIP events around
 * its kernels on the launch's stream.  rt_read_kernel_times returns (and resets) the summed
 * milliseconds ms4 = {frame kernel (primary rays, shadow rays and shading of every packet; or
 * the recursive kernel), order kernel (the next frame's dispatch order), other (0), all} and
 * the number of launches timed. */
int rt_set_kernel_timing(rt_scene* scene, int enable);
int rt_read_kernel_times(rt_scene* scene, double* ms4, long long* launches);
/* Seed of the per-pixel MSAA generators (see rt_render).  Replaces the reference's
 * system_clock seed (HW2/Scene.cpp:36-37) to make MSAA frames deterministic. */
int rt_set_msaa_seed(rt_scene* scene, unsigned long long seed);
int rt_num_tiles(const rt_scene* scene, int camera_index, int starting_row, int row_stride);
/* Reads (and resets) the device ray counters accumulated by rt_render_device calls. */
int rt_collect_stats(rt_scene* scene, rt_stats* stats);

/* Sums (and resets) all 16 device counter columns: [0] primary rays [1] shadow rays
 * [2] secondary rays [3] primary hits; RT_DIAG builds (libceng795_rt_diag.so) add packet-level
 * work: [4..7] primary node visits / active lanes summed over visits / leaf visits / leaf
 * lane tests, [8..11] the same for shadow rays, [12] lanes that fell back to the exact slab
 * test (node boxes and leaf guards), [13] leaf-batch guard tests (primary + shadow),
 * [14] / [15] the primary / shadow node visits that were 8-wide culling nodes (included in
 * [4] / [8]).
 * Returns 1 for a diagnostic build, 0 otherwise (columns 4..15 then read 0). */
int rt_debug_counters(rt_scene* scene, long long* out16);

/* RT_TIMELINE experiment builds (tools/timeline.py): copies and clears the per-wave start/end
 * ticks (100 MHz clock) and tile of the last traversal launches, out[2 kernels][2^18 waves][3].
 * Returns the number of values written (0 in other builds) or a negative RT_E_* code. */
long long rt_debug_timeline(unsigned long long* out, long long max_values);

/* RT_DIAG builds (tools/phases.py): copies and clears the per-phase attribution of the frame
 * kernel — per traversal kind (primary, shadow) the visit loop's events (visits, slots tested,
 * slot hits, leafy / pair / inner hits, stack pushes and pops, leaf-batch flushes and their
 * 64-test iterations), then shader-clock cycle sums per phase (rt_internal.h kPh*).  Returns the
 * number of values written (0 in other builds) or a negative RT_E_* code. */
long long rt_debug_phases(unsigned long long* out, long long max_values);

/* Device self-check of the triangle test's shared-reciprocal quotients (rt_kernels.hip,
 * tri_quotients) against IEEE division on `count` seeded random operand pairs of the fast
 * range; out2[0] = mismatching quotients (must be 0), out2[1] = cases run. */
int rt_debug_quotient_check(int device, unsigned long long seed, long long count,
                            long long* out2);

/* PNG output as HW2/main.cpp:43-57: per channel clamp(int(c), 0, 255), alpha 255. */
int rt_write_png(const char* path, const float* rgb, int width, int height);

/* Camera precompute of HW2/Camera.h:10-29 in the reference's fp32 operation order. */
int rt_camera_from_view(const float position[3], const float gaze[3], const float up[3],
                        const float near_plane[4] /* l r b t */, float near_distance,
                        int width, int height, int num_samples, rt_camera* out);

const char* rt_last_error(void);
int rt_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
