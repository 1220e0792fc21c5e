// C-ABI implementation (include/ceng795_rt.h): scene upload, render launches, counters.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/ceng795_rt.h"
#include "host_scene.h"
#include "rt_internal.h"

namespace rt {
hipError_t launch_render(const RenderParams& P, const DevNode* nodes, const DevPrim* prims,
                         const float* normals, const DevMaterial* mats, const DevLight* lights,
                         bool fast, bool deep, bool spheres, bool cull, bool wide_only,
                         const hipEvent_t* marks, hipStream_t stream);
int max_supported_depth();
hipError_t launch_msaa_resolve(const MsaaResolveParams& M, hipStream_t stream);
unsigned long long read_reset_exact_fallbacks();
hipError_t launch_quot_check(unsigned long long seed, long long count, unsigned long long* counts,
                             hipStream_t stream);
bool diag_build();
long long read_reset_timeline(unsigned long long* out, long long max_values);
void write_png(const std::string& path, const float* rgb, int w, int h);
}  // namespace rt

using namespace rt;

// Device buffers of one synchronous rt_render call, kept by the scene and reused: the
// reference calls render_image once per thread per camera (HW2/main.cpp:33-36), so a drop-in
// pays hipMalloc / hipFree only the first time a call of that size runs.  Calls on several
// host threads each take their own context (rt_render stays reentrant).
struct RenderCtx {
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  float* d_out = nullptr;
  size_t out_floats = 0;
  unsigned long long* d_cnt = nullptr;
  rt::int2_t* d_hits = nullptr;
  size_t hits_records = 0;
  unsigned* d_occ = nullptr;
  size_t occ_words = 0;
  unsigned* d_sched = nullptr;  // per tile: traversal cost, then the shadow dispatch order
  size_t sched_words = 0;
  float* d_frames = nullptr;
  size_t frames_floats = 0;
  float* d_samples = nullptr;
  size_t samples_floats = 0;
};

// Per-kernel HIP-event timing of render launches (rt_set_kernel_timing): one quad of events
// per launch, read back by rt_read_kernel_times.
struct KernelTiming {
  bool on = false;
  std::vector<std::array<hipEvent_t, 4>> pending, spare;
};

struct rt_scene {
  HostScene host;
  int device = 0;
  int mode = RT_TRAVERSAL_FAST;
  bool deep = false;
  bool needs_recursion = false;
  bool has_spheres = false;
  bool wide_only = false;  // the fast walk meets 4-wide culling nodes only (launch_render)
  DevNode* d_nodes = nullptr;
  DevPrim* d_prims = nullptr;
  float* d_normals = nullptr;
  DevAncestry* d_anc = nullptr;
  DevMaterial* d_mats = nullptr;
  DevLight* d_lights = nullptr;
  unsigned long long* d_counters = nullptr;
  int2_t* d_hits = nullptr;  // rt_render_device's primary-hit records (largest camera)
  unsigned* d_occ = nullptr; // rt_render_device's occlusion bits
  unsigned* d_sched = nullptr;  // rt_render_device's tile costs + shadow order (2 x tiles)
  float* d_frames = nullptr; // rt_render_device's ray-tree frames (recursive scenes)
  size_t frames_capacity = 0;
  size_t hits_capacity = 0;  // records
  float* d_samples = nullptr;  // MSAA per-sample colours [s][h][w][3]
  size_t samples_capacity = 0;
  // rt_render_device scratch of every further stream the scene renders on (the first one uses
  // the buffers above): frames on different streams may be in flight together
  struct StreamScratch {
    void* stream;
    int2_t* hits;
    unsigned* occ;
    unsigned* sched;
    float* frames;
    size_t frames_capacity;
    float* samples;
    size_t samples_capacity;
  };
  void* first_stream = nullptr;
  bool first_stream_set = false;
  std::vector<StreamScratch> streams;
  unsigned long long msaa_seed = 0;
  std::mutex ctx_mu;
  std::vector<RenderCtx*> ctx_free, ctx_all;
  KernelTiming timing;
};

namespace {

thread_local std::string g_error;

int set_error(int code, const std::string& msg) {
  g_error = msg;
  return code;
}

struct HipFailure {
  hipError_t err;
  const char* what;
};

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw HipFailure{e, what};
}

template <typename F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const HipFailure& h) {
    return set_error(RT_E_HIP, std::string(h.what) + ": " + hipGetErrorString(h.err));
  } catch (const std::domain_error& e) {
    return set_error(RT_E_UNSUPPORTED, e.what());
  } catch (const std::invalid_argument& e) {
    return set_error(RT_E_INVALID, e.what());
  } catch (const std::ios_base::failure& e) {
    return set_error(RT_E_IO, e.what());
  } catch (const std::runtime_error& e) {
    return set_error(RT_E_PARSE, e.what());
  } catch (const std::bad_alloc&) {
    return set_error(RT_E_INVALID, "out of host memory");
  } catch (const std::exception& e) {
    return set_error(RT_E_INVALID, e.what());
  }
}

template <typename T>
T* upload(const std::vector<T>& v, const char* what) {
  T* p = nullptr;
  // +64 B: the kernels may fetch a record with one 64-byte scalar load past its 48 bytes
  const size_t bytes = v.size() * sizeof(T) + 64;
  hip_check(hipMalloc(&p, bytes), what);
  if (!v.empty()) hip_check(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice), what);
  return p;
}

void free_ctx(RenderCtx* c) {
  (void)hipFree(c->d_out);
  (void)hipFree(c->d_cnt);
  (void)hipFree(c->d_hits);
  (void)hipFree(c->d_occ);
  (void)hipFree(c->d_sched);
  (void)hipFree(c->d_frames);
  (void)hipFree(c->d_samples);
  if (c->e0) (void)hipEventDestroy(c->e0);
  if (c->e1) (void)hipEventDestroy(c->e1);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

void free_device(rt_scene* s) {
  int cur = 0;
  if (hipGetDevice(&cur) == hipSuccess && cur != s->device) (void)hipSetDevice(s->device);
  for (RenderCtx* c : s->ctx_all) free_ctx(c);
  s->ctx_all.clear();
  s->ctx_free.clear();
  for (auto* v : {&s->timing.pending, &s->timing.spare})
    for (auto& q : *v)
      for (hipEvent_t e : q) (void)hipEventDestroy(e);
  (void)hipFree(s->d_nodes);
  (void)hipFree(s->d_prims);
  (void)hipFree(s->d_normals);
  (void)hipFree(s->d_anc);
  (void)hipFree(s->d_mats);
  (void)hipFree(s->d_lights);
  (void)hipFree(s->d_counters);
  (void)hipFree(s->d_hits);
  (void)hipFree(s->d_occ);
  (void)hipFree(s->d_sched);
  (void)hipFree(s->d_frames);
  (void)hipFree(s->d_samples);
  for (auto& x : s->streams) {
    (void)hipFree(x.hits);
    (void)hipFree(x.occ);
    (void)hipFree(x.sched);
    (void)hipFree(x.frames);
    (void)hipFree(x.samples);
  }
  if (cur != s->device) (void)hipSetDevice(cur);
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    hip_check(hipGetDevice(&prev), "hipGetDevice");
    if (prev != dev) hip_check(hipSetDevice(dev), "hipSetDevice");
  }
  ~DeviceGuard() {
    int cur;
    if (hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

constexpr int kFrameFloats = 28;  // rt_kernels.hip kFrFields

size_t frame_floats(const HostScene& h, int sel_tiles) {
  return (size_t)(h.max_depth + 1) * kFrameFloats * kTile * kTile * (size_t)std::max(1, sel_tiles);
}

int occ_words(const HostScene& h) { return std::max(1, ((int)h.lights.size() + 31) / 32); }

// A counter buffer: kCounterRows x kCounterWidth ray counters.
constexpr size_t kCounterAlloc = (size_t)kCounterWidth * kCounterRows;
// CENG795_RT_ORDER=0 turns the heavy-first shadow dispatch off (A/B experiments); the
// order cannot change any result, only which tiles start first.
bool order_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("CENG795_RT_ORDER");
    return !(e && e[0] == '0');
  }();
  return on;
}
void set_schedule(RenderParams& P, unsigned* sched) {
  // (the buffer holds 2 x the camera's tiles; a launch uses its first 2 x num_sel_tiles)
  P.tile_cost = order_enabled() ? sched : nullptr;
  P.tile_order = order_enabled() ? reinterpret_cast<int*>(sched) + P.num_sel_tiles : nullptr;
}

// True when the culling tree is 4-wide and no slot leads to a binary node (every guarded slot
// is a leaf or a leaf pair), so the fast walk never visits a binary node.
bool wide_only_tree(const HostScene& h) {
  if (h.accel_root < 0 || !(h.accel_root & kWideTag)) return false;
  for (size_t n = (size_t)(h.accel_root & ~kWideTag); n + 1 < h.nodes.size(); n += 2) {
    DevNode4 W;
    std::memcpy(&W, &h.nodes[n], sizeof W);
    for (int k = 0; k < 4; k++)
      if ((W.flags & (kWideValid << k)) && (W.flags & (kWideGuard << k)) && W.child[k] >= 0)
        return false;
  }
  return true;
}

int create_from_host(rt_scene* s, int device) {
  if (device < 0) hip_check(hipGetDevice(&device), "hipGetDevice");
  s->device = device;
  DeviceGuard g(device);
  build_accel(s->host, accel_treelet_leaves());
  if (s->host.accel_depth > max_supported_depth()) build_accel(s->host, 0);
  if (std::getenv("CENG795_RT_VERBOSE"))
    std::fprintf(stderr, "ceng795_rt: %zu nodes (reference depth %d), culling tree root %d over "
                 "%d treelets, depth %d\n", s->host.nodes.size(), s->host.depth,
                 s->host.accel_root, s->host.accel_items, s->host.accel_depth);
  const HostScene& h = s->host;
  if (h.depth > max_supported_depth())
    throw std::invalid_argument("BVH deeper than " + std::to_string(max_supported_depth()) +
                                " levels is not supported");
  s->deep = std::max(h.depth, h.accel_depth) > kLaneStack - 2;
  for (const DevPrim& p : h.prims) s->has_spheres |= p.kind == kPrimSphere;
  s->wide_only = wide_only_tree(h);
  for (const DevMaterial& m : h.materials) {
    const bool mirror = m.mirror[0] != 0 || m.mirror[1] != 0 || m.mirror[2] != 0;
    const bool glass = m.transparency[0] != 0 || m.transparency[1] != 0 || m.transparency[2] != 0;
    if ((mirror || glass) && h.max_depth > 0) s->needs_recursion = true;
  }
  s->d_nodes = upload(h.nodes, "upload nodes");
  s->d_prims = upload(h.prims, "upload prims");
  s->d_normals = upload(h.normals, "upload normals");
  s->d_anc = upload(h.ancestry, "upload ancestry");
  s->d_mats = upload(h.materials, "upload materials");
  s->d_lights = upload(h.lights, "upload lights");
  // ray counters
  hip_check(hipMalloc(&s->d_counters, sizeof(unsigned long long) * kCounterAlloc),
            "alloc counters");
  hip_check(hipMemset(s->d_counters, 0, sizeof(unsigned long long) * kCounterAlloc),
            "zero counters");
  size_t most = 1;
  for (const rt_camera& c : h.cameras) {
    const size_t tiles = (size_t)((c.width + kTile - 1) / kTile) * ((c.height + kTile - 1) / kTile);
    most = std::max(most, tiles * kTile * kTile);
  }
  hip_check(hipMalloc(&s->d_hits, most * sizeof(int2_t)), "alloc hit records");
  hip_check(hipMalloc(&s->d_occ, most * sizeof(unsigned) * occ_words(h)), "alloc occlusion bits");
  hip_check(hipMalloc(&s->d_sched, 2 * (most / (kTile * kTile)) * sizeof(unsigned)),
            "alloc tile schedule");
  s->hits_capacity = most;
  return RT_OK;
}

struct TilePlan {
  int rows, tiles_x, tiles_total;
};

TilePlan plan(const rt_camera& c, int row0, int row_stride) {
  TilePlan p;
  p.rows = row0 < c.height ? (c.height - row0 + row_stride - 1) / row_stride : 0;
  p.tiles_x = (c.width + kTile - 1) / kTile;
  p.tiles_total = p.tiles_x * ((p.rows + kTile - 1) / kTile);
  return p;
}

RenderParams make_params(const rt_scene* s, int cam, int row0, int row_stride, int tile_begin,
                         int tile_step, int tile_major, float* out, bool counters) {
  const HostScene& h = s->host;
  const rt_camera& c = h.cameras[cam];
  RenderParams P;
  std::memset(&P, 0, sizeof P);
  P.nodes = s->d_nodes;
  P.prims = s->d_prims;
  P.normals = s->d_normals;
  P.materials = s->d_mats;
  P.lights = s->d_lights;
  P.num_lights = (int)h.lights.size();
  P.max_depth = h.max_depth;
  std::memcpy(P.background, h.background, sizeof P.background);
  std::memcpy(P.ambient, h.ambient, sizeof P.ambient);
  P.eps = h.eps;
  P.root_kind = h.root_kind;
  P.root_ref = h.root_ref;
  std::memcpy(P.root_box, h.root_box, sizeof P.root_box);
  P.accel_root = h.accel_root;
  P.quot_ok = h.quot_ok;
  std::memcpy(P.accel_box, h.accel_box, sizeof P.accel_box);
  P.anc = s->d_anc;
  std::memcpy(P.cam_e, c.e, 12);
  std::memcpy(P.cam_tl, c.top_left, 12);
  std::memcpy(P.cam_su, c.s_u, 12);
  std::memcpy(P.cam_sv, c.s_v, 12);
  P.width = c.width;
  P.height = c.height;
  const TilePlan tp = plan(c, row0, row_stride);
  P.row0 = row0;
  P.row_stride = row_stride;
  P.rows = tp.rows;
  P.tiles_x = tp.tiles_x;
  P.tiles_total = tp.tiles_total;
  P.tile_begin = tile_begin;
  P.tile_step = tile_step;
  P.num_sel_tiles =
      tile_begin < tp.tiles_total ? (tp.tiles_total - tile_begin + tile_step - 1) / tile_step : 0;
  P.tile_major = tile_major;
  P.out = out;
  P.hits = s->d_hits;
  P.occ = s->d_occ;
  P.occ_words = occ_words(h);
  set_schedule(P, s->d_sched);
  P.counters = counters ? s->d_counters : nullptr;
  return P;
}

void check_render_args(const rt_scene* s, int cam, int row0, int row_stride) {
  if (!s) throw std::invalid_argument("scene is NULL");
  if (cam < 0 || cam >= (int)s->host.cameras.size())
    throw std::invalid_argument("camera index out of range");
  if (row0 < 0 || row_stride < 1) throw std::invalid_argument("bad row selection");
  // MSAA splats every sample into the 3x3 neighbourhood (HW2/Scene.cpp:48-62), so a row subset
  // is not a self-contained piece of the image: only whole frames are rendered.
  if (s->host.cameras[cam].num_samples > 1 && (row0 != 0 || row_stride != 1))
    throw std::domain_error("NumSamples > 1 renders whole frames only (starting_row 0, stride 1)");
}

unsigned powmod_minstd(unsigned a, unsigned e) {
  unsigned long long r = 1, b = a;
  while (e) {
    if (e & 1) r = r * b % kMinstdM;
    b = b * b % kMinstdM;
    e >>= 1;
  }
  return (unsigned)r;
}

// One frame of camera `cam` into d_out.  Pixel-centre cameras: the render kernels write
// d_out directly.  MSAA cameras (HW2/Scene.cpp:32-69): one render pass per sample index into
// d_samples[s], then the resolve kernel's splat + colour / weight into d_out (row-major).
// Events for one timed launch (nullptr when timing is off or the launch renders nothing).
const hipEvent_t* timing_marks(rt_scene* s, const RenderParams& P) {
  if (!s->timing.on || P.num_sel_tiles <= 0) return nullptr;
  std::lock_guard<std::mutex> lk(s->ctx_mu);
  KernelTiming& t = s->timing;
  if (t.spare.empty()) {
    std::array<hipEvent_t, 4> q{};
    for (hipEvent_t& e : q) hip_check(hipEventCreate(&e), "timing event");
    t.spare.push_back(q);
  }
  t.pending.push_back(t.spare.back());
  t.spare.pop_back();
  return t.pending.back().data();
}

void enqueue_frame(rt_scene* s, const RenderParams& P, int samples, float* d_samples,
                   hipStream_t stream) {
  const bool fast = s->mode != RT_TRAVERSAL_REFERENCE;
  const bool cull = s->mode == RT_TRAVERSAL_CULL;
  if (samples <= 1) {
    hip_check(launch_render(P, s->d_nodes, s->d_prims, s->d_normals, s->d_mats, s->d_lights,
                            fast, s->deep, s->has_spheres, cull, s->wide_only, timing_marks(s, P), stream),
              "render launch");
    return;
  }
  const size_t frame = (size_t)P.width * P.height * 3;
  for (int k = 0; k < samples * samples; k++) {
    RenderParams Q = P;
    Q.msaa_n = samples;
    Q.msaa_s = k;
    Q.msaa_mul[0] = powmod_minstd(kMinstdA, 2 * k + 1);
    Q.msaa_mul[1] = powmod_minstd(kMinstdA, 2 * k + 2);
    Q.msaa_seed = s->msaa_seed;
    Q.tile_major = 0;
    Q.out = d_samples + (size_t)k * frame;
    hip_check(launch_render(Q, s->d_nodes, s->d_prims, s->d_normals, s->d_mats, s->d_lights,
                            fast, s->deep, s->has_spheres, cull, s->wide_only, timing_marks(s, Q), stream),
              "render launch");
  }
  MsaaResolveParams M;
  M.samples = d_samples;
  M.out = P.out;
  M.width = P.width;
  M.height = P.height;
  M.n = samples;
  M.seed = s->msaa_seed;
  hip_check(launch_msaa_resolve(M, stream), "msaa resolve launch");
}

size_t sample_floats(const rt_camera& c) {
  return c.num_samples > 1 ? (size_t)c.num_samples * c.num_samples * c.width * c.height * 3 : 0;
}

}  // namespace

namespace {

// Grow-only device buffer.
template <typename T>
void ensure(T*& p, size_t& cap, size_t need, const char* what) {
  need = std::max<size_t>(need, 1);
  if (need <= cap) return;
  (void)hipFree(p);
  p = nullptr;
  cap = 0;
  hip_check(hipMalloc(&p, need * sizeof(T)), what);
  cap = need;
}

RenderCtx* acquire_ctx(rt_scene* s) {
  {
    std::lock_guard<std::mutex> lk(s->ctx_mu);
    if (!s->ctx_free.empty()) {
      RenderCtx* c = s->ctx_free.back();
      s->ctx_free.pop_back();
      return c;
    }
  }
  std::unique_ptr<RenderCtx> c(new RenderCtx);
  try {
    hip_check(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking), "stream");
    hip_check(hipEventCreate(&c->e0), "event");
    hip_check(hipEventCreate(&c->e1), "event");
    hip_check(hipMalloc(&c->d_cnt, sizeof(unsigned long long) * kCounterAlloc), "alloc counters");
  } catch (...) {
    free_ctx(c.release());
    throw;
  }
  std::lock_guard<std::mutex> lk(s->ctx_mu);
  s->ctx_all.push_back(c.get());
  return c.release();
}

void release_ctx(rt_scene* s, RenderCtx* c) {
  std::lock_guard<std::mutex> lk(s->ctx_mu);
  s->ctx_free.push_back(c);
}

}  // namespace

extern "C" {

int rt_abi_version(void) { return CENG795_RT_ABI_VERSION; }
const char* rt_last_error(void) { return g_error.c_str(); }

int rt_camera_from_view(const float position[3], const float gaze[3], const float up[3],
                        const float near_plane[4], float near_distance, int width, int height,
                        int num_samples, rt_camera* out) {
  if (!position || !gaze || !up || !near_plane || !out || width <= 0 || height <= 0)
    return set_error(RT_E_INVALID, "rt_camera_from_view: bad argument");
  camera_from_view(position, gaze, up, near_plane, near_distance, width, height,
                   num_samples < 1 ? 1 : num_samples, *out);
  return RT_OK;
}

int rt_scene_create(const rt_scene_desc* desc, int device, rt_scene** out) {
  if (!desc || !out) return set_error(RT_E_INVALID, "rt_scene_create: NULL argument");
  *out = nullptr;
  auto s = std::make_unique<rt_scene>();
  const int rc = guarded([&] {
    build_host_scene(*desc, s->host);
    return create_from_host(s.get(), device);
  });
  if (rc != RT_OK) {
    free_device(s.get());
    return rc;
  }
  *out = s.release();
  return RT_OK;
}

int rt_scene_load_xml(const char* xml_path, int device, rt_scene** out) {
  if (!xml_path || !out) return set_error(RT_E_INVALID, "rt_scene_load_xml: NULL argument");
  *out = nullptr;
  auto s = std::make_unique<rt_scene>();
  const int rc = guarded([&] {
    XmlSceneStorage st;
    rt_scene_desc d;
    load_scene_xml(xml_path, st, d);
    s->host.image_names = st.image_names;
    build_host_scene(d, s->host);
    return create_from_host(s.get(), device);
  });
  if (rc != RT_OK) {
    free_device(s.get());
    return rc;
  }
  *out = s.release();
  return RT_OK;
}

void rt_scene_destroy(rt_scene* s) {
  if (!s) return;
  free_device(s);
  delete s;
}

int rt_scene_num_cameras(const rt_scene* s) { return s ? (int)s->host.cameras.size() : 0; }
int rt_scene_num_lights(const rt_scene* s) { return s ? (int)s->host.lights.size() : 0; }
int rt_scene_bvh_depth(const rt_scene* s) { return s ? s->host.depth : 0; }

int rt_scene_camera(const rt_scene* s, int cam, rt_camera* out) {
  if (!s || !out || cam < 0 || cam >= (int)s->host.cameras.size())
    return set_error(RT_E_INVALID, "rt_scene_camera: bad argument");
  *out = s->host.cameras[cam];
  return RT_OK;
}

const char* rt_scene_image_name(const rt_scene* s, int cam) {
  if (!s || cam < 0 || cam >= (int)s->host.image_names.size()) return "";
  return s->host.image_names[cam].c_str();
}

int rt_scene_dump_bvh(const rt_scene* s, const char* path) {
  if (!s || !path) return set_error(RT_E_INVALID, "rt_scene_dump_bvh: NULL argument");
  FILE* f = std::fopen(path, "w");
  if (!f) return set_error(RT_E_IO, std::string("cannot open ") + path);
  const std::string d = dump_bvh(s->host);
  std::fwrite(d.data(), 1, d.size(), f);
  std::fclose(f);
  return RT_OK;
}

int rt_host_dump_bvh_xml(const char* xml_path, const char* out_path) {
  if (!xml_path || !out_path) return set_error(RT_E_INVALID, "rt_host_dump_bvh_xml: NULL argument");
  return guarded([&] {
    XmlSceneStorage st;
    rt_scene_desc d;
    load_scene_xml(xml_path, st, d);
    HostScene h;
    build_host_scene(d, h);
    FILE* f = std::fopen(out_path, "w");
    if (!f) throw std::ios_base::failure(std::string("cannot open ") + out_path);
    const std::string text = dump_bvh(h);
    std::fwrite(text.data(), 1, text.size(), f);
    std::fclose(f);
    return RT_OK;
  });
}

int rt_host_check_accel_xml(const char* xml_path, int treelet_leaves, long long* stats4) {
  if (!xml_path || !stats4) return set_error(RT_E_INVALID, "rt_host_check_accel_xml: NULL argument");
  return guarded([&] {
    XmlSceneStorage st;
    rt_scene_desc d;
    load_scene_xml(xml_path, st, d);
    HostScene h;
    build_host_scene(d, h);
    build_accel(h, treelet_leaves);
    const std::string err = check_accel(h, treelet_leaves, stats4);
    if (!err.empty()) throw std::invalid_argument("culling tree: " + err);
    return RT_OK;
  });
}

int rt_set_traversal(rt_scene* s, int mode) {
  if (!s || (mode != RT_TRAVERSAL_FAST && mode != RT_TRAVERSAL_REFERENCE &&
             mode != RT_TRAVERSAL_CULL))
    return set_error(RT_E_INVALID, "rt_set_traversal: bad argument");
  s->mode = mode;
  return RT_OK;
}

int rt_set_msaa_seed(rt_scene* s, unsigned long long seed) {
  if (!s) return set_error(RT_E_INVALID, "rt_set_msaa_seed: NULL scene");
  s->msaa_seed = seed;
  return RT_OK;
}

int rt_num_tiles(const rt_scene* s, int cam, int row0, int row_stride) {
  if (!s || cam < 0 || cam >= (int)s->host.cameras.size() || row0 < 0 || row_stride < 1)
    return set_error(RT_E_INVALID, "rt_num_tiles: bad argument");
  return plan(s->host.cameras[cam], row0, row_stride).tiles_total;
}

int rt_render_device(rt_scene* s, int cam, int row0, int row_stride, int tile_begin,
                     int tile_step, int tile_major, float* d_out, void* stream) {
  return rt_render_device_range(s, cam, row0, row_stride, tile_begin, tile_step, -1, tile_major,
                                d_out, stream);
}

// The scratch buffers of `stream`: the scene's own for the first stream it renders on, a set
// of its own (same sizes) for each further one.
struct Scratch {
  int2_t** hits;
  unsigned** occ;
  unsigned** sched;
  float** frames;
  size_t* frames_capacity;
  float** samples;
  size_t* samples_capacity;
};
Scratch scratch_for(rt_scene* s, void* stream) {
  std::lock_guard<std::mutex> lk(s->ctx_mu);
  if (!s->first_stream_set) {
    s->first_stream_set = true;
    s->first_stream = stream;
  }
  if (stream == s->first_stream)
    return {&s->d_hits, &s->d_occ, &s->d_sched, &s->d_frames, &s->frames_capacity,
            &s->d_samples, &s->samples_capacity};
  for (auto& x : s->streams)
    if (x.stream == stream)
      return {&x.hits, &x.occ, &x.sched, &x.frames, &x.frames_capacity, &x.samples,
              &x.samples_capacity};
  rt_scene::StreamScratch x{stream, nullptr, nullptr, nullptr, nullptr, 0, nullptr, 0};
  const size_t most = s->hits_capacity;
  try {
    hip_check(hipMalloc(&x.hits, most * sizeof(int2_t)), "alloc hit records");
    hip_check(hipMalloc(&x.occ, most * sizeof(unsigned) * occ_words(s->host)),
              "alloc occlusion bits");
    hip_check(hipMalloc(&x.sched, 2 * (most / (kTile * kTile)) * sizeof(unsigned)),
              "alloc tile schedule");
  } catch (...) {
    (void)hipFree(x.hits);
    (void)hipFree(x.occ);
    (void)hipFree(x.sched);
    throw;
  }
  s->streams.push_back(x);
  auto& y = s->streams.back();
  return {&y.hits, &y.occ, &y.sched, &y.frames, &y.frames_capacity, &y.samples,
          &y.samples_capacity};
}

int rt_render_device_range(rt_scene* s, int cam, int row0, int row_stride, int tile_begin,
                           int tile_step, int tile_count, int tile_major, float* d_out,
                           void* stream) {
  return guarded([&] {
      check_render_args(s, cam, row0, row_stride);
      if (tile_begin < 0 || tile_step < 1 || !d_out)
        throw std::invalid_argument("rt_render_device: bad tile selection / output");
      DeviceGuard g(s->device);
      const Scratch sc = scratch_for(s, stream);
      RenderParams P =
          make_params(s, cam, row0, row_stride, tile_begin, tile_step, tile_major, d_out, true);
      P.hits = *sc.hits;
      P.occ = *sc.occ;
      set_schedule(P, *sc.sched);
      if (tile_count >= 0 && tile_count < P.num_sel_tiles) {
        if (s->host.cameras[cam].num_samples > 1)
          throw std::domain_error("NumSamples > 1 renders whole row-major frames only");
        P.num_sel_tiles = tile_count;
      }
      if (s->needs_recursion) {
        const size_t need = frame_floats(s->host, P.num_sel_tiles);
        if (need > *sc.frames_capacity) {
          (void)hipFree(*sc.frames);
          *sc.frames = nullptr;
          *sc.frames_capacity = 0;
          hip_check(hipMalloc(sc.frames, need * sizeof(float)), "alloc ray-tree frames");
          *sc.frames_capacity = need;
        }
        P.frames = *sc.frames;
      }
      const rt_camera& c = s->host.cameras[cam];
      if (c.num_samples > 1) {
        if (tile_begin != 0 || tile_step != 1 || tile_major)
          throw std::domain_error("NumSamples > 1 renders whole row-major frames only");
        const size_t need = sample_floats(c);
        if (need > *sc.samples_capacity) {
          (void)hipFree(*sc.samples);
          *sc.samples = nullptr;
          *sc.samples_capacity = 0;
          hip_check(hipMalloc(sc.samples, need * sizeof(float)), "alloc MSAA samples");
          *sc.samples_capacity = need;
        }
      }
      enqueue_frame(s, P, c.num_samples, *sc.samples, (hipStream_t)stream);
      return RT_OK;
  });
}

int rt_collect_stats(rt_scene* s, rt_stats* stats) {
  if (!s || !stats) return set_error(RT_E_INVALID, "rt_collect_stats: NULL argument");
  return guarded([&] {
    DeviceGuard g(s->device);
    std::vector<unsigned long long> c(kCounterWidth * kCounterRows);
    hip_check(hipMemcpy(c.data(), s->d_counters, c.size() * sizeof c[0], hipMemcpyDeviceToHost),
              "read counters");
    hip_check(hipMemset(s->d_counters, 0, c.size() * sizeof c[0]), "reset counters");
    std::memset(stats, 0, sizeof *stats);
    for (int r = 0; r < kCounterRows; r++) {
      stats->primary_rays += (long long)c[kCounterWidth * r + kCntPrimary];
      stats->shadow_rays += (long long)c[kCounterWidth * r + kCntShadow];
      stats->secondary_rays += (long long)c[kCounterWidth * r + kCntSecondary];
      stats->primary_hits += (long long)c[kCounterWidth * r + kCntHits];
    }
    return RT_OK;
  });
}

int rt_debug_counters(rt_scene* s, long long* out16) {
  if (!s || !out16) return set_error(RT_E_INVALID, "rt_debug_counters: NULL argument");
  return guarded([&] {
    DeviceGuard g(s->device);
    std::vector<unsigned long long> c(kCounterWidth * kCounterRows);
    hip_check(hipMemcpy(c.data(), s->d_counters, c.size() * sizeof c[0], hipMemcpyDeviceToHost),
              "read counters");
    hip_check(hipMemset(s->d_counters, 0, c.size() * sizeof c[0]), "reset counters");
    for (int k = 0; k < kCounterWidth; k++) {
      unsigned long long sum = 0;
      for (int r = 0; r < kCounterRows; r++) sum += c[kCounterWidth * r + k];
      out16[k] = (long long)sum;
    }
    out16[kCntExactBox] = (long long)read_reset_exact_fallbacks();
    return diag_build() ? 1 : 0;
  });
}

long long rt_debug_timeline(unsigned long long* out, long long max_values) {
  if (!out || max_values < 0) return set_error(RT_E_INVALID, "rt_debug_timeline: bad argument");
  const long long n = read_reset_timeline(out, max_values);
  if (n < 0) return set_error(RT_E_INVALID, "rt_debug_timeline: buffer too small or copy failed");
  return n;
}

int rt_debug_quotient_check(int device, unsigned long long seed, long long count,
                            long long* out2) {
  if (!out2 || count < 0) return set_error(RT_E_INVALID, "rt_debug_quotient_check: bad argument");
  return guarded([&] {
    DeviceGuard g(device);
    unsigned long long* d = nullptr;
    hip_check(hipMalloc(&d, 2 * sizeof *d), "alloc");
    std::unique_ptr<unsigned long long, void (*)(unsigned long long*)> hold(
        d, [](unsigned long long* p) { (void)hipFree(p); });
    hip_check(hipMemset(d, 0, 2 * sizeof *d), "clear");
    hip_check(launch_quot_check(seed, count, d, nullptr), "quotient check launch");
    unsigned long long h[2];
    hip_check(hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost), "read");
    out2[0] = (long long)h[0];
    out2[1] = (long long)h[1];
    return RT_OK;
  });
}

int rt_render(rt_scene* s, int cam, int row0, int row_stride, float* out_rgb, rt_stats* stats) {
  return guarded([&] {
      check_render_args(s, cam, row0, row_stride);
      if (!out_rgb) throw std::invalid_argument("rt_render: out_rgb is NULL");
      DeviceGuard g(s->device);
      const rt_camera& c = s->host.cameras[cam];
      const TilePlan tp = plan(c, row0, row_stride);
      if (tp.rows == 0) return RT_OK;
      RenderCtx* x = acquire_ctx(s);
      struct Release {
        rt_scene* s;
        RenderCtx* x;
        ~Release() { release_ctx(s, x); }
      } release{s, x};
      const size_t frame = (size_t)c.width * c.height * 3;
      ensure(x->d_out, x->out_floats, frame, "alloc frame");
      // Counters are per scene; this call reports its own deltas via the context's buffer.
      hip_check(hipMemsetAsync(x->d_cnt, 0, sizeof(unsigned long long) * kCounterWidth * kCounterRows,
                               x->stream),
                "zero counters");
      RenderParams P = make_params(s, cam, row0, row_stride, 0, 1, 0, x->d_out, true);
      P.counters = x->d_cnt;
      const size_t lanes = (size_t)kTile * kTile * (size_t)std::max(1, P.num_sel_tiles);
      ensure(x->d_hits, x->hits_records, lanes, "alloc hit records");
      P.hits = x->d_hits;
      ensure(x->d_occ, x->occ_words, (size_t)P.occ_words * lanes, "alloc occlusion bits");
      P.occ = x->d_occ;
      ensure(x->d_sched, x->sched_words, 2 * lanes / (kTile * kTile), "alloc tile schedule");
      set_schedule(P, x->d_sched);
      if (s->needs_recursion) {
        ensure(x->d_frames, x->frames_floats, frame_floats(s->host, P.num_sel_tiles),
               "alloc ray-tree frames");
        P.frames = x->d_frames;
      }
      if (c.num_samples > 1)
        ensure(x->d_samples, x->samples_floats, sample_floats(c), "alloc MSAA samples");
      hip_check(hipEventRecord(x->e0, x->stream), "event record");
      enqueue_frame(s, P, c.num_samples, x->d_samples, x->stream);
      hip_check(hipEventRecord(x->e1, x->stream), "event record");
      // rows j = row0 + k*row_stride only: a strided 2D copy leaves the others untouched
      const size_t row_bytes = (size_t)c.width * 3 * sizeof(float);
      hip_check(hipMemcpy2DAsync(out_rgb + (size_t)row0 * c.width * 3, row_bytes * row_stride,
                                 x->d_out + (size_t)row0 * c.width * 3, row_bytes * row_stride,
                                 row_bytes, tp.rows, hipMemcpyDeviceToHost, x->stream),
                "copy rows");
      std::vector<unsigned long long> cnt(kCounterWidth * kCounterRows);
      hip_check(hipMemcpyAsync(cnt.data(), x->d_cnt, cnt.size() * sizeof cnt[0],
                               hipMemcpyDeviceToHost, x->stream),
                "copy counters");
      hip_check(hipStreamSynchronize(x->stream), "synchronize");
      if (stats) {
        std::memset(stats, 0, sizeof *stats);
        for (int r = 0; r < kCounterRows; r++) {
          stats->primary_rays += (long long)cnt[kCounterWidth * r + kCntPrimary];
          stats->shadow_rays += (long long)cnt[kCounterWidth * r + kCntShadow];
          stats->secondary_rays += (long long)cnt[kCounterWidth * r + kCntSecondary];
          stats->primary_hits += (long long)cnt[kCounterWidth * r + kCntHits];
        }
        float ms = 0;
        hip_check(hipEventElapsedTime(&ms, x->e0, x->e1), "elapsed");
        stats->kernel_ms = ms;
      }
      return RT_OK;
  });
}

int rt_set_kernel_timing(rt_scene* s, int enable) {
  if (!s) return set_error(RT_E_INVALID, "rt_set_kernel_timing: NULL scene");
  s->timing.on = enable != 0;
  return RT_OK;
}

int rt_read_kernel_times(rt_scene* s, double* ms4, long long* launches) {
  if (!s || !ms4) return set_error(RT_E_INVALID, "rt_read_kernel_times: NULL argument");
  return guarded([&] {
    DeviceGuard g(s->device);
    std::vector<std::array<hipEvent_t, 4>> done;
    {
      std::lock_guard<std::mutex> lk(s->ctx_mu);
      done.swap(s->timing.pending);
    }
    double sum[4] = {0, 0, 0, 0};
    for (auto& q : done) {
      hip_check(hipEventSynchronize(q[3]), "timing sync");
      float a = 0, b = 0, c = 0;
      hip_check(hipEventElapsedTime(&a, q[0], q[1]), "elapsed");
      hip_check(hipEventElapsedTime(&b, q[1], q[2]), "elapsed");
      hip_check(hipEventElapsedTime(&c, q[2], q[3]), "elapsed");
      sum[0] += a;
      sum[1] += b;
      sum[2] += c;
      sum[3] += (double)a + b + c;
    }
    std::memcpy(ms4, sum, sizeof sum);
    if (launches) *launches = (long long)done.size();
    std::lock_guard<std::mutex> lk(s->ctx_mu);
    for (auto& q : done) s->timing.spare.push_back(q);
    return RT_OK;
  });
}

int rt_write_png(const char* path, const float* rgb, int width, int height) {
  if (!path || !rgb) return set_error(RT_E_INVALID, "rt_write_png: NULL argument");
  return guarded([&] {
    write_png(path, rgb, width, height);
    return RT_OK;
  });
}

}  // extern "C"
