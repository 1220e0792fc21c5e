// C-ABI implementation (include/ceng795_rt.h): scene upload, render launches, counters,
// multi-device frames.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
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
                         bool fast, bool deep, bool spheres, const hipEvent_t* marks,
                         hipStream_t stream);
int max_supported_depth();
hipError_t launch_msaa_resolve(const MsaaResolveParams& M, hipStream_t stream);
hipError_t launch_untile(const UntileParams& U, hipStream_t stream);
hipError_t launch_resolve_rows(const RenderParams& P, const unsigned* rec, int row_begin,
                               int row_end, bool spheres, hipStream_t stream);
hipError_t launch_resolve(const RenderParams& P, const UntileParams& U, bool spheres,
                          hipStream_t stream);
unsigned long long read_reset_exact_fallbacks();
hipError_t launch_quot_check(unsigned long long seed, long long count, unsigned long long* counts,
                             hipStream_t stream);
bool diag_build();
long long read_reset_timeline(unsigned long long* out, long long max_values);
long long read_reset_phases(unsigned long long* out, long long max_values);
int launch_cold_order(RenderParams P, hipStream_t stream);
void write_png(const std::string& path, const float* rgb, int w, int h);
}  // namespace rt

using namespace rt;

// Device buffers of one synchronous call (rt_render, and every device's share of a
// multi-device frame), kept by the scene and reused: the reference calls render_image once per
// thread per camera (HW2/main.cpp:33-36), so a drop-in pays hipMalloc / hipFree only the first
// time a call of that size runs.  Calls on several host threads each take their own context
// (rt_render stays reentrant).
// rt_render into a caller buffer in pinned host memory: the frame kernel writes it directly
// (its device-visible address; C3 one frame at a time 0.94-0.97 -> 0.67-0.69 ms).  Into a
// pageable buffer: the frame as RT_RENDER_CHUNKS bands of tile rows, one launch each, each band
// copied out on a second stream as soon as it is done.  (The copies are blit kernels here,
// which wait for CU slots the render holds: pageable 1.00-1.05 ms unbanded, 0.89 with 2 bands,
// 0.98 with 4, 1.36 with 8; a high-priority copy stream changed nothing —
// profiles/r06/host_rate_bands.jsonl.)
#ifndef RT_DIRECT_PINNED  // (A/B builds)
#define RT_DIRECT_PINNED 1
#endif
#ifndef RT_RENDER_CHUNKS  // (A/B builds)
#define RT_RENDER_CHUNKS 2
#endif
constexpr int kRenderChunks = RT_RENDER_CHUNKS;

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
  float* d_recv = nullptr;  // multi-device frames, first device: the gathered tiles
  size_t recv_floats = 0;
  float* d_image = nullptr;  // multi-device rt_render, first device: the row-major frame
  size_t image_floats = 0;
  hipEvent_t ev_in = nullptr, ev_out = nullptr;  // multi-device frames: caller-stream ordering
  // copy-gather frames (a device listed twice): recorded on the first device's stream after it
  // has copied the shares out of the other contexts' buffers; a context renders its next share
  // only after it (the copy reads d_out / d_image on another stream: write-after-read)
  hipEvent_t ev_gathered = nullptr;
  // rt_render's chunked copy-out (render_to_host): a second stream for the device-to-host copies
  // and one event per row chunk (created on first use)
  hipStream_t copy_stream = nullptr;
  hipEvent_t ev_chunk[kRenderChunks] = {};
};

// rt_render_device scratch of one stream (hit records, occlusion bits, tile schedule, ray-tree
// frames, MSAA samples).  Owned through a unique_ptr, so its address is stable while the table
// grows; `mu` serialises host threads that enqueue on the same stream.
struct StreamScratch {
  void* stream = nullptr;
  std::mutex mu;
  int2_t* hits = nullptr;
  unsigned* occ = nullptr;
  unsigned* sched = nullptr;
  float* frames = nullptr;
  size_t frames_capacity = 0;
  float* samples = nullptr;
  size_t samples_capacity = 0;
  // warm order: the selection whose heavy-first unit order the last frame on this stream left
  // in `sched` (valid: that frame ran the order kernel)
  std::array<long long, 7> order_key{};
  bool order_valid = false;
  hipEvent_t done = nullptr;  // after the last frame enqueued on the stream (eviction waits on it)
  unsigned long long used = 0;  // Replica::tick of the last lookup (least recently used first)
};

// Streams a replica keeps scratch / a multi-device context for: beyond this many, the least
// recently used one is released (after its work has finished), so callers that make a new
// stream per frame do not grow device memory without bound.
constexpr size_t kMaxStreamTables = 64;

// Per-kernel HIP-event timing of render launches (rt_set_kernel_timing): one quad of events per
// launch of the first device.  Completed quads beyond kTimingPending are folded into `sum` so
// the list stays bounded while timing is on and nobody reads it.
struct KernelTiming {
  bool on = false;
  std::vector<std::array<hipEvent_t, 4>> pending, spare;
  double sum[4] = {0, 0, 0, 0};
  long long folded = 0;
};
constexpr size_t kTimingPending = 256;

// The scene on one device: the flattened scene in HBM, the ray counters, and the buffers of
// the calls that run there.
struct Replica {
  int device = 0;
  DevNode* d_nodes = nullptr;
  DevPrim* d_prims = nullptr;
  DevLeaf* d_leaves = nullptr;
  float* d_normals = nullptr;
  DevAncestry* d_anc = nullptr;
  DevMaterial* d_mats = nullptr;
  DevLight* d_lights = nullptr;
  unsigned long long* d_counters = nullptr;
  // per camera: its whole frame's cold order (seed_cold_orders), sched_words_for(tiles) words
  // laid out as a stream's `sched` (estimated costs, unit order, snapshot); nullptr: none
  std::vector<unsigned*> d_cold;
  std::mutex mu;  // ctx pool and stream tables
  std::vector<RenderCtx*> ctx_free, ctx_all;
  std::vector<std::unique_ptr<StreamScratch>> streams;
  // multi-device scenes: the context each caller stream renders its shares on (one per caller
  // stream and device, kept across calls), so frames on different caller streams have their
  // own device streams and buffers and overlap (frames in flight, as scratch_for on one device)
  std::vector<std::pair<void*, RenderCtx*>> stream_ctx;
  unsigned long long tick = 0;  // lookups of `streams` (LRU order)
};

struct rt_scene {
  HostScene host;
  int mode = RT_TRAVERSAL_FAST;
  bool deep = false;
  bool needs_recursion = false;
  bool has_spheres = false;
  size_t most = 1;         // pixel records of the largest camera frame (whole tiles)
  unsigned long long msaa_seed = 0;
  std::vector<std::unique_ptr<Replica>> rep;  // rep[0]: the first (output) device
  std::mutex timing_mu;
  KernelTiming timing;
  // multi-device scenes: one RCCL communicator per device (single process, ncclCommInitAll);
  // multi_mu serialises the frames that use them.  copy_gather: the shares are gathered by
  // peer copies instead (a device listed twice: the one-GPU rehearsal of the deal / gather /
  // untile path)
  std::mutex multi_mu;
  std::vector<ncclComm_t> comms;
  bool multi = false;  // made by rt_scene_*_multi: frames go through render_multi (any count)
  bool copy_gather = false;
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

struct NcclFailure {
  ncclResult_t err;
  const char* what;
};

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw HipFailure{e, what};
}

void nccl_check(ncclResult_t e, const char* what) {
  if (e != ncclSuccess) throw NcclFailure{e, what};
}

template <typename F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const HipFailure& h) {
    return set_error(RT_E_HIP, std::string(h.what) + ": " + hipGetErrorString(h.err));
  } catch (const NcclFailure& h) {
    return set_error(RT_E_HIP, std::string(h.what) + ": " + ncclGetErrorString(h.err));
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
  (void)hipFree(c->d_recv);
  (void)hipFree(c->d_image);
  if (c->ev_in) (void)hipEventDestroy(c->ev_in);
  if (c->ev_out) (void)hipEventDestroy(c->ev_out);
  if (c->ev_gathered) (void)hipEventDestroy(c->ev_gathered);
  if (c->e0) (void)hipEventDestroy(c->e0);
  if (c->e1) (void)hipEventDestroy(c->e1);
  for (hipEvent_t e : c->ev_chunk)
    if (e) (void)hipEventDestroy(e);
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

void free_scratch(StreamScratch& x) {
  (void)hipFree(x.hits);
  (void)hipFree(x.occ);
  (void)hipFree(x.sched);
  (void)hipFree(x.frames);
  (void)hipFree(x.samples);
  if (x.done) (void)hipEventDestroy(x.done);
  x.done = nullptr;
}

void free_replica(Replica& r) {
  int cur = 0;
  if (hipGetDevice(&cur) == hipSuccess && cur != r.device) (void)hipSetDevice(r.device);
  for (RenderCtx* c : r.ctx_all) free_ctx(c);
  r.ctx_all.clear();
  r.ctx_free.clear();
  r.stream_ctx.clear();
  for (auto& x : r.streams) free_scratch(*x);
  r.streams.clear();
  (void)hipFree(r.d_nodes);
  (void)hipFree(r.d_prims);
  (void)hipFree(r.d_leaves);
  (void)hipFree(r.d_normals);
  (void)hipFree(r.d_anc);
  (void)hipFree(r.d_mats);
  (void)hipFree(r.d_lights);
  (void)hipFree(r.d_counters);
  for (unsigned* p : r.d_cold) (void)hipFree(p);
  r.d_cold.clear();
  if (cur != r.device) (void)hipSetDevice(cur);
}

void free_device(rt_scene* s) {
  for (ncclComm_t c : s->comms) (void)ncclCommDestroy(c);
  s->comms.clear();
  if (!s->rep.empty()) {
    int cur = 0;
    const int d0 = s->rep[0]->device;
    if (hipGetDevice(&cur) == hipSuccess && cur != d0) (void)hipSetDevice(d0);
    for (auto* v : {&s->timing.pending, &s->timing.spare})
      for (auto& q : *v)
        for (hipEvent_t e : q) (void)hipEventDestroy(e);
    if (cur != d0) (void)hipSetDevice(cur);
  }
  s->timing.pending.clear();
  s->timing.spare.clear();
  for (auto& r : s->rep) free_replica(*r);
  s->rep.clear();
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
constexpr size_t kTileFloats = (size_t)kTile * kTile * 3;

size_t frame_floats(const HostScene& h, int sel_tiles) {
  return (size_t)(h.max_depth + 1) * kFrameFloats * kTile * kTile * (size_t)std::max(1, sel_tiles);
}

int occ_words(const HostScene& h) { return std::max(1, ((int)h.lights.size() + 31) / 32); }

// A counter buffer: kCounterRows x kCounterWidth ray counters.
constexpr size_t kCounterAlloc = (size_t)kCounterWidth * kCounterRows;
// Dispatch order of the traversal kernels: heavy first within each XCD's
// part of the frame (RT_ORDER_REGIONS regions, one per XCD; 0 = block order), each region
// RT_ORDER_CHUNKS contiguous bands of the frame, chunk c in region c mod regions.  Two: an XCD's
// L2 still holds its bands' part of the tree (shadow kernel reads 91 vs 130 MB per C3 frame with
// interleaved half-row chunks, profiles/r03/ab_order_chunks.jsonl), and two bands half a frame
// apart even out the XCDs' shares of the heavy rows (C3 frame kernel 0.352 -> 0.339 ms one at a
// time, 0.327 -> 0.319 six in flight; 4 / 8 / 16 chunks 0.343 / 0.343 / 0.346;
// profiles/r06/ab_order_chunks.json).  The order never changes a result, only which tiles start
// first.  (Macros: A/B builds, `make exp EXTRA=-D...`.)
#ifndef RT_ORDER_REGIONS
#define RT_ORDER_REGIONS 8
#endif
#ifndef RT_ORDER_CHUNKS
#define RT_ORDER_CHUNKS 2
#endif
// sched: sched_words_for(num_sel_tiles) words — tile costs, then the unit order lists
// The untile kernel copies 16-B chunks when every frame row and both buffers are 16-B aligned.
int untile_vec(const UntileParams& U) {
  return (U.width % 4 == 0) && ((uintptr_t)U.out % 16 == 0) && ((uintptr_t)U.recv % 16 == 0);
}


void set_schedule(RenderParams& P, unsigned* sched) {
  const int regions = RT_ORDER_REGIONS;
  P.tile_cost = regions ? sched : nullptr;
  P.unit_order = regions ? reinterpret_cast<int*>(sched) + P.num_sel_tiles : nullptr;
  P.order_regions = regions;
  P.order_chunk = RT_ORDER_CHUNKS;
}

// Estimated cost of every tile of camera c's whole frame, for the dispatch order of a frame
// without a previous one (the cold frame): 16 x (1 + the primitives whose
// projected bounds touch the tile, each weighted by 1 / |cos| of the angle between its normal
// and the view direction, at most 20).  Where many primitives project into one tile — surfaces
// seen edge-on — its rays walk more of the tree (C3: correlation 0.62 with measured tile times,
// 0.59 unweighted).  A point X projects to the image-plane point tl + su fx - sv fy that
// e + l (X - e) reaches (Cramer's rule; l > 0: in front of the camera); a primitive with a point
// not in front is left out.  Only the order depends on it, never a pixel.
#ifndef RT_COLD_WEIGHT  // (A/B builds: 0 = every primitive counts 1)
#define RT_COLD_WEIGHT 1
#endif
std::vector<unsigned> cold_costs(const HostScene& h, const rt_camera& c) {
  const int tx = (c.width + kTile - 1) / kTile, ty = (c.height + kTile - 1) / kTile;
  std::vector<double> acc((size_t)tx * ty, 1.0);
  const double e[3] = {c.e[0], c.e[1], c.e[2]};
  const double nu[3] = {-c.s_u[0], -c.s_u[1], -c.s_u[2]}, sv[3] = {c.s_v[0], c.s_v[1], c.s_v[2]};
  const double r[3] = {c.top_left[0] - e[0], c.top_left[1] - e[1], c.top_left[2] - e[2]};
  auto cross = [](const double* a, const double* b, double* o) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
  };
  auto dot = [](const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; };
  double nuxsv[3], rxsv[3], nuxr[3];
  cross(nu, sv, nuxsv);
  cross(r, sv, rxsv);
  cross(nu, r, nuxr);
  const double lnum = dot(r, nuxsv);
  auto project = [&](const double* X, double& fx, double& fy) {
    const double a[3] = {X[0] - e[0], X[1] - e[1], X[2] - e[2]};
    const double det = dot(a, nuxsv);
    if (!(std::fabs(det) > 0.0) || !(lnum / det > 0.0)) return false;
    fx = dot(a, rxsv) / det;
    fy = dot(a, nuxr) / det;
    return std::isfinite(fx) && std::isfinite(fy);
  };
  for (const DevPrim& p : h.prims) {
    double pts[8][3];
    int n = 0;
    double weight = 1.0;
    if (p.kind == kPrimTriangle) {
      for (int k = 0; k < 3; k++) {
        pts[0][k] = p.v0[k];
        pts[1][k] = (double)p.v0[k] - p.a1[k];
        pts[2][k] = (double)p.v0[k] - p.a2[k];
      }
      n = 3;
      if (RT_COLD_WEIGHT) {
        const double a1[3] = {p.a1[0], p.a1[1], p.a1[2]}, a2[3] = {p.a2[0], p.a2[1], p.a2[2]};
        double nrm[3];
        cross(a1, a2, nrm);
        const double d[3] = {(pts[0][0] + pts[1][0] + pts[2][0]) / 3 - e[0],
                             (pts[0][1] + pts[1][1] + pts[2][1]) / 3 - e[1],
                             (pts[0][2] + pts[1][2] + pts[2][2]) / 3 - e[2]};
        const double len = std::sqrt(dot(nrm, nrm) * dot(d, d));
        const double cosv = len > 0.0 ? std::fabs(dot(nrm, d)) / len : 1.0;
        weight = 1.0 / std::max(cosv, 0.05);
      }
    } else {
      const double rad = std::fabs((double)p.a1[0]);
      for (int m = 0; m < 8; m++)
        for (int k = 0; k < 3; k++) pts[m][k] = p.v0[k] + (((m >> k) & 1) ? rad : -rad);
      n = 8;
    }
    double x0 = 1e300, x1 = -1e300, y0 = 1e300, y1 = -1e300;
    bool ok = true;
    for (int m = 0; m < n && ok; m++) {
      double fx, fy;
      ok = project(pts[m], fx, fy);
      if (ok) {
        x0 = std::min(x0, fx), x1 = std::max(x1, fx);
        y0 = std::min(y0, fy), y1 = std::max(y1, fy);
      }
    }
    if (!ok || x1 < 0.0 || y1 < 0.0 || x0 >= c.width || y0 >= c.height) continue;
    const int a0 = std::max(0, (int)(x0 / kTile)), a1 = std::min(tx - 1, (int)(x1 / kTile));
    const int b0 = std::max(0, (int)(y0 / kTile)), b1 = std::min(ty - 1, (int)(y1 / kTile));
    for (int b = b0; b <= b1; b++)
      for (int a = a0; a <= a1; a++) acc[(size_t)b * tx + a] += weight;
  }
  std::vector<unsigned> est(acc.size());
  for (size_t i = 0; i < acc.size(); i++) est[i] = (unsigned)std::min(16.0 * acc[i], 4e9);
  return est;
}

RenderParams make_params(const rt_scene* s, const Replica& r, int cam, int row0, int row_stride,
                         int tile_begin, int tile_step, int tile_major, float* out,
                         unsigned long long* counters);

// Every orderable camera's whole-frame cold order on replica r (the order kernel over
// cold_costs), made once with the scene: a camera's first frame on a stream dispatches by it
// instead of in block order (launch_variant in rt_kernels.hip).
void seed_cold_orders(const rt_scene* s, Replica& r) {
  const HostScene& h = s->host;
#ifndef RT_COLD_SEED  // (A/B builds: 0 = cold frames in block order)
#define RT_COLD_SEED 1
#endif
  r.d_cold.assign(h.cameras.size(), nullptr);
  if (!RT_COLD_SEED || s->needs_recursion || h.lights.empty()) return;  // (no warm order either)
  for (size_t cam = 0; cam < h.cameras.size(); cam++) {
    const rt_camera& c = h.cameras[cam];
    if (c.num_samples > 1) continue;
    const std::vector<unsigned> est = cold_costs(h, c);
    unsigned* buf = nullptr;
    hip_check(hipMalloc(&buf, sched_words_for(est.size()) * sizeof(unsigned)), "alloc cold order");
    hip_check(hipMemcpy(buf, est.data(), est.size() * sizeof(unsigned), hipMemcpyHostToDevice),
              "upload tile cost estimate");
    RenderParams P = make_params(s, r, (int)cam, 0, 1, 0, 1, 0, nullptr, nullptr);
    set_schedule(P, buf);
    if (launch_cold_order(P, nullptr)) {
      r.d_cold[cam] = buf;
    } else {
      (void)hipFree(buf);
    }
  }
  hip_check(hipDeviceSynchronize(), "cold orders");
}

void upload_replica(const rt_scene* s, Replica& r) {
  DeviceGuard g(r.device);
  const HostScene& h = s->host;
  r.d_nodes = upload(h.nodes, "upload nodes");
  r.d_prims = upload(h.prims, "upload prims");
  r.d_leaves = upload(h.leaves, "upload culling leaves");
  r.d_normals = upload(h.normals, "upload normals");
  r.d_anc = upload(h.ancestry, "upload ancestry");
  r.d_mats = upload(h.materials, "upload materials");
  r.d_lights = upload(h.lights, "upload lights");
  hip_check(hipMalloc(&r.d_counters, sizeof(unsigned long long) * kCounterAlloc), "alloc counters");
  hip_check(hipMemset(r.d_counters, 0, sizeof(unsigned long long) * kCounterAlloc), "zero counters");
  seed_cold_orders(s, r);
}

// Builds the culling tree once on the host, then uploads the scene to every device.  Several
// devices: one RCCL communicator each, for the framebuffer gather (render_multi).
int create_from_host(rt_scene* s, const std::vector<int>& devices, bool multi) {
  build_accel(s->host, kDefaultTreeletLeaves);
  if (s->host.accel_depth > max_supported_depth()) build_accel(s->host, 0);
  const HostScene& h = s->host;
  if (h.prims.size() >= (size_t(1) << 26))  // leaf indices share a 32-bit queue word with a lane
    throw std::invalid_argument("scenes of 2^26 primitives or more are not supported");
  if (h.depth > max_supported_depth())
    throw std::invalid_argument("BVH deeper than " + std::to_string(max_supported_depth()) +
                                " levels is not supported");
  s->deep = std::max(h.depth, h.accel_depth) > kLaneStack - 2;
  for (const DevPrim& p : h.prims) s->has_spheres |= p.kind == kPrimSphere;
  for (const DevMaterial& m : h.materials) {
    const bool mirror = m.mirror[0] != 0 || m.mirror[1] != 0 || m.mirror[2] != 0;
    const bool glass = m.transparency[0] != 0 || m.transparency[1] != 0 || m.transparency[2] != 0;
    if ((mirror || glass) && h.max_depth > 0) s->needs_recursion = true;
  }
  for (const rt_camera& c : h.cameras) {
    const size_t tiles = (size_t)((c.width + kTile - 1) / kTile) * ((c.height + kTile - 1) / kTile);
    s->most = std::max(s->most, tiles * kTile * kTile);
  }
  for (int d : devices) {
    s->rep.push_back(std::make_unique<Replica>());
    s->rep.back()->device = d;
    upload_replica(s, *s->rep.back());
  }
  s->multi = multi;
  if (multi) {
    std::vector<int> distinct = devices;
    std::sort(distinct.begin(), distinct.end());
    s->copy_gather = std::unique(distinct.begin(), distinct.end()) != distinct.end();
    if (!s->copy_gather) {
      s->comms.resize(devices.size());
      nccl_check(ncclCommInitAll(s->comms.data(), (int)devices.size(), devices.data()),
                 "ncclCommInitAll");
    }
  }
  return RT_OK;
}

std::vector<int> device_list(int device_count, const int* devices) {
  int n = 0;
  hip_check(hipGetDeviceCount(&n), "hipGetDeviceCount");
  if (device_count < 1) throw std::invalid_argument("device_count must be >= 1");
  std::vector<int> out;
  for (int i = 0; i < device_count; i++) {
    const int d = devices ? devices[i] : i;
    if (d < 0 || d >= n)
      throw std::invalid_argument("device " + std::to_string(d) + " does not exist (" +
                                  std::to_string(n) + " visible)");
    out.push_back(d);
  }
  return out;
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

RenderParams make_params(const rt_scene* s, const Replica& r, int cam, int row0, int row_stride,
                         int tile_begin, int tile_step, int tile_major, float* out,
                         unsigned long long* counters) {
  const HostScene& h = s->host;
  const rt_camera& c = h.cameras[cam];
  RenderParams P;
  std::memset(&P, 0, sizeof P);
  P.nodes = r.d_nodes;
  P.leaves = r.d_leaves;
  P.prims = r.d_prims;
  P.normals = r.d_normals;
  P.materials = r.d_mats;
  P.lights = r.d_lights;
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
  P.anc = r.d_anc;
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
  P.block_deal = (tile_major & RT_TILE_BLOCKS) ? 1 : 0;
  const int units = P.block_deal ? deal_blocks(tp.tiles_x, tp.tiles_total / tp.tiles_x) : tp.tiles_total;
  const int sel_units = tile_begin < units ? (units - tile_begin + tile_step - 1) / tile_step : 0;
  P.num_sel_tiles = P.block_deal ? 4 * sel_units : sel_units;
  P.tile_major = tile_major & RT_TILE_MAJOR;
  P.records = (tile_major & RT_TILE_RECORDS) ? 1 : 0;
  P.out = out;
  P.occ_words = occ_words(h);
  P.counters = counters;
  if (row0 == 0 && row_stride == 1 && tile_begin == 0 && tile_step == 1 && !P.block_deal &&
      cam < (int)r.d_cold.size() && r.d_cold[cam]) {  // the whole frame: its cold order
    P.cold_order = reinterpret_cast<const int*>(r.d_cold[cam]) + P.num_sel_tiles;
    P.cold_tiles = P.num_sel_tiles;
  }
  return P;
}

// P restricted to its first `rows` selected rows (rows row0 .. row0 + rows - 1 at stride 1):
// the band launches of a multi-device MSAA frame.
void limit_rows(RenderParams& P, int rows) {
  P.rows = std::min(P.rows, rows);
  P.tiles_total = P.tiles_x * ((P.rows + kTile - 1) / kTile);
  P.num_sel_tiles = P.tile_begin < P.tiles_total
                        ? (P.tiles_total - P.tile_begin + P.tile_step - 1) / P.tile_step
                        : 0;
}

// Pixel records (RT_TILE_RECORDS) carry the primary hit and up to kRecMaxLights shadow bits:
// pixel-centre cameras of scenes without mirror/dielectric recursion.
bool records_ok(const rt_scene* s, int cam) {
  return s->host.cameras[cam].num_samples <= 1 && !s->needs_recursion &&
         (int)s->host.lights.size() <= kRecMaxLights;
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

// Folds the completed quads at the front of the pending list into the running sums.
void fold_timing(KernelTiming& t) {
  size_t k = 0;
  for (; k < t.pending.size(); k++) {
    auto& q = t.pending[k];
    if (hipEventQuery(q[3]) != hipSuccess) break;
    float a = 0, b = 0, c = 0;
    if (hipEventElapsedTime(&a, q[0], q[1]) != hipSuccess ||
        hipEventElapsedTime(&b, q[1], q[2]) != hipSuccess ||
        hipEventElapsedTime(&c, q[2], q[3]) != hipSuccess)
      break;
    t.sum[0] += a;
    t.sum[1] += b;
    t.sum[2] += c;
    t.sum[3] += (double)a + b + c;
    t.folded++;
    t.spare.push_back(q);
  }
  t.pending.erase(t.pending.begin(), t.pending.begin() + (long)k);
}

// Events for one timed launch (nullptr when timing is off or the launch renders nothing).
const hipEvent_t* timing_marks(rt_scene* s, const RenderParams& P) {
  if (!s->timing.on || P.num_sel_tiles <= 0) return nullptr;
  std::lock_guard<std::mutex> lk(s->timing_mu);
  KernelTiming& t = s->timing;
  if (t.pending.size() >= kTimingPending) fold_timing(t);
  if (t.spare.empty()) {
    std::array<hipEvent_t, 4> q{};
    for (hipEvent_t& e : q) hip_check(hipEventCreate(&e), "timing event");
    t.spare.push_back(q);
  }
  t.pending.push_back(t.spare.back());
  t.spare.pop_back();
  return t.pending.back().data();
}

// The sample passes of an MSAA camera (HW2/Scene.cpp:32-69) over P's rows: pass k renders
// sample k of every selected pixel into d_samples[k] (row-major, full-frame positions).
void enqueue_samples(rt_scene* s, const Replica& r, const RenderParams& P, int samples,
                     float* d_samples, hipStream_t stream, bool timed) {
  const bool fast = s->mode != RT_TRAVERSAL_REFERENCE;
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
    hip_check(launch_render(Q, r.d_nodes, r.d_prims, r.d_normals, r.d_mats, r.d_lights, fast,
                            s->deep, s->has_spheres, timed ? timing_marks(s, Q) : nullptr, stream),
              "render launch");
  }
}

// The splat + colour / weight of rows [row_lo, row_hi) into out (row-major, full frame).
void enqueue_resolve(rt_scene* s, int width, int height, int samples, const float* d_samples,
                     float* out, int row_lo, int row_hi, hipStream_t stream) {
  MsaaResolveParams M;
  M.samples = d_samples;
  M.out = out;
  M.width = width;
  M.height = height;
  M.n = samples;
  M.seed = s->msaa_seed;
  M.row_lo = row_lo;
  M.row_hi = row_hi;
  hip_check(launch_msaa_resolve(M, stream), "msaa resolve launch");
}

// One frame (or a tile subset of one) of camera `cam` into P.out.  Pixel-centre cameras: the
// render kernels write P.out directly.  MSAA cameras (HW2/Scene.cpp:32-69): one render pass per
// sample index into d_samples[s], then the resolve kernel's splat + colour / weight into P.out
// (row-major).  `timed`: this launch may take kernel-timing events (the first device only).
void enqueue_frame(rt_scene* s, const Replica& r, const RenderParams& P, int samples,
                   float* d_samples, hipStream_t stream, bool timed) {
  const bool fast = s->mode != RT_TRAVERSAL_REFERENCE;
  if (samples <= 1) {
    hip_check(launch_render(P, r.d_nodes, r.d_prims, r.d_normals, r.d_mats, r.d_lights, fast,
                            s->deep, s->has_spheres, timed ? timing_marks(s, P) : nullptr, stream),
              "render launch");
    return;
  }
  enqueue_samples(s, r, P, samples, d_samples, stream, timed);
  enqueue_resolve(s, P.width, P.height, samples, d_samples, P.out, 0, P.height, stream);
}

size_t sample_floats(const rt_camera& c) {
  return c.num_samples > 1 ? (size_t)c.num_samples * c.num_samples * c.width * c.height * 3 : 0;
}

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

RenderCtx* acquire_ctx(Replica& r) {
  {
    std::lock_guard<std::mutex> lk(r.mu);
    if (!r.ctx_free.empty()) {
      RenderCtx* c = r.ctx_free.back();
      r.ctx_free.pop_back();
      return c;
    }
  }
  DeviceGuard g(r.device);
  std::unique_ptr<RenderCtx> c(new RenderCtx);
  try {
    hip_check(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking), "stream");
    hip_check(hipEventCreate(&c->e0), "event");
    hip_check(hipEventCreate(&c->e1), "event");
    hip_check(hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming), "event");
    hip_check(hipEventCreateWithFlags(&c->ev_out, hipEventDisableTiming), "event");
    hip_check(hipEventCreateWithFlags(&c->ev_gathered, hipEventDisableTiming), "event");
    hip_check(hipEventRecord(c->ev_gathered, c->stream), "event record");  // (complete)
    hip_check(hipMalloc(&c->d_cnt, sizeof(unsigned long long) * kCounterAlloc), "alloc counters");
  } catch (...) {
    free_ctx(c.release());
    throw;
  }
  std::lock_guard<std::mutex> lk(r.mu);
  r.ctx_all.push_back(c.get());
  return c.release();
}

void release_ctx(Replica& r, RenderCtx* c) {
  std::lock_guard<std::mutex> lk(r.mu);
  r.ctx_free.push_back(c);
}

// The context of caller stream `stream` on replica r (created on first use, then kept; the
// table is capped at kMaxStreamTables: the oldest caller stream's context goes back to the pool
// once its device stream has drained).  Caller holds s->multi_mu (no other multi-device frame
// is being enqueued).
RenderCtx* stream_ctx_for(Replica& r, void* stream) {
  RenderCtx* old = nullptr;
  {
    std::lock_guard<std::mutex> lk(r.mu);
    for (size_t k = 0; k < r.stream_ctx.size(); k++)
      if (r.stream_ctx[k].first == stream) {
        std::rotate(r.stream_ctx.begin() + (long)k, r.stream_ctx.begin() + (long)k + 1,
                    r.stream_ctx.end());  // most recently used last
        return r.stream_ctx.back().second;
      }
    if (r.stream_ctx.size() >= kMaxStreamTables) {
      old = r.stream_ctx.front().second;
      r.stream_ctx.erase(r.stream_ctx.begin());
    }
  }
  if (old) {
    DeviceGuard g(r.device);
    hip_check(hipStreamSynchronize(old->stream), "synchronize evicted context");
    release_ctx(r, old);
  }
  RenderCtx* c = acquire_ctx(r);
  std::lock_guard<std::mutex> lk(r.mu);
  r.stream_ctx.emplace_back(stream, c);
  return c;
}

// Contexts of one call on several replicas: pooled ones handed back on scope exit (rt_render),
// or the caller stream's own (rt_render_device: consecutive frames on different caller streams
// then run on different device streams, and frames on one caller stream stay ordered).
struct CtxSet {
  rt_scene* s;
  std::vector<RenderCtx*> x;
  bool pooled = true;
  CtxSet(rt_scene* sc, size_t n) : s(sc) {
    for (size_t d = 0; d < n; d++) x.push_back(acquire_ctx(*s->rep[d]));
  }
  CtxSet(rt_scene* sc, size_t n, void* stream) : s(sc), pooled(false) {
    for (size_t d = 0; d < n; d++) x.push_back(stream_ctx_for(*s->rep[d], stream));
  }
  ~CtxSet() {
    if (!pooled) return;
    for (size_t d = 0; d < x.size(); d++) release_ctx(*s->rep[d], x[d]);
  }
};

// Sizes a context's per-call buffers for `sel_tiles` selected tiles of camera `cam` and points
// P at them.
void bind_ctx(rt_scene* s, RenderCtx* x, RenderParams& P, const rt_camera& c) {
  const size_t lanes = (size_t)kTile * kTile * (size_t)std::max(1, P.num_sel_tiles);
  ensure(x->d_hits, x->hits_records, lanes, "alloc hit records");
  P.hits = x->d_hits;
  ensure(x->d_occ, x->occ_words, (size_t)P.occ_words * lanes, "alloc occlusion bits");
  P.occ = x->d_occ;
  ensure(x->d_sched, x->sched_words, (size_t)sched_words_for(lanes / (kTile * kTile)),
         "alloc tile schedule");
  set_schedule(P, x->d_sched);
  if (s->needs_recursion) {
    ensure(x->d_frames, x->frames_floats, frame_floats(s->host, P.num_sel_tiles),
           "alloc ray-tree frames");
    P.frames = x->d_frames;
  }
  if (c.num_samples > 1) ensure(x->d_samples, x->samples_floats, sample_floats(c), "alloc MSAA samples");
}

void add_counters(const std::vector<unsigned long long>& cnt, rt_stats* stats) {
  for (int r = 0; r < kCounterRows; r++) {
    stats->primary_rays += (long long)cnt[kCounterWidth * r + kCntPrimary];
    stats->shadow_rays += (long long)cnt[kCounterWidth * r + kCntShadow];
    stats->secondary_rays += (long long)cnt[kCounterWidth * r + kCntSecondary];
    stats->primary_hits += (long long)cnt[kCounterWidth * r + kCntHits];
  }
}

// One frame of an MSAA camera over every device of a multi-device scene (the
// Gaussian splat of HW2/Scene.cpp:51-63 reaches the 3x3 neighbours, so pixels do not shard as
// independent tiles).  Device d owns the band of rows [H*d/D, H*(d+1)/D) and renders every
// sample pass over its band plus a one-row halo on each side (the halo rows' samples are
// recomputed, bit for bit: each pixel's generators depend only on the seed and the pixel, §7),
// resolves its band, and one RCCL group of send / receive pairs lands the bands in d_frame on
// the first device.  Halo launches carry no counters, so the ray counts are one frame's.
// Caller holds s->multi_mu.
void render_multi_msaa(rt_scene* s, CtxSet& cx, int cam, float* d_frame, hipStream_t s0,
                       bool per_call) {
  const int D = (int)s->rep.size();
  const rt_camera& c = s->host.cameras[cam];
  const int H = c.height, W = c.width, n = c.num_samples;
  const size_t frame = (size_t)W * H * 3;
  RenderCtx* x0 = cx.x[0];
  {
    DeviceGuard g(s->rep[0]->device);
    hip_check(hipEventRecord(x0->ev_in, s0), "event record");  // d_frame's earlier work
    hip_check(hipStreamWaitEvent(x0->stream, x0->ev_in, 0), "wait event");
  }
  for (int d = 0; d < D; d++) {
    const int lo = (int)((long long)H * d / D), hi = (int)((long long)H * (d + 1) / D);
    if (hi <= lo) continue;
    Replica& r = *s->rep[d];
    RenderCtx* x = cx.x[d];
    DeviceGuard g(r.device);
    float* dst = d_frame;
    // copy gather: the previous frame's band copy out of d_image (on the first device's
    // stream) has finished before this frame renders into it
    if (d > 0 && s->copy_gather) hip_check(hipStreamWaitEvent(x->stream, x0->ev_gathered, 0), "wait event");
    if (d > 0) {
      ensure(x->d_image, x->image_floats, frame, "alloc band frame");
      dst = x->d_image;
    }
    RenderParams P = make_params(s, r, cam, lo, 1, 0, 1, 0, dst, per_call ? x->d_cnt : r.d_counters);
    limit_rows(P, hi - lo);
    bind_ctx(s, x, P, c);
    enqueue_samples(s, r, P, n, x->d_samples, x->stream, d == 0);
    for (const int row : {lo - 1, hi}) {  // the halo rows the splat of the band's edges reads
      if (row < 0 || row >= H) continue;
      RenderParams Q = make_params(s, r, cam, row, 1, 0, 1, 0, dst, nullptr);
      limit_rows(Q, 1);
      Q.hits = P.hits;
      Q.occ = P.occ;
      Q.frames = P.frames;
      set_schedule(Q, x->d_sched);
      enqueue_samples(s, r, Q, n, x->d_samples, x->stream, false);
    }
    enqueue_resolve(s, W, H, n, x->d_samples, dst, lo, hi, x->stream);
  }
  DeviceGuard g(s->rep[0]->device);
  if (D > 1) {
    auto band = [&](int d, float* base) {
      const int lo = (int)((long long)H * d / D), hi = (int)((long long)H * (d + 1) / D);
      return std::make_pair(base + (size_t)lo * W * 3, (size_t)(hi - lo) * W * 3);
    };
    if (s->copy_gather) {
      for (int d = 1; d < D; d++) {
        const auto src = band(d, cx.x[d]->d_image);
        if (!src.second) continue;
        {
          DeviceGuard gd(s->rep[d]->device);
          hip_check(hipEventRecord(cx.x[d]->ev_out, cx.x[d]->stream), "event record");
        }
        hip_check(hipStreamWaitEvent(x0->stream, cx.x[d]->ev_out, 0), "wait event");
        hip_check(hipMemcpyPeerAsync(band(d, d_frame).first, s->rep[0]->device, src.first,
                                     s->rep[d]->device, src.second * sizeof(float), x0->stream),
                  "gather copy");
      }
      hip_check(hipEventRecord(x0->ev_gathered, x0->stream), "event record");
    } else {
      nccl_check(ncclGroupStart(), "ncclGroupStart");
      for (int d = 1; d < D; d++) {
        const auto src = band(d, cx.x[d]->d_image);
        if (!src.second) continue;
        nccl_check(ncclSend(src.first, src.second, ncclFloat, 0, s->comms[d], cx.x[d]->stream),
                   "ncclSend");
        nccl_check(ncclRecv(band(d, d_frame).first, src.second, ncclFloat, d, s->comms[0],
                            x0->stream),
                   "ncclRecv");
      }
      nccl_check(ncclGroupEnd(), "ncclGroupEnd");
    }
  }
  if (s0 != x0->stream) {
    hip_check(hipEventRecord(x0->ev_out, x0->stream), "event record");
    hip_check(hipStreamWaitEvent(s0, x0->ev_out, 0), "wait event");
  }
}

// One frame (rows row0 + k*row_stride) of a pixel-centre camera over every device of a
// multi-device scene, into the row-major frame d_frame on the first device, ordered on its
// stream s0.  The frame's 2x2-tile blocks are dealt round-robin over the D devices in deal
// order (the reference's row interleave over threads, HW2/main.cpp:33-36, at block
// granularity; block d -> device d mod D, deal_block_tile); each device renders its blocks
// tile-major into a slot of 4 ceil(B / D) tiles on its context's stream — as 32-bit pixel
// records where records_ok (a third of RGB's bytes), else RGB; one RCCL group of send / receive
// pairs (single process, one communicator per device) gathers the slots onto the first device,
// whose resolve kernel shades the records into the rows (or untile kernel copies the RGB).
// Counters: `per_call` adds each device's rays to its context's counters (rt_render's stats),
// else to the replica's (rt_collect_stats).  Caller holds s->multi_mu.
void render_multi(rt_scene* s, CtxSet& cx, int cam, int row0, int row_stride, float* d_frame,
                  hipStream_t s0, bool per_call) {
  const int D = (int)s->rep.size();
  const rt_camera& c = s->host.cameras[cam];
  const TilePlan tp = plan(c, row0, row_stride);
  if (tp.tiles_total == 0) return;
  const int blocks = deal_blocks(tp.tiles_x, tp.tiles_total / tp.tiles_x);
  const int slot = 4 * ((blocks + D - 1) / D);  // tiles: whole 2x2 blocks (block deal)
  // the other devices' shares travel as 32-bit pixel records where the scene allows, else as RGB
  const bool records = records_ok(s, cam);
  const size_t tile_words = records ? (size_t)kTile * kTile : (size_t)kTileFloats;
  RenderCtx* x0 = cx.x[0];
  {
    DeviceGuard g(s->rep[0]->device);
    hip_check(hipEventRecord(x0->ev_in, s0), "event record");  // d_frame's earlier work
    // the first device renders its own blocks in place into d_frame (after d_frame's earlier
    // work); the others render tile-major into their slots for the gather
    hip_check(hipStreamWaitEvent(x0->stream, x0->ev_in, 0), "wait event");
  }
  for (int d = 0; d < D; d++) {
    Replica& r = *s->rep[d];
    RenderCtx* x = cx.x[d];
    DeviceGuard g(r.device);
    // copy gather: the previous frame's peer copy out of d_out (on the first device's stream)
    // has finished before this frame renders into it
    if (d > 0 && s->copy_gather) hip_check(hipStreamWaitEvent(x->stream, x0->ev_gathered, 0), "wait event");
    if (d > 0) ensure(x->d_out, x->out_floats, (size_t)slot * tile_words, "alloc tile slot");
    RenderParams P = make_params(s, r, cam, row0, row_stride, d, D,
                                 d == 0 ? RT_TILE_BLOCKS
                                        : RT_TILE_MAJOR | RT_TILE_BLOCKS | (records ? RT_TILE_RECORDS : 0),
                                 d == 0 ? d_frame : x->d_out, per_call ? x->d_cnt : r.d_counters);
    bind_ctx(s, x, P, c);
    enqueue_frame(s, r, P, 1, nullptr, x->stream, d == 0);
  }
  DeviceGuard g(s->rep[0]->device);
  ensure(x0->d_recv, x0->recv_floats, (size_t)D * slot * tile_words, "alloc gathered slots");
  const size_t count = (size_t)slot * tile_words;  // 4-B words (floats or pixel records)
  if (D == 1) {
    // nothing to gather: the one device rendered the frame in place
  } else if (s->copy_gather) {
    for (int d = 1; d < D; d++) {
      {
        DeviceGuard gd(s->rep[d]->device);
        hip_check(hipEventRecord(cx.x[d]->ev_out, cx.x[d]->stream), "event record");
      }
      hip_check(hipStreamWaitEvent(x0->stream, cx.x[d]->ev_out, 0), "wait event");
      hip_check(hipMemcpyPeerAsync(x0->d_recv + (size_t)d * count, s->rep[0]->device,
                                   cx.x[d]->d_out, s->rep[d]->device, count * sizeof(float),
                                   x0->stream),
                "gather copy");
    }
    hip_check(hipEventRecord(x0->ev_gathered, x0->stream), "event record");
  } else {
    nccl_check(ncclGroupStart(), "ncclGroupStart");
    for (int d = 1; d < D; d++)
      nccl_check(ncclSend(cx.x[d]->d_out, count, ncclFloat, 0, s->comms[d], cx.x[d]->stream),
                 "ncclSend");
    for (int d = 1; d < D; d++)
      nccl_check(ncclRecv(x0->d_recv + (size_t)d * count, count, ncclFloat, d, s->comms[0],
                          x0->stream),
                 "ncclRecv");
    nccl_check(ncclGroupEnd(), "ncclGroupEnd");
  }
  UntileParams U;
  U.recv = x0->d_recv;
  U.out = d_frame;
  U.width = c.width;
  U.row0 = row0;
  U.row_stride = row_stride;
  U.rows = tp.rows;
  U.tiles_x = tp.tiles_x;
  U.tiles_total = tp.tiles_total;
  U.devices = D;
  U.slot = slot;
  U.tile_offset = 0;
  U.blocks = 1;
  U.skip_root = 1;  // the first device's blocks are already in d_frame
  U.vec = untile_vec(U);
  if (D > 1 && records) {  // the others' pixel records shaded into the frame
    const RenderParams P0 = make_params(s, *s->rep[0], cam, row0, row_stride, 0, 1, 0, d_frame,
                                        nullptr);
    U.vec = 0;
    hip_check(launch_resolve(P0, U, s->has_spheres, x0->stream), "resolve launch");
  } else if (D > 1) {
    hip_check(launch_untile(U, x0->stream), "untile launch");
  }
  if (s0 != x0->stream) {
    hip_check(hipEventRecord(x0->ev_out, x0->stream), "event record");
    hip_check(hipStreamWaitEvent(s0, x0->ev_out, 0), "wait event");
  }
}

// Frees the least recently used scratch no host thread is enqueueing on (its mutex is free:
// holders of a scratch pointer keep it locked, and new ones need r.mu), after the GPU work of
// its last frame.  Caller holds r.mu.
void evict_scratch(Replica& r) {
  size_t victim = r.streams.size();
  for (size_t k = 0; k < r.streams.size(); k++) {
    if (!r.streams[k]->mu.try_lock()) continue;
    r.streams[k]->mu.unlock();
    if (victim == r.streams.size() || r.streams[k]->used < r.streams[victim]->used) victim = k;
  }
  if (victim == r.streams.size()) return;  // every one in use: let the table grow
  StreamScratch& x = *r.streams[victim];
  if (x.done) hip_check(hipEventSynchronize(x.done), "synchronize evicted scratch");
  free_scratch(x);
  r.streams.erase(r.streams.begin() + (long)victim);
}

// The scratch of `stream` on replica r, returned with its mutex held in `held`: allocated on
// first use at the largest camera's size; beyond kMaxStreamTables streams the least recently
// used one is evicted.
StreamScratch* scratch_for(rt_scene* s, Replica& r, void* stream, std::unique_lock<std::mutex>& held) {
  std::lock_guard<std::mutex> lk(r.mu);
  for (auto& x : r.streams)
    if (x->stream == stream) {
      held = std::unique_lock<std::mutex>(x->mu);
      x->used = ++r.tick;
      return x.get();
    }
  if (r.streams.size() >= kMaxStreamTables) evict_scratch(r);
  auto x = std::make_unique<StreamScratch>();
  x->stream = stream;
  x->used = ++r.tick;
  const size_t most = s->most;
  try {
    hip_check(hipEventCreateWithFlags(&x->done, hipEventDisableTiming), "event");
    hip_check(hipMalloc(&x->hits, most * sizeof(int2_t)), "alloc hit records");
    hip_check(hipMalloc(&x->occ, most * sizeof(unsigned) * occ_words(s->host)),
              "alloc occlusion bits");
    hip_check(hipMalloc(&x->sched, sched_words_for(most / (kTile * kTile)) * sizeof(unsigned)),
              "alloc tile schedule");
  } catch (...) {
    free_scratch(*x);
    throw;
  }
  r.streams.push_back(std::move(x));
  held = std::unique_lock<std::mutex>(r.streams.back()->mu);
  return r.streams.back().get();
}

int load_xml_into(rt_scene* s, const char* xml_path, const std::vector<int>* devices,
                  int device_count, const int* device_ids) {
  return guarded([&] {
    XmlSceneStorage st;
    rt_scene_desc d;
    load_scene_xml(xml_path, st, d);
    s->host.image_names = st.image_names;
    build_host_scene(d, s->host);
    std::vector<int> devs;
    if (devices) {
      devs = *devices;
    } else {
      devs = device_list(device_count, device_ids);
    }
    return create_from_host(s, devs, devices == nullptr);
  });
}

std::vector<int> single_device(int device) {
  if (device < 0) hip_check(hipGetDevice(&device), "hipGetDevice");
  return {device};
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

int rt_scene_create_multi(const rt_scene_desc* desc, int device_count, const int* devices,
                          rt_scene** out) {
  if (!desc || !out) return set_error(RT_E_INVALID, "rt_scene_create: NULL argument");
  *out = nullptr;
  auto s = std::make_unique<rt_scene>();
  const int rc = guarded([&] {
    const std::vector<int> devs = device_list(device_count, devices);
    build_host_scene(*desc, s->host);
    return create_from_host(s.get(), devs, true);
  });
  if (rc != RT_OK) {
    free_device(s.get());
    return rc;
  }
  *out = s.release();
  return RT_OK;
}

int rt_scene_create(const rt_scene_desc* desc, int device, rt_scene** out) {
  if (!desc || !out) return set_error(RT_E_INVALID, "rt_scene_create: NULL argument");
  *out = nullptr;
  auto s = std::make_unique<rt_scene>();
  const int rc = guarded([&] {
    const std::vector<int> devs = single_device(device);
    build_host_scene(*desc, s->host);
    return create_from_host(s.get(), devs, false);
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
  std::vector<int> devs;
  int rc = guarded([&] {
    devs = single_device(device);
    return RT_OK;
  });
  if (rc == RT_OK) rc = load_xml_into(s.get(), xml_path, &devs, 0, nullptr);
  if (rc != RT_OK) {
    free_device(s.get());
    return rc;
  }
  *out = s.release();
  return RT_OK;
}

int rt_scene_load_xml_multi(const char* xml_path, int device_count, const int* devices,
                            rt_scene** out) {
  if (!xml_path || !out) return set_error(RT_E_INVALID, "rt_scene_load_xml_multi: NULL argument");
  *out = nullptr;
  auto s = std::make_unique<rt_scene>();
  const int rc = load_xml_into(s.get(), xml_path, nullptr, device_count, devices);
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
int rt_scene_device_count(const rt_scene* s) { return s ? (int)s->rep.size() : 0; }

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

int rt_host_dump_bvh_desc(const rt_scene_desc* desc, const char* out_path) {
  if (!desc || !out_path) return set_error(RT_E_INVALID, "rt_host_dump_bvh_desc: NULL argument");
  return guarded([&] {
    HostScene h;
    build_host_scene(*desc, h);
    FILE* f = std::fopen(out_path, "w");
    if (!f) throw std::ios_base::failure(std::string("cannot open ") + out_path);
    const std::string text = dump_bvh(h);
    std::fwrite(text.data(), 1, text.size(), f);
    std::fclose(f);
    return RT_OK;
  });
}

void* rt_host_alloc(size_t bytes) {
  void* p = nullptr;
  const int rc = guarded([&] {
    hip_check(hipHostMalloc(&p, std::max<size_t>(bytes, 1), hipHostMallocDefault),
              "rt_host_alloc");
    return RT_OK;
  });
  return rc == RT_OK ? p : nullptr;
}

void rt_host_free(void* p) {
  if (p) (void)hipHostFree(p);
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
  if (!s || (mode != RT_TRAVERSAL_FAST && mode != RT_TRAVERSAL_REFERENCE))
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

int rt_render_device_range(rt_scene* s, int cam, int row0, int row_stride, int tile_begin,
                           int tile_step, int tile_count, int tile_major, float* d_out,
                           void* stream) {
  return guarded([&] {
    check_render_args(s, cam, row0, row_stride);
    if (tile_begin < 0 || tile_step < 1 || !d_out ||
        (tile_major & ~(RT_TILE_MAJOR | RT_TILE_BLOCKS | RT_TILE_RECORDS)))
      throw std::invalid_argument("rt_render_device: bad tile selection / output");
    if ((tile_major & RT_TILE_RECORDS) && !records_ok(s, cam))
      throw std::domain_error("rt_render_device: pixel records need a pixel-centre camera, no "
                              "mirror/dielectric recursion and at most 4 lights");
    const rt_camera& c = s->host.cameras[cam];
    if (s->multi) {
      // a multi-device scene renders whole frames (rows subsets allowed) split over its devices
      if (tile_begin != 0 || tile_step != 1 || tile_major || tile_count >= 0)
        throw std::domain_error("multi-device scenes render whole row-major frames only");
      std::lock_guard<std::mutex> lk(s->multi_mu);
      CtxSet cx(s, s->rep.size(), stream);
      if (c.num_samples > 1)
        render_multi_msaa(s, cx, cam, d_out, (hipStream_t)stream, false);
      else
        render_multi(s, cx, cam, row0, row_stride, d_out, (hipStream_t)stream, false);
      return RT_OK;
    }
    Replica& r = *s->rep[0];
    DeviceGuard g(r.device);
    std::unique_lock<std::mutex> lk;
    StreamScratch* sc = scratch_for(s, r, stream, lk);
    RenderParams P = make_params(s, r, cam, row0, row_stride, tile_begin, tile_step, tile_major,
                                 d_out, r.d_counters);
    P.hits = sc->hits;
    P.occ = sc->occ;
    set_schedule(P, sc->sched);
    const int unit_tiles = P.block_deal ? 4 : 1;  // tile_count counts deal units
    if (tile_count >= 0 && (long long)tile_count * unit_tiles < P.num_sel_tiles) {
      if (c.num_samples > 1) throw std::domain_error("NumSamples > 1 renders whole row-major frames only");
      P.num_sel_tiles = tile_count * unit_tiles;
    }
    if (s->needs_recursion) {
      ensure(sc->frames, sc->frames_capacity, frame_floats(s->host, P.num_sel_tiles),
             "alloc ray-tree frames");
      P.frames = sc->frames;
    }
    if (c.num_samples > 1) {
      if (tile_begin != 0 || tile_step != 1 || tile_major)
        throw std::domain_error("NumSamples > 1 renders whole row-major frames only");
      ensure(sc->samples, sc->samples_capacity, sample_floats(c), "alloc MSAA samples");
    }
    // warm order: a frame of the same selection as the stream's previous one
    // dispatches its primary kernel heaviest-first by that frame's measured tile costs
    const std::array<long long, 7> key{cam, row0, row_stride, tile_begin, tile_step,
                                       P.num_sel_tiles, P.block_deal};
    const bool orderable = c.num_samples <= 1 && !P.frames && P.num_lights > 0;
    P.primary_order = orderable && sc->order_valid && sc->order_key == key ? 1 : 0;
    enqueue_frame(s, r, P, c.num_samples, sc->samples, (hipStream_t)stream, true);
    hip_check(hipEventRecord(sc->done, (hipStream_t)stream), "event record");
    sc->order_key = key;
    sc->order_valid = orderable;
    return RT_OK;
  });
}

int rt_untile_device(rt_scene* s, int cam, int row0, int row_stride, int devices, int slot,
                     int tile_offset, int flags, const float* d_gathered, float* d_out,
                     void* stream) {
  return guarded([&] {
    check_render_args(s, cam, row0, row_stride);
    if (devices < 1 || slot < 0 || tile_offset < 0 || !d_gathered || !d_out ||
        (flags & ~(RT_UNTILE_BLOCKS | RT_UNTILE_SKIP_ROOT)) ||
        ((flags & RT_UNTILE_BLOCKS) && slot % 4))
      throw std::invalid_argument("rt_untile_device: bad argument");
    const rt_camera& c = s->host.cameras[cam];
    const TilePlan tp = plan(c, row0, row_stride);
    const int blocks = (flags & RT_UNTILE_BLOCKS) ? 1 : 0;
    const long long units = blocks ? deal_blocks(tp.tiles_x, tp.tiles_total / tp.tiles_x) : tp.tiles_total;
    if ((long long)devices * (blocks ? slot / 4 : slot) < units)
      throw std::invalid_argument("rt_untile_device: devices * slot is smaller than the frame's share");
    DeviceGuard g(s->rep[0]->device);
    UntileParams U;
    U.recv = d_gathered;
    U.out = d_out;
    U.width = c.width;
    U.row0 = row0;
    U.row_stride = row_stride;
    U.rows = tp.rows;
    U.tiles_x = tp.tiles_x;
    U.tiles_total = tp.tiles_total;
    U.devices = devices;
    U.slot = slot;
    U.tile_offset = tile_offset % devices;
    U.blocks = blocks;
    U.skip_root = (flags & RT_UNTILE_SKIP_ROOT) ? 1 : 0;
    U.vec = untile_vec(U);
    hip_check(launch_untile(U, (hipStream_t)stream), "untile launch");
    return RT_OK;
  });
}

int rt_tile_costs(rt_scene* s, void* stream, unsigned* host_out, int capacity) {
  if (!s || !host_out || capacity < 0) return set_error(RT_E_INVALID, "rt_tile_costs: bad argument");
  return guarded([&]() -> int {
    if (s->multi) throw std::domain_error("rt_tile_costs: single-device scenes only");
    Replica& r = *s->rep[0];
    DeviceGuard g(r.device);
    StreamScratch* x = nullptr;
    std::unique_lock<std::mutex> held;
    {
      std::lock_guard<std::mutex> lk(r.mu);
      for (auto& p : r.streams)
        if (p->stream == stream) x = p.get();
      if (x) held = std::unique_lock<std::mutex>(x->mu);
    }
    if (!x || !x->order_valid)
      throw std::domain_error("rt_tile_costs: no ordered frame was rendered on this stream");
    const long long n = x->order_key[5];  // the last selection's tiles
    if (n > capacity) throw std::invalid_argument("rt_tile_costs: capacity below the frame's tiles");
    hip_check(hipStreamSynchronize((hipStream_t)stream), "synchronize stream");
    hip_check(hipMemcpy(host_out, x->sched + sched_snap_offset((unsigned long long)n),
                        (size_t)n * sizeof(unsigned), hipMemcpyDeviceToHost),
              "read tile costs");
    return (int)n;
  });
}

int rt_scene_records_ok(const rt_scene* s, int cam) {
  if (!s || cam < 0 || cam >= (int)s->host.cameras.size())
    return set_error(RT_E_INVALID, "rt_scene_records_ok: bad argument");
  return records_ok(s, cam) ? 1 : 0;
}

int rt_resolve_device(rt_scene* s, int cam, int row0, int row_stride, int devices, int slot,
                      int tile_offset, int flags, const unsigned* d_gathered, float* d_out,
                      void* stream) {
  return guarded([&] {
    check_render_args(s, cam, row0, row_stride);
    if (devices < 1 || slot < 0 || tile_offset < 0 || !d_gathered || !d_out ||
        (flags & ~(RT_UNTILE_BLOCKS | RT_UNTILE_SKIP_ROOT)) ||
        ((flags & RT_UNTILE_BLOCKS) && slot % 4))
      throw std::invalid_argument("rt_resolve_device: bad argument");
    if (!records_ok(s, cam)) throw std::domain_error("rt_resolve_device: no pixel records here");
    const rt_camera& c = s->host.cameras[cam];
    const TilePlan tp = plan(c, row0, row_stride);
    const int blocks = (flags & RT_UNTILE_BLOCKS) ? 1 : 0;
    const long long units = blocks ? deal_blocks(tp.tiles_x, tp.tiles_total / tp.tiles_x) : tp.tiles_total;
    if ((long long)devices * (blocks ? slot / 4 : slot) < units)
      throw std::invalid_argument("rt_resolve_device: devices * slot is smaller than the frame's share");
    Replica& r = *s->rep[0];
    DeviceGuard g(r.device);
    const RenderParams P = make_params(s, r, cam, row0, row_stride, 0, 1, 0, d_out, nullptr);
    UntileParams U;
    U.recv = reinterpret_cast<const float*>(d_gathered);
    U.out = d_out;
    U.width = c.width;
    U.row0 = row0;
    U.row_stride = row_stride;
    U.rows = tp.rows;
    U.tiles_x = tp.tiles_x;
    U.tiles_total = tp.tiles_total;
    U.devices = devices;
    U.slot = slot;
    U.tile_offset = tile_offset % devices;
    U.blocks = blocks;
    U.skip_root = (flags & RT_UNTILE_SKIP_ROOT) ? 1 : 0;
    U.vec = 0;
    hip_check(launch_resolve(P, U, s->has_spheres, (hipStream_t)stream), "resolve launch");
    return RT_OK;
  });
}

int rt_resolve_rows(rt_scene* s, int cam, int row_begin, int row_end, const unsigned* d_records,
                    float* d_out, void* stream) {
  return guarded([&] {
    check_render_args(s, cam, 0, 1);
    const rt_camera& c = s->host.cameras[cam];
    if (row_begin < 0 || row_end < row_begin || row_end > c.height || !d_records || !d_out)
      throw std::invalid_argument("rt_resolve_rows: bad argument");
    if (s->multi) throw std::domain_error("rt_resolve_rows: single-device scenes only");
    if (!records_ok(s, cam)) throw std::domain_error("rt_resolve_rows: no pixel records here");
    Replica& r = *s->rep[0];
    DeviceGuard g(r.device);
    const RenderParams P = make_params(s, r, cam, 0, 1, 0, 1, 0, d_out, nullptr);
    hip_check(launch_resolve_rows(P, d_records, row_begin, row_end, s->has_spheres,
                                  (hipStream_t)stream), "resolve launch");
    return RT_OK;
  });
}

int rt_release_stream_scratch(rt_scene* s, void* stream) {
  if (!s) return set_error(RT_E_INVALID, "rt_release_stream_scratch: NULL scene");
  return guarded([&] {
    for (auto& rp : s->rep) {
      Replica& r = *rp;
      std::unique_ptr<StreamScratch> x;
      RenderCtx* sc = nullptr;
      {
        std::lock_guard<std::mutex> lk(r.mu);
        for (size_t k = 0; k < r.streams.size(); k++)
          if (r.streams[k]->stream == stream) {
            x = std::move(r.streams[k]);
            r.streams.erase(r.streams.begin() + (long)k);
            break;
          }
        for (size_t k = 0; k < r.stream_ctx.size(); k++)
          if (r.stream_ctx[k].first == stream) {
            sc = r.stream_ctx[k].second;
            r.stream_ctx.erase(r.stream_ctx.begin() + (long)k);
            break;
          }
      }
      if (sc) {  // a multi-device scene's context of that caller stream: back to the pool
        DeviceGuard g(r.device);
        hip_check(hipStreamSynchronize(sc->stream), "synchronize context stream");
        release_ctx(r, sc);
      }
      if (!x) continue;
      DeviceGuard g(r.device);
      std::lock_guard<std::mutex> lk(x->mu);  // no enqueue on it is in progress
      hip_check(hipStreamSynchronize((hipStream_t)stream), "synchronize stream");
      free_scratch(*x);
    }
    return RT_OK;
  });
}

int rt_collect_stats(rt_scene* s, rt_stats* stats) {
  if (!s || !stats) return set_error(RT_E_INVALID, "rt_collect_stats: NULL argument");
  return guarded([&] {
    std::memset(stats, 0, sizeof *stats);
    for (auto& rp : s->rep) {
      DeviceGuard g(rp->device);
      std::vector<unsigned long long> c(kCounterWidth * kCounterRows);
      hip_check(hipMemcpy(c.data(), rp->d_counters, c.size() * sizeof c[0], hipMemcpyDeviceToHost),
                "read counters");
      hip_check(hipMemset(rp->d_counters, 0, c.size() * sizeof c[0]), "reset counters");
      add_counters(c, stats);
    }
    return RT_OK;
  });
}

int rt_debug_counters(rt_scene* s, long long* out16) {
  if (!s || !out16) return set_error(RT_E_INVALID, "rt_debug_counters: NULL argument");
  return guarded([&] {
    for (int k = 0; k < kCounterWidth; k++) out16[k] = 0;
    for (auto& rp : s->rep) {
      DeviceGuard g(rp->device);
      std::vector<unsigned long long> c(kCounterWidth * kCounterRows);
      hip_check(hipMemcpy(c.data(), rp->d_counters, c.size() * sizeof c[0], hipMemcpyDeviceToHost),
                "read counters");
      hip_check(hipMemset(rp->d_counters, 0, c.size() * sizeof c[0]), "reset counters");
      for (int k = 0; k < kCounterWidth; k++) {
        unsigned long long sum = 0;
        for (int r = 0; r < kCounterRows; r++) sum += c[kCounterWidth * r + k];
        out16[k] += (long long)sum;
      }
    }
    out16[kCntExactBox] = (long long)read_reset_exact_fallbacks();
    return diag_build() ? 1 : 0;
  });
}

long long rt_debug_phases(unsigned long long* out, long long max_values) {
  if (!out || max_values < 0) return set_error(RT_E_INVALID, "rt_debug_phases: bad argument");
  const long long n = read_reset_phases(out, max_values);
  if (n < 0) return set_error(RT_E_INVALID, "rt_debug_phases: buffer too small or copy failed");
  return n;
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
    const rt_camera& c = s->host.cameras[cam];
    const TilePlan tp = plan(c, row0, row_stride);
    if (tp.rows == 0) return RT_OK;
    const bool multi = s->multi;
    std::unique_lock<std::mutex> multi_lock(s->multi_mu, std::defer_lock);
    if (multi) multi_lock.lock();
    CtxSet cx(s, multi ? s->rep.size() : 1);
    Replica& r = *s->rep[0];
    RenderCtx* x = cx.x[0];
    DeviceGuard g(r.device);
    const size_t frame = (size_t)c.width * c.height * 3;
    float* d_frame = nullptr;
    if (multi) {  // (d_out holds the first device's tile slot)
      ensure(x->d_image, x->image_floats, frame, "alloc frame");
      d_frame = x->d_image;
    } else {
      ensure(x->d_out, x->out_floats, frame, "alloc frame");
      d_frame = x->d_out;
    }
    // Counters are per scene; this call reports its own deltas via the contexts' buffers.
    for (size_t d = 0; d < cx.x.size(); d++) {
      DeviceGuard gd(s->rep[d]->device);
      hip_check(hipMemsetAsync(cx.x[d]->d_cnt, 0,
                               sizeof(unsigned long long) * kCounterWidth * kCounterRows,
                               cx.x[d]->stream),
                "zero counters");
    }
    hip_check(hipEventRecord(x->e0, x->stream), "event record");
    // rows j = row0 + k*row_stride only: strided 2D copies leave the others untouched
    const size_t row_bytes = (size_t)c.width * 3 * sizeof(float);
    auto copy_rows = [&](int lr0, int lr1, hipStream_t st) {  // logical rows [lr0, lr1)
      if (lr1 <= lr0) return;
      const size_t off = (size_t)(row0 + (size_t)lr0 * row_stride) * c.width * 3;
      hip_check(hipMemcpy2DAsync(out_rgb + off, row_bytes * row_stride, d_frame + off,
                                 row_bytes * row_stride, row_bytes, (size_t)(lr1 - lr0),
                                 hipMemcpyDeviceToHost, st),
                "copy rows");
    };
    const int tiles_y = tp.tiles_total / tp.tiles_x;
    const int chunks = std::min(kRenderChunks, tiles_y);
    // a caller buffer in pinned host memory (hipHostMalloc / registered, e.g. torch pin_memory)
    // is written by the frame kernel itself, through its device-visible address: no copy
    float* direct = nullptr;
    if (!multi && c.num_samples <= 1 && RT_DIRECT_PINNED) {
      void* dp = nullptr;
      if (hipHostGetDevicePointer(&dp, out_rgb, 0) == hipSuccess && dp)
        direct = static_cast<float*>(dp);
      else
        (void)hipGetLastError();  // pageable memory: not an error here
    }
    if (direct) {
      RenderParams P = make_params(s, r, cam, row0, row_stride, 0, 1, 0, direct, x->d_cnt);
      bind_ctx(s, x, P, c);
      // block order: the frame is bound by its writes over PCIe, which the heavy-first (cold)
      // order scatters (0.674 -> 0.742 ms per C3 frame, profiles/r06/ab_dropin_cold.jsonl)
      P.tile_cost = nullptr;
#ifndef RT_PAIR_ROWS  // (A/B builds: 0 = each wave writes its own tile)
#define RT_PAIR_ROWS 1
#endif
      P.pair_rows = RT_PAIR_ROWS;
      enqueue_frame(s, r, P, c.num_samples, x->d_samples, x->stream, true);
      hip_check(hipEventRecord(x->e1, x->stream), "event record");
    } else if (!multi && c.num_samples <= 1 && chunks > 1) {
      // the drop-in seam: the frame as `chunks` bands of tile rows, one
      // launch each on the context's stream; each band goes to the caller's buffer on the copy
      // stream as soon as its launch is done, while the next bands render
      if (!x->copy_stream)
        hip_check(hipStreamCreateWithFlags(&x->copy_stream, hipStreamNonBlocking), "copy stream");
      for (int k = 0; k < chunks; k++) {
        const int ty0 = (int)((long long)tiles_y * k / chunks);
        const int ty1 = (int)((long long)tiles_y * (k + 1) / chunks);
        RenderParams P = make_params(s, r, cam, row0, row_stride, ty0 * tp.tiles_x, 1, 0, d_frame,
                                     x->d_cnt);
        P.num_sel_tiles = (ty1 - ty0) * tp.tiles_x;
        bind_ctx(s, x, P, c);
        P.tile_cost = nullptr;  // no dispatch order for a next frame (nothing reuses it here)
        enqueue_frame(s, r, P, c.num_samples, x->d_samples, x->stream, true);
        if (!x->ev_chunk[k])
          hip_check(hipEventCreateWithFlags(&x->ev_chunk[k], hipEventDisableTiming), "event");
        hip_check(hipEventRecord(x->ev_chunk[k], x->stream), "event record");
      }
      hip_check(hipEventRecord(x->e1, x->stream), "event record");
      for (int k = 0; k < chunks; k++) {
        const int ty0 = (int)((long long)tiles_y * k / chunks);
        const int ty1 = (int)((long long)tiles_y * (k + 1) / chunks);
        hip_check(hipStreamWaitEvent(x->copy_stream, x->ev_chunk[k], 0), "wait band");
        copy_rows(kTile * ty0, std::min(tp.rows, kTile * ty1), x->copy_stream);
      }
      hip_check(hipStreamSynchronize(x->copy_stream), "synchronize copies");
    } else {
      if (multi && c.num_samples > 1) {
        render_multi_msaa(s, cx, cam, d_frame, x->stream, true);
      } else if (multi) {
        render_multi(s, cx, cam, row0, row_stride, d_frame, x->stream, true);
      } else {
        RenderParams P = make_params(s, r, cam, row0, row_stride, 0, 1, 0, d_frame, x->d_cnt);
        bind_ctx(s, x, P, c);
        enqueue_frame(s, r, P, c.num_samples, x->d_samples, x->stream, true);
      }
      hip_check(hipEventRecord(x->e1, x->stream), "event record");
      copy_rows(0, tp.rows, x->stream);
    }
    std::vector<std::vector<unsigned long long>> cnt(cx.x.size(),
                                                     std::vector<unsigned long long>(kCounterAlloc));
    for (size_t d = 0; d < cx.x.size(); d++) {
      DeviceGuard gd(s->rep[d]->device);
      hip_check(hipMemcpyAsync(cnt[d].data(), cx.x[d]->d_cnt, kCounterAlloc * sizeof(unsigned long long),
                               hipMemcpyDeviceToHost, cx.x[d]->stream),
                "copy counters");
    }
    for (size_t d = 0; d < cx.x.size(); d++) {
      DeviceGuard gd(s->rep[d]->device);
      hip_check(hipStreamSynchronize(cx.x[d]->stream), "synchronize");
    }
    if (stats) {
      std::memset(stats, 0, sizeof *stats);
      for (auto& v : cnt) add_counters(v, stats);
      float ms = 0;
      hip_check(hipEventElapsedTime(&ms, x->e0, x->e1), "elapsed");
      stats->kernel_ms = ms;
    }
    return RT_OK;
  });
}

int rt_set_kernel_timing(rt_scene* s, int enable) {
  if (!s) return set_error(RT_E_INVALID, "rt_set_kernel_timing: NULL scene");
  std::lock_guard<std::mutex> lk(s->timing_mu);
  s->timing.on = enable != 0;
  return RT_OK;
}

int rt_read_kernel_times(rt_scene* s, double* ms4, long long* launches) {
  if (!s || !ms4) return set_error(RT_E_INVALID, "rt_read_kernel_times: NULL argument");
  return guarded([&] {
    DeviceGuard g(s->rep[0]->device);
    std::vector<std::array<hipEvent_t, 4>> done;
    double sum[4];
    long long n;
    {
      std::lock_guard<std::mutex> lk(s->timing_mu);
      done.swap(s->timing.pending);
      std::memcpy(sum, s->timing.sum, sizeof sum);
      n = s->timing.folded;
      std::memset(s->timing.sum, 0, sizeof s->timing.sum);
      s->timing.folded = 0;
    }
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
    if (launches) *launches = n + (long long)done.size();
    std::lock_guard<std::mutex> lk(s->timing_mu);
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
