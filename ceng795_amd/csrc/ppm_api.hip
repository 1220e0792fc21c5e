// C-ABI implementation of the photon-mapping path (include/ceng795_ppm.h): scene upload, the
// eye / grid / photon / density passes and their device buffers.  One HIP stream per scene.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <exception>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ceng795_ppm.h"
#include "ppm_host.h"
#include "ppm_internal.h"

namespace ppm {  // ppm_kernels.hip
hipError_t launch_eye(const PScene&, const PCamera&, unsigned long long, int*, const int*,
                      PHitPoint*, unsigned long long*, hipStream_t);
hipError_t launch_grid(const PHitPoint*, int, int, int, PGrid*, float4*, unsigned*, hipStream_t);
hipError_t launch_photons(const PScene&, unsigned long long, long long, int, int, PDeposit*, int*,
                          unsigned long long*, hipStream_t);
hipError_t launch_deposit_keys(const PDeposit*, const int*, const int*, int, int, const PGrid*,
                               unsigned*, PDeposit*, float4*, hipStream_t);
hipError_t launch_group_buckets(const PHitPoint*, const int*, const int*, int, const PGrid*,
                                unsigned*, int*, int*, hipStream_t);
hipError_t launch_bucket_group_pairs(const unsigned*, const int*, const int*, const int*, int,
                                     unsigned*, unsigned*, hipStream_t);
hipError_t launch_expand_count(const unsigned*, int, const int*, const int*, int*, hipStream_t);
hipError_t launch_expand_write(const unsigned*, int, const int*, const int*, const unsigned*,
                               const int*, unsigned*, unsigned*, hipStream_t);
hipError_t launch_bucket_bounds(const unsigned*, int, unsigned, int*, int*, hipStream_t);
hipError_t launch_group_keys(const PHitPoint*, int, const PGrid*, unsigned long long*, int*, int*,
                            hipStream_t);
hipError_t launch_group_flags(const unsigned long long*, int, int*, hipStream_t);
hipError_t launch_group_starts(const int*, const int*, int, int*, hipStream_t);
hipError_t launch_group_tiles(const int*, int, int*, hipStream_t);
hipError_t launch_tile_table(const int*, const int*, int, int2*, hipStream_t);
hipError_t launch_tile_work(const int2*, int, const int*, const int*, unsigned*, hipStream_t);
hipError_t launch_tile_shard(const int2*, int, int, int, const int*, const int*, int2*, int*,
                             hipStream_t);
hipError_t launch_merge_state(const int*, int, int, const float4*, const unsigned*, float4*,
                              unsigned*, hipStream_t);
hipError_t launch_rr_table(float*, int, hipStream_t);
hipError_t launch_materialize(const unsigned*, const unsigned*, int, const float4*, float4*,
                              hipStream_t);
hipError_t launch_group_update(const PScene&, const PHitPoint*, const int*, const int*,
                               const int2*, int, const int*, const int*, const float4*,
                               const PDeposit*, const float*, int, float4*, unsigned*,
                               const long long*, float4*, unsigned long long*, hipStream_t);
hipError_t launch_tile_compact_need(const int2*, int, const int*, const int*, long long, int, int,
                                    long long*, hipStream_t);
hipError_t launch_density(const PHitPoint*, const float4*, const int*, int, double, float*,
                          hipStream_t);
}  // namespace ppm
namespace rt {
void write_png(const std::string& path, const float* rgb, int w, int h);
}

using namespace ppm;

namespace {

thread_local std::string g_error;

struct HipFailure {
  hipError_t err;
  const char* what;
};
void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw HipFailure{e, what};
}
int set_error(int code, const std::string& msg) {
  g_error = msg;
  return code;
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
  } catch (const std::exception& e) {
    return set_error(RT_E_INVALID, e.what());
  }
}

template <typename T>
struct DevBuf {  // grow-only device array
  T* p = nullptr;
  size_t cap = 0;
  void reserve(size_t n, const char* what) {
    if (n <= cap) return;
    (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hip_check(hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)), what);
    cap = n;
  }
  void release() {
    (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

template <typename T>
T* upload(const std::vector<T>& v, const char* what) {
  T* p = nullptr;
  hip_check(hipMalloc(&p, std::max<size_t>(v.size() * sizeof(T), 16)), what);
  if (!v.empty()) hip_check(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice), what);
  return p;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) hip_check(hipSetDevice(dev), "hipSetDevice");
  }
  ~DeviceGuard() {
    int cur;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// Deposit slot rows per photon batch.  Default 16 GiB: C5's 1e7 photons x 19 slots x 48 B
// (9.1 GB) run as one batch (one sort, one update launch).  The budget actually used is also
// capped at a quarter of the device memory free when the pass starts (plus what the scene's
// slots already hold), so a smaller or shared GPU falls back to more batches instead of failing
// in hipMalloc.  ppm_set_batching sets it per scene.
constexpr int kRRTable = 1 << 20;  // rr(n) tabulated for n < 2^20 (larger n computed inline)
struct WidenInt {
  __host__ __device__ long long operator()(int x) const { return (long long)x; }
};

size_t default_slot_bytes() { return size_t(16) << 30; }

}  // namespace

struct ppm_scene {
  HostPPM host;
  int device = 0;
  hipStream_t stream = nullptr;
  unsigned long long seed = 0;
  PScene S{};
  std::vector<void*> owned;  // scene arrays
  // eye pass / hash grid
  int eye_cam = -1;
  int n_hp = 0;
  bool grid_ready = false;
  DevBuf<PHitPoint> hp;
  DevBuf<float4> state;
  DevBuf<unsigned> nupd;
  DevBuf<int> pix_cnt, pix_off;
  DevBuf<PGrid> grid;
  DevBuf<int> bstart, bend;
  DevBuf<unsigned long long> gkeys, gkeys2;  // hit-point groups (same hash-cell range)
  DevBuf<int> gidx, perm, gflags, gid, gstart, ntile, tile_off;
  DevBuf<int2> tiles, tiles_lpt;  // tile table; per batch, heaviest first
  DevBuf<unsigned> tkey, tkey2;
  int n_groups = 0, n_tiles = 0;
  // photon batches
  DevBuf<PDeposit> slots;
  DevBuf<int> ndep, dep_off;
  DevBuf<unsigned> dbucket;                      // per dense deposit: its bucket
  DevBuf<PDeposit> dense;                        // deposits in photon order
  DevBuf<float4> dpos;                           // their positions alone
  DevBuf<int> pcount, poff, list_start, list_end;  // (group, deposit) expansion
  DevBuf<unsigned> pkey, pval, pkey2, pval2;
  DevBuf<unsigned> gb;                           // per group: buckets, multiplicity
  DevBuf<int> gm, gnb, goff, bg_start, bg_end;
  DevBuf<unsigned> bgkey, bgval, bgkey2, bgval2;  // bucket -> groups
  DevBuf<float4> gpos;  // per-group deposit lists, materialised (position, index | multiplicity)
  DevBuf<long long> cneed, cofs;  // per tile: compaction range size, offset (update pass)
  DevBuf<float4> cbuf;            // the compacted tile lists
  long long compact_min = -1;     // ppm_set_update_compaction (-1: default_compact_min())
  DevBuf<float> rrtab;                           // rr(n), n < kRRTable
  DevBuf<unsigned char> temp;
  DevBuf<unsigned long long> stats;  // [photons, photon_rays, deposits, updates, eye_rays]
  DevBuf<int> error;
  DevBuf<unsigned long long> wide;  // 64-bit scratch scalar (expansion total)
  DevBuf<unsigned long long> stats_keep;  // stats before a batch (restored when it is split)
  DevBuf<float> image;
  // update-kernel launches since the last collection: event pairs (reused from upd_spare),
  // completed ones beyond kMaxUpdEvents folded into upd_ms_folded / upd_folded
  std::vector<std::pair<hipEvent_t, hipEvent_t>> upd_events, upd_spare;
  double upd_ms_folded = 0;
  long long upd_folded = 0;
  long long photons = 0;
  size_t slot_bytes = 0;          // ppm_set_batching (0: default_slot_bytes())
  long long max_updates = INT_MAX;  // ppm_set_batching: (group, deposit) pairs per batch
  // update-pass shard (ppm_set_update_shard; replica d of a multi-device scene is shard d):
  // the update kernel runs only the tiles t with t mod shards == shard (build_grid)
  int shard = 0, shards = 1;
  DevBuf<int> owner;  // per hit point: the shard whose tiles update it (shards > 1)
  // multi-device scene (ppm_scene_load_xml_multi): this object is replica 0 on the first
  // device; peers[d - 1] is replica d.  Every replica runs the eye pass, the grid and the
  // whole photon sequence; each applies the update pass to its own tiles; `merged` is false
  // until the peers' hit-point state has been gathered here (merge_peers).
  std::vector<std::unique_ptr<ppm_scene>> peers;
  DevBuf<float4> peer_state;  // gathered peer state, shards x n_hp
  DevBuf<unsigned> peer_nupd;
  bool merged = true;
  // a single-device scene with shards > 1 (process per GPU) holds only its own tiles' results
  // after ppm_trace_photons, until ppm_write_hit_state brings in the merged state
  bool shard_partial = false;

  void drop_update_events() {  // (back to the pool)
    upd_spare.insert(upd_spare.end(), upd_events.begin(), upd_events.end());
    upd_events.clear();
    upd_ms_folded = 0;
    upd_folded = 0;
  }
  // an event pair for one update launch; the pending list stays bounded while nobody collects
  std::pair<hipEvent_t, hipEvent_t> update_event_pair() {
    static constexpr size_t kMaxUpdEvents = 64;
    if (upd_events.size() >= kMaxUpdEvents) {
      size_t k = 0;
      for (; k < upd_events.size(); k++) {
        float ms = 0;
        if (hipEventQuery(upd_events[k].second) != hipSuccess ||
            hipEventElapsedTime(&ms, upd_events[k].first, upd_events[k].second) != hipSuccess)
          break;
        upd_ms_folded += ms;
        upd_folded++;
        upd_spare.push_back(upd_events[k]);
      }
      upd_events.erase(upd_events.begin(), upd_events.begin() + (long)k);
    }
    std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
    if (!upd_spare.empty()) {
      ev = upd_spare.back();
      upd_spare.pop_back();
    } else {
      hip_check(hipEventCreate(&ev.first), "event");
      hip_check(hipEventCreate(&ev.second), "event");
    }
    upd_events.push_back(ev);
    return ev;
  }
  void free_all() {
    drop_update_events();
    for (auto& ev : upd_spare) (void)hipEventDestroy(ev.first), (void)hipEventDestroy(ev.second);
    upd_spare.clear();
    for (void* p : owned) (void)hipFree(p);
    owned.clear();
    hp.release(), state.release(), nupd.release(), pix_cnt.release(), pix_off.release();
    grid.release(), bstart.release(), bend.release(), slots.release(), ndep.release();
    owner.release(), peer_state.release(), peer_nupd.release();
    gkeys.release(), gkeys2.release(), gidx.release(), perm.release(), gflags.release();
    gid.release(), gstart.release(), ntile.release(), tile_off.release(), tiles.release();
    tiles_lpt.release(), tkey.release(), tkey2.release();
    dep_off.release(), dbucket.release(), dense.release(), dpos.release(), pcount.release(), poff.release();
    list_start.release(), list_end.release(), pkey.release(), pval.release(), pkey2.release();
    pval2.release(), gb.release(), gm.release(), gnb.release(), goff.release();
    bg_start.release(), bg_end.release(), bgkey.release(), bgval.release(), bgkey2.release();
    bgval2.release(), gpos.release(), rrtab.release();
    cneed.release(), cofs.release(), cbuf.release();
    temp.release(), stats.release(), error.release(), image.release();
    wide.release(), stats_keep.release();
    if (stream) (void)hipStreamDestroy(stream);
    stream = nullptr;
  }
};

namespace {


// Tile-list compaction in the update pass (group_update_kernel phase (0)): tiles whose group
// list holds at least this many deposits copy the reachable ones first.  Results do not depend
// on it (the copy is a superset of every window's candidates, in order).
// ppm_set_update_compaction sets it per scene (0: off).
#ifndef PPM_COMPACT_SHIFT  // (A/B builds)
#define PPM_COMPACT_SHIFT 2
#endif
constexpr int kCompactShift = PPM_COMPACT_SHIFT;  // scratch per compacted tile: a quarter of its list
constexpr int kDefaultCompactSeg = 32768;  // deposits per compaction segment
long long default_compact_min() { return 65536LL; }

template <typename T>
const T* own(ppm_scene* s, const std::vector<T>& v, const char* what) {
  T* p = upload(v, what);
  s->owned.push_back(p);
  return p;
}

void create_device(ppm_scene* s, int device) {
  s->device = device;
  DeviceGuard g(device);
  hip_check(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking), "stream");
  const HostPPM& h = s->host;
  PScene& S = s->S;
  S.top_nodes = own(s, h.top_nodes, "upload top nodes");
  S.objects = own(s, h.objects, "upload objects");
  S.mesh_nodes = own(s, h.mesh_nodes, "upload mesh nodes");
  S.triangles = own(s, h.triangles, "upload triangles");
  S.meshes = own(s, h.meshes, "upload meshes");
  S.vpos = own(s, h.vpos, "upload vertices");
  S.vnormal = own(s, h.vnormal, "upload vertex normals");
  S.materials = own(s, h.materials, "upload materials");
  S.top_root = h.top_root;
  S.max_depth = h.max_depth;
  S.lds_stack = (h.top_depth + 1 <= kLdsStack && h.mesh_depth + 1 <= kLdsStack) ? 1 : 0;
  S.eps = h.eps;
#ifdef PPM_DIAG_LEVEL  // experiment builds (make ppm-exp EXTRA=-DPPM_DIAG_LEVEL=2): diag counters
  S.diag = PPM_DIAG_LEVEL;
#endif
  S.compact_seg = kDefaultCompactSeg;
  std::memcpy(S.light_pos, h.lights.data(), 12);  // lights[0] (Scene.cpp:97)
  std::memcpy(S.light_intensity, h.lights.data() + 3, 12);
  s->stats.reserve(kStatSlots, "alloc counters");
  hip_check(hipMemset(s->stats.p, 0, kStatSlots * sizeof(unsigned long long)), "zero counters");
  s->error.reserve(1, "alloc error flag");
  s->wide.reserve(1, "alloc scratch scalar");
  s->stats_keep.reserve(kStatSlots, "alloc stats snapshot");
  hip_check(hipMemset(s->error.p, 0, sizeof(int)), "zero error flag");
  s->grid.reserve(1, "alloc grid");
  s->rrtab.reserve(kRRTable, "alloc radius-reduction table");
  hip_check(launch_rr_table(s->rrtab.p, kRRTable, s->stream), "radius-reduction table");
}

void check_scene(const ppm_scene* s) {
  if (!s) throw std::invalid_argument("scene is NULL");
}

void eye_pass(ppm_scene* s, int cam) {
  if (cam < 0 || cam >= (int)s->host.cameras.size())
    throw std::invalid_argument("camera index out of range");
  const PCamera C = s->host.cameras[cam].cam;
  const int npix = C.width * C.height;
  s->pix_cnt.reserve(npix + 1, "alloc pixel counts");
  s->pix_off.reserve(npix + 1, "alloc pixel offsets");
  hip_check(hipMemsetAsync(s->pix_cnt.p, 0, (npix + 1) * sizeof(int), s->stream), "zero counts");
  hip_check(launch_eye(s->S, C, s->seed, s->pix_cnt.p, nullptr, nullptr, s->stats.p, s->stream),
            "eye pass (count)");
  size_t bytes = 0;
  hip_check(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, s->pix_cnt.p, s->pix_off.p, npix + 1,
                                             s->stream), "scan size");
  s->temp.reserve(bytes, "alloc scan temp");
  hip_check(hipcub::DeviceScan::ExclusiveSum(s->temp.p, bytes, s->pix_cnt.p, s->pix_off.p,
                                             npix + 1, s->stream), "scan hit points");
  int total = 0;
  hip_check(hipMemcpyAsync(&total, s->pix_off.p + npix, sizeof(int), hipMemcpyDeviceToHost,
                           s->stream), "read hit-point count");
  hip_check(hipStreamSynchronize(s->stream), "eye pass");
  s->hp.reserve(total, "alloc hit points");
  s->state.reserve(total, "alloc hit-point state");
  s->nupd.reserve(total, "alloc hit-point counts");
  hip_check(launch_eye(s->S, C, s->seed, nullptr, s->pix_off.p, s->hp.p, nullptr, s->stream),
            "eye pass (write)");
  s->n_hp = total;
  s->eye_cam = cam;
  s->grid_ready = false;
}

void build_grid(ppm_scene* s, int width, int height) {
  if (s->eye_cam < 0) throw std::invalid_argument("build_hash_grid before the eye pass");
  const int n = s->n_hp;
  s->grid_ready = false;
  s->shard_partial = false;  // the state is reset below
  // a failed earlier build may have left the device error flag set: every pass reads it
  hip_check(hipMemsetAsync(s->error.p, 0, sizeof(int), s->stream), "zero error flag");
  hip_check(launch_grid(s->hp.p, n, width, height, s->grid.p, s->state.p, s->nupd.p, s->stream),
            "build hash grid");
  s->bstart.reserve(std::max(1, n), "alloc bucket starts");
  s->bend.reserve(std::max(1, n), "alloc bucket ends");
  s->n_groups = 0;
  if (n > 0) {  // group the hit points by hash-cell range (group_update_kernel)
    s->gkeys.reserve(n, "alloc group keys");
    s->gkeys2.reserve(n, "alloc group keys");
    s->gidx.reserve(n, "alloc group index");
    s->perm.reserve(n, "alloc group permutation");
    s->gflags.reserve(n + 1, "alloc group flags");
    s->gid.reserve(n + 1, "alloc group ids");
    s->gstart.reserve(n + 1, "alloc group starts");
    hip_check(launch_group_keys(s->hp.p, n, s->grid.p, s->gkeys.p, s->gidx.p, s->error.p,
                                s->stream), "group keys");
    size_t bytes = 0;
    hip_check(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, s->gkeys.p, s->gkeys2.p, s->gidx.p,
                                                 s->perm.p, n, 0, 64, s->stream), "sort size");
    s->temp.reserve(bytes, "alloc sort temp");
    hip_check(hipcub::DeviceRadixSort::SortPairs(s->temp.p, bytes, s->gkeys.p, s->gkeys2.p,
                                                 s->gidx.p, s->perm.p, n, 0, 64, s->stream),
              "sort hit points by cell range");
    hip_check(launch_group_flags(s->gkeys2.p, n, s->gflags.p, s->stream), "group flags");
    bytes = 0;
    hip_check(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, s->gflags.p, s->gid.p, n + 1,
                                               s->stream), "scan size");
    s->temp.reserve(bytes, "alloc scan temp");
    hip_check(hipcub::DeviceScan::ExclusiveSum(s->temp.p, bytes, s->gflags.p, s->gid.p, n + 1,
                                               s->stream), "scan groups");
    hip_check(launch_group_starts(s->gflags.p, s->gid.p, n, s->gstart.p, s->stream), "group starts");
    int groups = 0, err = 0;
    hip_check(hipMemcpyAsync(&groups, s->gid.p + n, sizeof(int), hipMemcpyDeviceToHost, s->stream),
              "read group count");
    hip_check(hipMemcpyAsync(&err, s->error.p, sizeof(int), hipMemcpyDeviceToHost, s->stream),
              "read error flag");
    hip_check(hipStreamSynchronize(s->stream), "group hit points");
    if (err) throw std::domain_error("a hit point's radius box spans more hash cells than supported");
    s->n_groups = groups;
    // tiles of <= kTileHP (5) hit points per group (group_update_kernel)
    s->ntile.reserve(groups + 1, "alloc tile counts");
    s->tile_off.reserve(groups + 1, "alloc tile offsets");
    hip_check(launch_group_tiles(s->gstart.p, groups, s->ntile.p, s->stream), "group tiles");
    bytes = 0;
    hip_check(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, s->ntile.p, s->tile_off.p, groups + 1,
                                               s->stream), "scan size");
    s->temp.reserve(bytes, "alloc scan temp");
    hip_check(hipcub::DeviceScan::ExclusiveSum(s->temp.p, bytes, s->ntile.p, s->tile_off.p,
                                               groups + 1, s->stream), "scan tiles");
    int ntiles = 0;
    hip_check(hipMemcpyAsync(&ntiles, s->tile_off.p + groups, sizeof(int), hipMemcpyDeviceToHost,
                             s->stream), "read tile count");
    hip_check(hipStreamSynchronize(s->stream), "tile count");
    s->tiles.reserve(std::max(1, ntiles), "alloc tiles");
    hip_check(launch_tile_table(s->gstart.p, s->tile_off.p, groups, s->tiles.p, s->stream),
              "tile table");
    s->n_tiles = ntiles;
    if (s->shards > 1) {  // this shard's tiles (table order), and every hit point's shard
      s->owner.reserve(n, "alloc hit-point shards");
      s->tiles_lpt.reserve(std::max(1, ntiles), "alloc shard tiles");
      hip_check(launch_tile_shard(s->tiles.p, ntiles, s->shard, s->shards, s->gstart.p, s->perm.p,
                                  s->tiles_lpt.p, s->owner.p, s->stream), "tile shard");
      s->n_tiles = ntiles > s->shard ? (ntiles - s->shard + s->shards - 1) / s->shards : 0;
      if (s->n_tiles > 0)
        hip_check(hipMemcpyAsync(s->tiles.p, s->tiles_lpt.p, s->n_tiles * sizeof(int2),
                                 hipMemcpyDeviceToDevice, s->stream), "shard tiles");
    }
    // each group's buckets, and the bucket -> groups map the expansion uses
    s->gb.reserve((size_t)groups * kMaxCells, "alloc group buckets");
    s->gm.reserve((size_t)groups * kMaxCells, "alloc group multiplicities");
    s->gnb.reserve(groups + 1, "alloc group bucket counts");
    s->goff.reserve(groups + 1, "alloc group bucket offsets");
    hip_check(launch_group_buckets(s->hp.p, s->perm.p, s->gstart.p, groups, s->grid.p, s->gb.p,
                                   s->gm.p, s->gnb.p, s->stream), "group buckets");
    bytes = 0;
    hip_check(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, s->gnb.p, s->goff.p, groups + 1,
                                               s->stream), "scan size");
    s->temp.reserve(bytes, "alloc scan temp");
    hip_check(hipcub::DeviceScan::ExclusiveSum(s->temp.p, bytes, s->gnb.p, s->goff.p, groups + 1,
                                               s->stream), "scan group buckets");
    int npairs = 0;
    hip_check(hipMemcpyAsync(&npairs, s->goff.p + groups, sizeof(int), hipMemcpyDeviceToHost,
                             s->stream), "read pair count");
    hip_check(hipStreamSynchronize(s->stream), "pair count");
    s->bgkey.reserve(npairs, "alloc bucket-group keys");
    s->bgval.reserve(npairs, "alloc bucket-group values");
    s->bgkey2.reserve(npairs, "alloc bucket-group keys");
    s->bgval2.reserve(npairs, "alloc bucket-group values");
    if (groups >= (1 << kGroupBits)) throw std::domain_error("too many hit-point groups");
    hip_check(launch_bucket_group_pairs(s->gb.p, s->gm.p, s->gnb.p, s->goff.p, groups, s->bgkey.p,
                                        s->bgval.p, s->stream), "bucket-group pairs");
    int hbits = 1;
    while (hbits < 32 && (1ull << hbits) < (unsigned long long)n) hbits++;
    bytes = 0;
    hip_check(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, s->bgkey.p, s->bgkey2.p, s->bgval.p,
                                                 s->bgval2.p, npairs, 0, hbits, s->stream), "sort size");
    s->temp.reserve(bytes, "alloc sort temp");
    hip_check(hipcub::DeviceRadixSort::SortPairs(s->temp.p, bytes, s->bgkey.p, s->bgkey2.p,
                                                 s->bgval.p, s->bgval2.p, npairs, 0, hbits,
                                                 s->stream), "sort bucket-group pairs");
    s->bg_start.reserve(n, "alloc bucket-group starts");
    s->bg_end.reserve(n, "alloc bucket-group ends");
    hip_check(hipMemsetAsync(s->bg_start.p, 0, n * sizeof(int), s->stream), "zero");
    hip_check(hipMemsetAsync(s->bg_end.p, 0, n * sizeof(int), s->stream), "zero");
    hip_check(launch_bucket_bounds(s->bgkey2.p, npairs, ~0u, s->bg_start.p, s->bg_end.p, s->stream),
              "bucket-group bounds");
    s->list_start.reserve(groups, "alloc list starts");
    s->list_end.reserve(groups, "alloc list ends");
  }
  s->grid_ready = true;
}

void trace_photons(ppm_scene* s, long long first, long long count) {
  if (count < 0 || first < 0) throw std::invalid_argument("bad photon range");
  if (!s->grid_ready) throw std::invalid_argument("trace_photons before build_hash_grid");
  const int K = std::max(1, s->host.max_depth - 1);
  size_t budget = s->slot_bytes ? s->slot_bytes : default_slot_bytes();
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) == hipSuccess)
    budget = std::min(budget, (free_b + s->slots.cap * sizeof(PDeposit)) / 4);
  // slot rows and deposit counts are indexed with int: b * K < 2^31
  long long batch_max = std::max<long long>(1, (long long)(budget / (sizeof(PDeposit) * K)));
  batch_max = std::min<long long>(batch_max, (INT_MAX - 1) / K);
  const int H = s->n_hp;
  for (long long done = 0; done < count;) {
    int b = (int)std::min(count - done, batch_max);
    s->slots.reserve((size_t)b * K, "alloc deposit slots");
    s->ndep.reserve(b + 1, "alloc deposit counts");
    s->dep_off.reserve(b + 1, "alloc deposit offsets");
    hip_check(hipMemsetAsync(s->ndep.p + b, 0, sizeof(int), s->stream), "zero sentinel");
    hip_check(hipMemcpyAsync(s->stats_keep.p, s->stats.p, kStatSlots * sizeof(unsigned long long),
                             hipMemcpyDeviceToDevice, s->stream), "stats snapshot");
    hip_check(launch_photons(s->S, s->seed, first + done, b, K, s->slots.p, s->ndep.p, s->stats.p,
                             s->stream), "photon pass");
    if (H > 0) {
      size_t bytes = 0;
      hip_check(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, s->ndep.p, s->dep_off.p, b + 1,
                                                 s->stream), "scan size");
      s->temp.reserve(bytes, "alloc scan temp");
      hip_check(hipcub::DeviceScan::ExclusiveSum(s->temp.p, bytes, s->ndep.p, s->dep_off.p, b + 1,
                                                 s->stream), "scan deposits");
      int D = 0;
      hip_check(hipMemcpyAsync(&D, s->dep_off.p + b, sizeof(int), hipMemcpyDeviceToHost,
                               s->stream), "read deposit count");
      hip_check(hipStreamSynchronize(s->stream), "photon batch");
      if (D > 0) {
        // deposits in photon order, with their buckets
        s->dense.reserve(D, "alloc dense deposits");
        s->dbucket.reserve(D, "alloc deposit buckets");
        s->dpos.reserve(D, "alloc deposit positions");
        hip_check(launch_deposit_keys(s->slots.p, s->ndep.p, s->dep_off.p, b, K, s->grid.p,
                                      s->dbucket.p, s->dense.p, s->dpos.p, s->stream), "deposit keys");
        // each deposit into every group filed under its bucket; a stable sort by group gives
        // each group its deposit list in photon order
        s->pcount.reserve(D + 1, "alloc expansion counts");
        s->poff.reserve(D + 1, "alloc expansion offsets");
        hip_check(launch_expand_count(s->dbucket.p, D, s->bg_start.p, s->bg_end.p, s->pcount.p,
                                      s->stream), "expansion count");
        // the expansion size in 64 bits first: the int scan below must not wrap
        long long* d_total = reinterpret_cast<long long*>(s->wide.p);
        hipcub::TransformInputIterator<long long, WidenInt, const int*> wide_in(s->pcount.p,
                                                                               WidenInt());
        bytes = 0;
        hip_check(hipcub::DeviceReduce::Sum(nullptr, bytes, wide_in, d_total, D, s->stream),
                  "reduce size");
        s->temp.reserve(bytes, "alloc reduce temp");
        hip_check(hipcub::DeviceReduce::Sum(s->temp.p, bytes, wide_in, d_total, D, s->stream),
                  "expansion total");
        long long P64 = 0;
        hip_check(hipMemcpyAsync(&P64, d_total, sizeof P64, hipMemcpyDeviceToHost, s->stream),
                  "read expansion total");
        hip_check(hipStreamSynchronize(s->stream), "expansion total");
        if (P64 >= std::min<long long>(INT_MAX, s->max_updates) || D >= kMaxBatchDeposits) {
          // too many (group, deposit) pairs, or deposits, for one batch (the pair records
          // index deposits in 27 bits): trace a smaller batch (photon streams are per photon,
          // so the same photons come out again) and keep it smaller
          if (b == 1) throw std::domain_error("one photon expands to more than 2^31 updates");
          batch_max = std::max(1, b / 2);
          hip_check(hipMemcpyAsync(s->stats.p, s->stats_keep.p, kStatSlots * sizeof(unsigned long long),
                                   hipMemcpyDeviceToDevice, s->stream), "stats restore");
          continue;
        }
        bytes = 0;
        hip_check(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, s->pcount.p, s->poff.p, D + 1,
                                                   s->stream), "scan size");
        s->temp.reserve(bytes, "alloc scan temp");
        hip_check(hipcub::DeviceScan::ExclusiveSum(s->temp.p, bytes, s->pcount.p, s->poff.p, D + 1,
                                                   s->stream), "scan expansion");
        const int P = (int)P64;
        hip_check(hipMemsetAsync(s->list_start.p, 0, s->n_groups * sizeof(int), s->stream), "zero");
        hip_check(hipMemsetAsync(s->list_end.p, 0, s->n_groups * sizeof(int), s->stream), "zero");
        if (P > 0) {
          s->pkey.reserve(P, "alloc expansion keys");
          s->pval.reserve(P, "alloc expansion values");
          s->pkey2.reserve(P, "alloc expansion keys");
          s->pval2.reserve(P, "alloc expansion values");
          hip_check(launch_expand_write(s->dbucket.p, D, s->bg_start.p, s->bg_end.p, s->bgval2.p,
                                        s->poff.p, s->pkey.p, s->pval.p, s->stream),
                    "expansion write");
          int gbits = 1;
          while (gbits < 32 && (1ull << gbits) < (unsigned long long)s->n_groups) gbits++;
          bytes = 0;
          hip_check(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, s->pkey.p, s->pkey2.p,
                                                       s->pval.p, s->pval2.p, P, 0, gbits,
                                                       s->stream), "sort size");
          s->temp.reserve(bytes, "alloc sort temp");
          hip_check(hipcub::DeviceRadixSort::SortPairs(s->temp.p, bytes, s->pkey.p, s->pkey2.p,
                                                       s->pval.p, s->pval2.p, P, 0, gbits,
                                                       s->stream), "sort expansion by group");
          hip_check(launch_bucket_bounds(s->pkey2.p, P, (1u << kGroupBits) - 1u, s->list_start.p,
                                         s->list_end.p, s->stream),
                    "group list bounds");
          s->gpos.reserve(P, "alloc group deposit lists");
          hip_check(launch_materialize(s->pkey2.p, s->pval2.p, P, s->dpos.p, s->gpos.p, s->stream),
                    "materialise group lists");
          // longest-first update order (tile_work_kernel): the hot groups' serial chains start
          // in the first dispatch round.  The order cannot change results: tiles own disjoint
          // hit points.
          const int2* tiles = s->tiles.p;
          {
            s->tkey.reserve(s->n_tiles, "alloc tile keys");
            s->tkey2.reserve(s->n_tiles, "alloc tile keys");
            s->tiles_lpt.reserve(s->n_tiles, "alloc tile order");
            hip_check(launch_tile_work(s->tiles.p, s->n_tiles, s->list_start.p, s->list_end.p,
                                       s->tkey.p, s->stream), "tile work");
            bytes = 0;
            hip_check(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, s->tkey.p, s->tkey2.p,
                                                         s->tiles.p, s->tiles_lpt.p, s->n_tiles,
                                                         0, 32, s->stream), "sort size");
            s->temp.reserve(bytes, "alloc sort temp");
            hip_check(hipcub::DeviceRadixSort::SortPairs(s->temp.p, bytes, s->tkey.p, s->tkey2.p,
                                                         s->tiles.p, s->tiles_lpt.p, s->n_tiles,
                                                         0, 32, s->stream), "sort tiles");
            tiles = s->tiles_lpt.p;
          }
          // scratch ranges of the tiles whose lists get compacted (none: cofs stays null)
          const long long cmin = s->compact_min >= 0 ? s->compact_min : default_compact_min();
          const long long* cofs = nullptr;
          if (cmin > 0) {
            s->cneed.reserve(s->n_tiles + 1, "alloc compaction sizes");
            s->cofs.reserve(s->n_tiles + 1, "alloc compaction offsets");
            hip_check(launch_tile_compact_need(tiles, s->n_tiles, s->list_start.p, s->list_end.p,
                                               cmin, kCompactShift, s->S.compact_seg,
                                               s->cneed.p, s->stream),
                      "compaction sizes");
            bytes = 0;
            hip_check(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, s->cneed.p, s->cofs.p,
                                                       s->n_tiles + 1, s->stream), "scan size");
            s->temp.reserve(bytes, "alloc scan temp");
            hip_check(hipcub::DeviceScan::ExclusiveSum(s->temp.p, bytes, s->cneed.p, s->cofs.p,
                                                       s->n_tiles + 1, s->stream),
                      "compaction offsets");
            long long ctotal = 0;
            hip_check(hipMemcpyAsync(&ctotal, s->cofs.p + s->n_tiles, sizeof ctotal,
                                     hipMemcpyDeviceToHost, s->stream), "read compaction total");
            hip_check(hipStreamSynchronize(s->stream), "compaction total");
            size_t cfree = 0, ctot = 0;
            const bool fits = hipMemGetInfo(&cfree, &ctot) == hipSuccess &&
                              (size_t)ctotal * sizeof(float4) <=
                                  (cfree + s->cbuf.cap * sizeof(float4)) / 4;
            if (ctotal > 0 && fits) {
              s->cbuf.reserve((size_t)ctotal, "alloc compacted tile lists");
              cofs = s->cofs.p;
            }
          }
          const auto ev = s->update_event_pair();
          const hipEvent_t e0 = ev.first, e1 = ev.second;
          hip_check(hipEventRecord(e0, s->stream), "event");
          hip_check(launch_group_update(s->S, s->hp.p, s->perm.p, s->gstart.p, tiles,
                                        s->n_tiles, s->list_start.p, s->list_end.p, s->gpos.p,
                                        s->dense.p, s->rrtab.p, kRRTable, s->state.p, s->nupd.p,
                                        cofs, s->cbuf.p, s->stats.p, s->stream),
                    "hit-point updates");
          hip_check(hipEventRecord(e1, s->stream), "event");
        }
      }
    }
    done += b;
  }
  s->photons += count;
  int err = 0;
  hip_check(hipMemcpyAsync(&err, s->error.p, sizeof(int), hipMemcpyDeviceToHost, s->stream),
            "read error flag");
  hip_check(hipStreamSynchronize(s->stream), "photon pass");
  if (err) throw std::domain_error("photon pass: device error flag set");
}

void density(ppm_scene* s, long long total, float* out) {
  if (s->eye_cam < 0) throw std::invalid_argument("density_estimation before the eye pass");
  const PCamera& C = s->host.cameras[s->eye_cam].cam;
  const int npix = C.width * C.height;
  s->image.reserve((size_t)npix * 3, "alloc image");
  hip_check(launch_density(s->hp.p, s->state.p, s->pix_off.p, npix, (double)total, s->image.p,
                           s->stream), "density estimation");
  hip_check(hipMemcpyAsync(out, s->image.p, (size_t)npix * 3 * sizeof(float),
                           hipMemcpyDeviceToHost, s->stream), "copy image");
  hip_check(hipStreamSynchronize(s->stream), "density estimation");
}

// Runs f on every replica of a multi-device scene — replica 0 on the calling thread, each peer
// on a thread of its own with its device current — and rethrows the first failure once all
// have finished.  A single-device scene runs f(s) alone.
template <typename F>
void each_replica(ppm_scene* s, F&& f) {
  if (s->peers.empty()) {
    DeviceGuard g(s->device);  // the scene's buffers and stream live on its device
    f(s);
    return;
  }
  std::vector<std::exception_ptr> err(s->peers.size() + 1);
  std::vector<std::thread> th;
  th.reserve(s->peers.size());
  for (size_t d = 0; d < s->peers.size(); d++) {
    ppm_scene* p = s->peers[d].get();
    th.emplace_back([&f, &err, p, d] {
      try {
        DeviceGuard g(p->device);
        f(p);
      } catch (...) {
        err[d + 1] = std::current_exception();
      }
    });
  }
  try {
    DeviceGuard g(s->device);
    f(s);
  } catch (...) {
    err[0] = std::current_exception();
  }
  for (auto& t : th) t.join();
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
}

// Gathers a multi-device scene's sharded update results onto replica 0: each peer's (state,
// count) arrays are copied device to device (xGMI peer copies; the peers' passes have ended
// with a stream synchronisation), then every hit point takes the values of the replica whose
// tiles own it (merge_state_kernel).  Ordered on replica 0's stream.
void merge_peers(ppm_scene* s) {
  if (s->merged || s->peers.empty() || !s->grid_ready || s->n_hp == 0) {
    s->merged = true;
    return;
  }
  const int n = s->n_hp;
  const size_t D = s->peers.size() + 1;
  DeviceGuard g(s->device);
  s->peer_state.reserve(D * n, "alloc gathered hit-point state");
  s->peer_nupd.reserve(D * n, "alloc gathered hit-point counts");
  for (size_t d = 1; d < D; d++) {
    const ppm_scene* p = s->peers[d - 1].get();
    if (p->n_hp != n) throw std::runtime_error("multi-device PPM: replicas disagree on the hit points");
    hip_check(hipMemcpyPeerAsync(s->peer_state.p + d * n, s->device, p->state.p, p->device,
                                 (size_t)n * sizeof(float4), s->stream), "gather state");
    hip_check(hipMemcpyPeerAsync(s->peer_nupd.p + d * n, s->device, p->nupd.p, p->device,
                                 (size_t)n * sizeof(unsigned), s->stream), "gather counts");
  }
  hip_check(launch_merge_state(s->owner.p, n, 0, s->peer_state.p, s->peer_nupd.p, s->state.p,
                               s->nupd.p, s->stream), "merge state");
  s->merged = true;
}

// Device counters of one replica's passes since the last collection (and resets them).
void collect(ppm_scene* s, ppm_stats* st) {
  DeviceGuard g(s->device);
  unsigned long long c[kStatSlots];
  hip_check(hipMemcpyAsync(c, s->stats.p, sizeof c, hipMemcpyDeviceToHost, s->stream), "read counters");
  hip_check(hipMemsetAsync(s->stats.p, 0, sizeof c, s->stream), "reset counters");
  hip_check(hipStreamSynchronize(s->stream), "counters");
  std::memset(st, 0, sizeof *st);
  st->photons = s->photons;
  st->photon_rays = (long long)c[1];
  st->deposits = (long long)c[2];
  st->updates = (long long)c[3];
  st->eye_rays = (long long)c[4];
  st->hit_points = s->n_hp;
  st->update_deposit_visits = (long long)c[6];
  st->update_candidates = (long long)c[16];
  st->update_launches = s->upd_folded + (long long)s->upd_events.size();
  st->update_compacted_segments = (long long)c[20];
  st->update_compaction_fallbacks = (long long)c[21];
  st->update_compacted_deposits = (long long)c[22];
  st->update_ms = s->upd_ms_folded;
  for (auto& ev : s->upd_events) {
    float ms = 0;
    hip_check(hipEventElapsedTime(&ms, ev.first, ev.second), "update time");
    st->update_ms += ms;
  }
  s->drop_update_events();
  if (s->S.diag == 2) std::fprintf(stderr, "ppm diag: windows %llu deposit-visits %llu tiles %d groups %d "
                                   "longest tile %llu ticks phases(max) stage+filter %llu "
                                   "counts %llu scan %llu scatter %llu color %llu gate %llu max-window-updates %llu "
                                   "unstaged-rr %llu candidates %llu max-tile-candidates %llu max-wave-updates %llu max-tile-windows %llu "
                                   "compacted-segments %llu fallbacks %llu compacted-deposits %llu "
                                   "tile-ticks-sum %llu phases(sum) %llu %llu %llu %llu %llu %llu gate0(RK, all) %llu %llu "
                                   "compaction(sum, max) %llu %llu\n",
                                   c[5], c[6], s->n_tiles, s->n_groups, c[7], c[8], c[9],
                                   c[10], c[11], c[12], c[13], c[14], c[15], c[16], c[17], c[18], c[19],
                                   c[20], c[21], c[22], c[23], c[24], c[25], c[26], c[27], c[28], c[29], c[30], c[31],
                                   c[32], c[33]);
  s->photons = 0;
}

// The counters of every replica: the photon sequence, eye pass and grid are replicated, so
// those counts are replica 0's; the update pass is sharded, so its work is summed, and its
// device time is the longest replica's (they run concurrently).
void collect_all(ppm_scene* s, ppm_stats* st) {
  collect(s, st);
  for (auto& p : s->peers) {
    ppm_stats q;
    collect(p.get(), &q);
    st->updates += q.updates;
    st->update_deposit_visits += q.update_deposit_visits;
    st->update_candidates += q.update_candidates;
    st->update_launches += q.update_launches;
    st->update_compacted_segments += q.update_compacted_segments;
    st->update_compaction_fallbacks += q.update_compaction_fallbacks;
    st->update_compacted_deposits += q.update_compacted_deposits;
    st->update_ms = std::max(st->update_ms, q.update_ms);
  }
}

}  // namespace

extern "C" {

int ppm_abi_version(void) { return CENG795_PPM_ABI_VERSION; }
const char* ppm_last_error(void) { return g_error.c_str(); }

int ppm_scene_load_xml(const char* xml_path, int device, ppm_scene** out) {
  if (!xml_path || !out) return set_error(RT_E_INVALID, "ppm_scene_load_xml: NULL argument");
  *out = nullptr;
  auto s = std::make_unique<ppm_scene>();
  const int rc = guarded([&] {
    load_ppm_xml(xml_path, s->host);
    create_device(s.get(), device);
    return RT_OK;
  });
  if (rc != RT_OK) {
    s->free_all();
    return rc;
  }
  *out = s.release();
  return RT_OK;
}

int ppm_scene_load_xml_multi(const char* xml_path, int device_count, const int* devices,
                             ppm_scene** out) {
  if (!xml_path || !out || device_count < 1 || !devices)
    return set_error(RT_E_INVALID, "ppm_scene_load_xml_multi: bad argument");
  *out = nullptr;
  auto s = std::make_unique<ppm_scene>();
  const int rc = guarded([&] {
    load_ppm_xml(xml_path, s->host);
    create_device(s.get(), devices[0]);
    s->shards = device_count;
    for (int d = 1; d < device_count; d++) {
      s->peers.push_back(std::make_unique<ppm_scene>());
      ppm_scene* p = s->peers.back().get();
      p->host = s->host;
      create_device(p, devices[d]);
      p->shard = d;
      p->shards = device_count;
    }
    return RT_OK;
  });
  if (rc != RT_OK) {
    ppm_scene_destroy(s.release());
    return rc;
  }
  *out = s.release();
  return RT_OK;
}

void ppm_scene_destroy(ppm_scene* s) {
  if (!s) return;
  for (auto& p : s->peers) ppm_scene_destroy(p.release());
  s->peers.clear();
  int cur = -1;
  if (hipGetDevice(&cur) == hipSuccess && cur != s->device) (void)hipSetDevice(s->device);
  s->free_all();
  if (cur >= 0 && cur != s->device) (void)hipSetDevice(cur);
  delete s;
}

int ppm_scene_device_count(const ppm_scene* s) { return s ? 1 + (int)s->peers.size() : 0; }

int ppm_set_update_shard(ppm_scene* s, int shard, int shards) {
  if (!s || shards < 1 || shard < 0 || shard >= shards)
    return set_error(RT_E_INVALID, "ppm_set_update_shard: bad argument (0 <= shard < shards)");
  if (!s->peers.empty())
    return set_error(RT_E_INVALID, "ppm_set_update_shard: a multi-device scene shards its own update pass");
  s->shard = shard;
  s->shards = shards;
  s->shard_partial = false;
  s->grid_ready = false;  // the tile table is the grid's: build_hash_grid again
  return RT_OK;
}

int ppm_hit_point_shards(ppm_scene* s, int* out) {
  return guarded([&] {
    check_scene(s);
    if (!out) throw std::invalid_argument("ppm_hit_point_shards: NULL output");
    if (!s->grid_ready) throw std::invalid_argument("no hash grid yet");
    DeviceGuard g(s->device);
    if (s->shards == 1 || s->n_hp == 0) {
      std::fill(out, out + s->n_hp, 0);
      return RT_OK;
    }
    hip_check(hipMemcpyAsync(out, s->owner.p, (size_t)s->n_hp * sizeof(int), hipMemcpyDeviceToHost,
                             s->stream), "read hit-point shards");
    hip_check(hipStreamSynchronize(s->stream), "read hit-point shards");
    return RT_OK;
  });
}

int ppm_write_hit_state(ppm_scene* s, const float* in) {
  return guarded([&] {
    check_scene(s);
    if (!in) throw std::invalid_argument("ppm_write_hit_state: NULL input");
    if (!s->grid_ready) throw std::invalid_argument("no hash grid yet");
    const int n = s->n_hp;
    std::vector<float4> st(n);
    std::vector<unsigned> cnt(n);
    for (int k = 0; k < n; k++) {
      const float* r = in + 5 * (size_t)k;
      // counts travel as float32 (the read_hit_state layout): exact up to 2^24
      if (!(r[4] >= 0.0f && r[4] <= 16777216.0f && r[4] == (float)(unsigned)r[4]))
        throw std::invalid_argument("bad update count (a whole number <= 2^24 expected)");
      st[k] = make_float4(r[0], r[1], r[2], r[3]);
      cnt[k] = (unsigned)r[4];
    }
    each_replica(s, [&](ppm_scene* r) {
      if (n == 0) return;
      hip_check(hipMemcpyAsync(r->state.p, st.data(), n * sizeof(float4), hipMemcpyHostToDevice,
                               r->stream), "write state");
      hip_check(hipMemcpyAsync(r->nupd.p, cnt.data(), n * sizeof(unsigned), hipMemcpyHostToDevice,
                               r->stream), "write counts");
      hip_check(hipStreamSynchronize(r->stream), "write state");
    });
    s->merged = true;
    s->shard_partial = false;
    return RT_OK;
  });
}

int ppm_num_cameras(const ppm_scene* s) { return s ? (int)s->host.cameras.size() : 0; }

int ppm_camera_info(const ppm_scene* s, int cam, int* w, int* h, int* n) {
  if (!s || cam < 0 || cam >= (int)s->host.cameras.size() || !w || !h || !n)
    return set_error(RT_E_INVALID, "ppm_camera_info: bad argument");
  const PCamera& c = s->host.cameras[cam].cam;
  *w = c.width, *h = c.height, *n = c.samples;
  return RT_OK;
}

const char* ppm_image_name(const ppm_scene* s, int cam) {
  if (!s || cam < 0 || cam >= (int)s->host.cameras.size()) return "";
  return s->host.cameras[cam].image_name.c_str();
}

int ppm_settings(const ppm_scene* s, int* per_iteration, int* iterations, int* max_depth) {
  if (!s || !per_iteration || !iterations || !max_depth)
    return set_error(RT_E_INVALID, "ppm_settings: NULL argument");
  *per_iteration = s->host.per_iteration;
  *iterations = s->host.iterations;
  *max_depth = s->host.max_depth;
  return RT_OK;
}

int ppm_set_update_compaction(ppm_scene* s, long long min_list) {
  if (!s || min_list < -1) return set_error(RT_E_INVALID, "ppm_set_update_compaction: bad argument");
  s->compact_min = min_list;
  for (auto& p : s->peers) p->compact_min = min_list;
  return RT_OK;
}

int ppm_set_update_segment(ppm_scene* s, int seg_len) {
  if (!s || seg_len < 0 || (seg_len > 0 && seg_len < 64))
    return set_error(RT_E_INVALID, "ppm_set_update_segment: bad argument (0, or >= 64)");
  s->S.compact_seg = seg_len ? seg_len : kDefaultCompactSeg;
  for (auto& p : s->peers) p->S.compact_seg = s->S.compact_seg;
  return RT_OK;
}

int ppm_set_batching(ppm_scene* s, long long slot_bytes, long long max_updates) {
  if (!s || slot_bytes < 0 || max_updates < 0)
    return set_error(RT_E_INVALID, "ppm_set_batching: bad argument");
  s->slot_bytes = (size_t)slot_bytes;
  s->max_updates = max_updates ? std::min<long long>(max_updates, INT_MAX) : INT_MAX;
  for (auto& p : s->peers) p->slot_bytes = s->slot_bytes, p->max_updates = s->max_updates;
  return RT_OK;
}

int ppm_set_seed(ppm_scene* s, unsigned long long seed) {
  if (!s) return set_error(RT_E_INVALID, "ppm_set_seed: NULL scene");
  s->seed = seed;
  for (auto& p : s->peers) p->seed = seed;
  return RT_OK;
}

int ppm_eye_pass(ppm_scene* s, int cam) {
  return guarded([&] {
    check_scene(s);
    each_replica(s, [&](ppm_scene* r) {
      eye_pass(r, cam);
      hip_check(hipStreamSynchronize(r->stream), "eye pass");
    });
    return RT_OK;
  });
}

int ppm_build_hash_grid(ppm_scene* s, int width, int height, double* info) {
  return guarded([&] {
    check_scene(s);
    if (width <= 0 || height <= 0) throw std::invalid_argument("bad image size");
    each_replica(s, [&](ppm_scene* r) {
      build_grid(r, width, height);
      hip_check(hipStreamSynchronize(r->stream), "build hash grid");
    });
    s->merged = true;
    DeviceGuard g(s->device);
    PGrid G;
    hip_check(hipMemcpyAsync(&G, s->grid.p, sizeof G, hipMemcpyDeviceToHost, s->stream), "read grid");
    hip_check(hipStreamSynchronize(s->stream), "build hash grid");
    if (info) {
      const double v[8] = {G.radius, G.hash_scale, G.bmin[0], G.bmin[1], G.bmin[2],
                           G.bmax[0], G.bmax[1], G.bmax[2]};
      std::memcpy(info, v, sizeof v);
    }
    return RT_OK;
  });
}

int ppm_num_hit_points(const ppm_scene* s) { return s ? s->n_hp : 0; }

int ppm_read_hit_points(ppm_scene* s, float* out) {
  return guarded([&] {
    check_scene(s);
    if (!out) throw std::invalid_argument("ppm_read_hit_points: NULL output");
    merge_peers(s);
    DeviceGuard g(s->device);
    std::vector<PHitPoint> hp(s->n_hp);
    std::vector<float4> st(s->n_hp);
    if (s->n_hp) {
      hip_check(hipMemcpyAsync(hp.data(), s->hp.p, hp.size() * sizeof(PHitPoint),
                               hipMemcpyDeviceToHost, s->stream), "read hit points");
      if (s->grid_ready)
        hip_check(hipMemcpyAsync(st.data(), s->state.p, st.size() * sizeof(float4),
                                 hipMemcpyDeviceToHost, s->stream), "read hit-point state");
      hip_check(hipStreamSynchronize(s->stream), "read hit points");
    }
    for (int k = 0; k < s->n_hp; k++) {
      const PHitPoint& h = hp[k];
      float* r = out + 16 * (size_t)k;
      std::memcpy(r, h.pos, 12);
      std::memcpy(r + 3, h.normal, 12);
      std::memcpy(r + 6, h.w_o, 12);
      std::memcpy(r + 9, h.att, 12);
      r[12] = (float)h.pixel;
      r[13] = h.weight;
      r[14] = s->grid_ready ? st[k].w : 0.0f;
      r[15] = (float)s->host.materials[h.material].type;
    }
    return RT_OK;
  });
}

int ppm_read_hit_state(ppm_scene* s, float* out) {
  return guarded([&] {
    check_scene(s);
    if (!out) throw std::invalid_argument("ppm_read_hit_state: NULL output");
    if (!s->grid_ready) throw std::invalid_argument("no hash grid yet");
    merge_peers(s);
    DeviceGuard g(s->device);
    std::vector<float4> st(s->n_hp);
    std::vector<unsigned> n(s->n_hp);
    if (s->n_hp) {
      hip_check(hipMemcpyAsync(st.data(), s->state.p, st.size() * sizeof(float4),
                               hipMemcpyDeviceToHost, s->stream), "read state");
      hip_check(hipMemcpyAsync(n.data(), s->nupd.p, n.size() * sizeof(unsigned),
                               hipMemcpyDeviceToHost, s->stream), "read counts");
      hip_check(hipStreamSynchronize(s->stream), "read state");
    }
    for (int k = 0; k < s->n_hp; k++) {
      float* r = out + 5 * (size_t)k;
      r[0] = st[k].x, r[1] = st[k].y, r[2] = st[k].z, r[3] = st[k].w, r[4] = (float)n[k];
    }
    return RT_OK;
  });
}

int ppm_trace_photons(ppm_scene* s, long long first, long long count) {
  return guarded([&] {
    check_scene(s);
    each_replica(s, [&](ppm_scene* r) { trace_photons(r, first, count); });
    if (!s->peers.empty()) s->merged = false;
    if (s->peers.empty() && s->shards > 1) s->shard_partial = true;
    return RT_OK;
  });
}

int ppm_density_estimation(ppm_scene* s, long long total, float* out) {
  return guarded([&] {
    check_scene(s);
    if (!out) throw std::invalid_argument("ppm_density_estimation: NULL output");
    if (s->shard_partial)
      throw std::invalid_argument("ppm_density_estimation: update shard " + std::to_string(s->shard) +
                                  " of " + std::to_string(s->shards) +
                                  " holds only its own hit points; write the merged state "
                                  "(ppm_write_hit_state) first");
    merge_peers(s);
    DeviceGuard g(s->device);
    density(s, total, out);
    return RT_OK;
  });
}

int ppm_collect_stats(ppm_scene* s, ppm_stats* st) {
  return guarded([&] {
    check_scene(s);
    if (!st) throw std::invalid_argument("ppm_collect_stats: NULL output");
    collect_all(s, st);
    return RT_OK;
  });
}

int ppm_render(ppm_scene* s, int cam, int threads, float* out, ppm_stats* stats) {
  return guarded([&] {
    check_scene(s);
    if (threads < 1 || !out) throw std::invalid_argument("ppm_render: bad argument");
    if (cam < 0 || cam >= (int)s->host.cameras.size())
      throw std::invalid_argument("camera index out of range");
    if (s->peers.empty() && s->shards > 1)
      throw std::invalid_argument("ppm_render: the scene applies only update shard " +
                                  std::to_string(s->shard) + " of " + std::to_string(s->shards) +
                                  " (ppm_set_update_shard); reset it to 0 of 1 or render the "
                                  "passes and merge the shards' states");
    DeviceGuard g(s->device);
    const PCamera& C = s->host.cameras[cam].cam;
    hipEvent_t ev[5];
    for (auto& e : ev) hip_check(hipEventCreate(&e), "event");
    struct Events {
      hipEvent_t* e;
      ~Events() {
        for (int k = 0; k < 5; k++) (void)hipEventDestroy(e[k]);
      }
    } guard{ev};
    // a multi-device scene runs each pass on every replica (update pass sharded), then
    // gathers the hit-point state onto replica 0 for the density estimation
    each_replica(s, [&](ppm_scene* r) {
      hip_check(hipMemsetAsync(r->stats.p, 0, kStatSlots * sizeof(unsigned long long), r->stream),
                "zero counters");
      r->photons = 0;
      r->drop_update_events();
    });
    hip_check(hipEventRecord(ev[0], s->stream), "event");
    each_replica(s, [&](ppm_scene* r) { eye_pass(r, cam); });
    hip_check(hipEventRecord(ev[1], s->stream), "event");
    each_replica(s, [&](ppm_scene* r) { build_grid(r, C.width, C.height); });
    s->merged = true;
    hip_check(hipEventRecord(ev[2], s->stream), "event");
    const long long P = s->host.per_iteration, I = s->host.iterations;
    const long long per_thread = P / threads;
    const long long traced = C.height < threads ? P * I : per_thread * I * threads;
    each_replica(s, [&](ppm_scene* r) { trace_photons(r, 0, traced); });
    if (!s->peers.empty()) s->merged = false;
    hip_check(hipEventRecord(ev[3], s->stream), "event");
    merge_peers(s);
    const int normalizer = (int)(P * per_thread * threads);  // main.cpp:94, int arithmetic
    density(s, normalizer, out);
    hip_check(hipEventRecord(ev[4], s->stream), "event");
    hip_check(hipEventSynchronize(ev[4]), "render");
    if (stats) {
      const long long photons = s->photons;
      ppm_collect_stats(s, stats);
      stats->photons = photons;
      float ms[4];
      for (int k = 0; k < 4; k++) hip_check(hipEventElapsedTime(&ms[k], ev[k], ev[k + 1]), "elapsed");
      stats->eye_ms = ms[0], stats->grid_ms = ms[1], stats->photon_ms = ms[2], stats->density_ms = ms[3];
    }
    return RT_OK;
  });
}

int ppm_write_png(const char* path, const float* rgb, int w, int h) {
  if (!path || !rgb || w <= 0 || h <= 0) return set_error(RT_E_INVALID, "ppm_write_png: bad argument");
  return guarded([&] {
    std::vector<float> v((size_t)w * h * 3);
    for (size_t k = 0; k < v.size(); k++)  // main.cpp:148-154: double exp / pow
      v[k] = (float)(int)(std::pow(1 - std::exp(-(double)rgb[k]), (double)(1 / 2.2f)) * 255 + 0.5f);
    rt::write_png(path, v.data(), w, h);
    return RT_OK;
  });
}

}  // extern "C"
