/* ceng795_ppm.h — C ABI of the MI355X progressive-photon-mapping path (BASELINE config C5).
 *
 * Replaces the reference's PPM Scene passes (PPM/include/Scene.h:44-56, PPM/src/Scene.cpp):
 *   Scene::Scene(xml)                       -> ppm_scene_load_xml             (Scene.cpp:373)
 *   reset_hash_grid + eye_trace_lines       -> ppm_eye_pass                   (Scene.cpp:46, 250)
 *   build_hash_grid(width, height)          -> ppm_build_hash_grid            (Scene.cpp:53)
 *   trace_n_photons(n, iterations)          -> ppm_trace_photons              (Scene.cpp:95)
 *   density_estimation(pixels, total)       -> ppm_density_estimation         (Scene.cpp:363)
 *   main.cpp:30-104 for one camera          -> ppm_render
 * The reference runs these on T host threads (main.cpp:36-90); here each is one or a few HIP
 * launches.  Hit points, the hash grid and the photon deposits stay in device memory.
 *
 * Results are those of the reference run on ONE thread (pixels row-major, photons in order,
 * each photon's hit-point updates applied before the next photon's), with two documented
 * substitutions for the reference's non-reproducible parts: random numbers come from a
 * per-photon SplitMix64 stream (seed, photon index) instead of random_device-seeded mt19937,
 * and sinf/cosf/asinf/powf are correctly rounded (ceng795_amd/csrc/ppm_math.h).  The photon
 * sequence is therefore a pure function of (scene, seed, photon index range).
 *
 * Error codes are the RT_E* values of ceng795_rt.h; messages via ppm_last_error().
 */
#ifndef CENG795_PPM_H_
#define CENG795_PPM_H_
#include "ceng795_rt.h"
#ifdef __cplusplus
extern "C" {
#endif

#define CENG795_PPM_ABI_VERSION 6  /* 2: ppm_set_batching; 3: update-pass work in ppm_stats;
                                     4: tile-list compaction (setter + counters); 5: compaction
                                     segment length, counters per segment; 6: multi-device
                                     scenes, update-pass shards, hit-state write */

typedef struct ppm_scene ppm_scene;

typedef struct ppm_stats {
  long long photons;      /* photons emitted                                     */
  long long photon_rays;  /* photon segments traced (closest-hit queries)        */
  long long deposits;     /* diffuse photon hits (hash-cell lookups)             */
  long long updates;      /* hit-point radius / flux updates applied             */
  long long eye_rays;     /* eye-pass closest-hit queries                        */
  long long hit_points;
  double eye_ms, grid_ms, photon_ms, density_ms;  /* device time of each pass (ppm_render) */
  /* the update pass (Scene.cpp:131-168) as the GPU runs it: (hit-point tile, deposit) pairs its
   * filter examined, candidates it passed to the exact recurrence, and the device time of its
   * kernel summed over the photon batches since the last collection */
  long long update_deposit_visits, update_candidates, update_launches;
  double update_ms;
  /* list segments (of ppm_set_update_segment deposits) that compacted tiles copied before
   * their windows (ppm_set_update_compaction), segments whose copy did not fit the tile's
   * scratch range (they ran over the segment itself), and the deposits the copies kept */
  long long update_compacted_segments, update_compaction_fallbacks, update_compacted_deposits;
} ppm_stats;

int ppm_abi_version(void);
const char* ppm_last_error(void);

/* PPM/src/Scene.cpp:373-505 (+ Camera / Material / Transformation / Point_light / Sphere /
 * Mesh loaders) and the BVH builds; uploads to HIP device `device`. */
int ppm_scene_load_xml(const char* xml_path, int device, ppm_scene** out);
void ppm_scene_destroy(ppm_scene* scene);
int ppm_num_cameras(const ppm_scene* scene);
int ppm_camera_info(const ppm_scene* scene, int camera, int* width, int* height,
                    int* num_samples);
const char* ppm_image_name(const ppm_scene* scene, int camera);
/* PhotonCountPerIteration, NumberOfIterations, MaxRecursionDepth (Scene.cpp:388-430). */
int ppm_settings(const ppm_scene* scene, int* per_iteration, int* iterations, int* max_depth);
int ppm_set_seed(ppm_scene* scene, unsigned long long seed);

/* Photon-pass batching (no effect on results: a batch of photons is traced, its deposits
 * sorted and applied in photon order, then the next batch).  slot_bytes: device memory for
 * one batch's deposit slots (19 x 48 B per photon at MaxRecursionDepth 20); 0 = the default
 * (16 GiB, or CENG795_PPM_SLOT_MB), always capped at a quarter of the free device memory.
 * max_updates: (hit-point group, deposit) pairs one batch may expand to (0 = 2^31 - 1, the
 * limit of the 32-bit sort); a batch that would exceed it is traced again as two halves. */
int ppm_set_batching(ppm_scene* scene, long long slot_bytes, long long max_updates);
/* Update-pass tile-list compaction (no effect on results): a hit-point tile whose group's
 * deposit list holds at least min_list deposits first copies, in photon order, the deposits
 * within the radius its hit points have when the pass starts, then streams that copy.
 * min_list: -1 = the default (65536, or CENG795_PPM_COMPACT), 0 = off. */
int ppm_set_update_compaction(ppm_scene* scene, long long min_list);
/* Segment length of that compaction (no effect on results): a compacted tile takes its list
 * in segments of seg_len deposits, each copied with the radii its hit points have at the
 * segment's start, into a scratch range of seg_len / 4.  0 = the default (32768). */
int ppm_set_update_segment(ppm_scene* scene, int seg_len);
/* reset_hash_grid + eye_trace_lines over all rows: builds the hit points. */
int ppm_eye_pass(ppm_scene* scene, int camera);
/* build_hash_grid; info8 (nullable) receives {initial radius, hash scale, grid bbox min xyz,
 * max xyz}. */
int ppm_build_hash_grid(ppm_scene* scene, int width, int height, double* info8);
int ppm_num_hit_points(const ppm_scene* scene);
/* 16 floats per hit point: position, normal, w_o, attenuation, pixel, pixel_weight,
 * radius_squared, material type (the layout oracle/_ref/ppm_harness `hitpoints` writes). */
int ppm_read_hit_points(ppm_scene* scene, float* out16);
/* 5 floats per hit point: flux xyz, radius_squared, n. */
int ppm_read_hit_state(ppm_scene* scene, float* out5);
/* Photons [first, first + count) of the scene's photon sequence (trace_n_photons). */
int ppm_trace_photons(ppm_scene* scene, long long first, long long count);
/* density_estimation(pixels, total) + Pixel::get_color into out_rgb (w*h*3, host memory). */
int ppm_density_estimation(ppm_scene* scene, long long total_num_of_photons, float* out_rgb);

/* main.cpp:30-104 for one camera with the photon budget and normaliser the reference uses on
 * `reference_threads` host threads: traces T*(P/T)*I photons (P*I when height < T) and
 * normalises by P*(P/T)*T (main.cpp:74, 94).  Synchronous; stats nullable. */
int ppm_render(ppm_scene* scene, int camera, int reference_threads, float* out_rgb,
               ppm_stats* stats);
/* Reads (and resets) the device counters of the passes run since the last call.  On a
 * multi-device scene the photon / eye counts are replica 0's (every replica traces the whole
 * sequence), the update-pass work is summed over the replicas and update_ms is the longest
 * replica's. */
int ppm_collect_stats(ppm_scene* scene, ppm_stats* stats);

/* ---- several GPUs ("PPM photons shard freely, but the hit-point flux state is
 * shared").  The reference's T threads share every hit point under a mutex
 * (PPM/src/Scene.cpp:131-168, PPM/include/Hit_point.h:22).  Here the update pass is split by
 * hit point instead: the grid's update tiles (hit points of one hash-cell range, <= 5 each)
 * are dealt round-robin over S shards, a shard applies the complete photon-order recurrence
 * of its own hit points, and the shards' results are merged by hit point.  Results are
 * bit-identical to the one-device scene for any S. */

/* One process over several GPUs: replica d (on devices[d]) runs the eye pass, grid and the
 * whole photon sequence, and the update pass of shard d of device_count; density estimation,
 * ppm_read_hit_state and ppm_read_hit_points first gather the replicas' hit-point state onto
 * devices[0] (device-to-device copies + a merge kernel).  The same device may be listed more
 * than once.  Every other call of this header accepts the scene and fans out to the replicas
 * (passes run concurrently, one host thread per replica). */
int ppm_scene_load_xml_multi(const char* xml_path, int device_count, const int* devices,
                             ppm_scene** out);
int ppm_scene_device_count(const ppm_scene* scene);
/* One process per GPU: this scene applies only the update tiles of shard `shard` of
 * `shards` (0 <= shard < shards; 0 of 1 = all, the default).  Takes effect at the next
 * ppm_build_hash_grid (call it again).  Not for multi-device scenes, which shard themselves. */
int ppm_set_update_shard(ppm_scene* scene, int shard, int shards);
/* The shard owning each hit point (ppm_num_hit_points ints), after ppm_build_hash_grid. */
int ppm_hit_point_shards(ppm_scene* scene, int* out);
/* Overwrites the hit-point state with 5 floats per hit point (the ppm_read_hit_state layout:
 * flux xyz, radius_squared, n) — e.g. the merge of the shards' states before
 * ppm_density_estimation.  After ppm_build_hash_grid.  n travels as float32, so it must be a
 * whole number <= 2^24 (RT_E_INVALID otherwise); n sets rr(n) of later updates.
 * A scene with shards > 1 that has traced photons holds only its own hit points' results:
 * ppm_density_estimation refuses it until this call has written the merged state, and
 * ppm_render refuses such a scene outright. */
int ppm_write_hit_state(ppm_scene* scene, const float* in5);

/* main.cpp:142-156 (no tone-mapping operator): c -> int(pow(1 - exp(-c), 1/2.2f)*255 + 0.5f),
 * clamped to [0, 255], RGBA8 PNG. */
int ppm_write_png(const char* path, const float* rgb, int width, int height);

#ifdef __cplusplus
}
#endif
#endif
