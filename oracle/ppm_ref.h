/* ORACLE TEST INFRASTRUCTURE — CPU restatement of the reference's progressive photon
 * mapping path (PPM/src/Scene.cpp, PPM/src/main.cpp).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / CPU baseline — never as the product path.
 *
 * It restates the reference sequentially: one thread, pixels in row-major order (each
 * pixel's eye-ray tree depth first, reflection before refraction), photons in index order,
 * every photon applying its hit-point updates before the next photon starts — i.e. the
 * reference run on one thread.  The random numbers come from ppm_math::Rng (one stream per
 * photon / per eye sample, see ceng795_amd/csrc/ppm_math.h) instead of random_device-seeded
 * mt19937 generators, and sinf/cosf/asinf/powf from ppm_math (correctly rounded) instead of
 * glibc's; everything else follows the reference's fp32 operation order.
 *
 * Parity pinning (tests/test_ppm_oracle.py): the eye pass and hash grid are deterministic in
 * the reference and are compared bit for bit with oracle/_ref/ppm_harness (compiled from the
 * unmodified /root/reference/PPM sources); the photon pass is stochastic in the reference and
 * is pinned statistically against independent reference renders (tests/golden/).
 */
#ifndef CENG795_ORACLE_PPM_REF_H_
#define CENG795_ORACLE_PPM_REF_H_
#ifdef __cplusplus
extern "C" {
#endif

typedef struct ppmref_scene ppmref_scene;

typedef struct ppmref_stats {
  long long photons;          /* photons emitted                                  */
  long long photon_rays;      /* photon segments traced (closest-hit queries)     */
  long long deposits;         /* diffuse photon hits (hash-cell lookups)          */
  long long updates;          /* hit-point radius/flux updates applied            */
  long long eye_rays;         /* eye-pass closest-hit queries                     */
  long long hit_points;
} ppmref_stats;

ppmref_scene* ppmref_load(const char* xml_path, char* err, int errlen);
void ppmref_free(ppmref_scene* s);
int ppmref_num_cameras(const ppmref_scene* s);
int ppmref_camera_info(const ppmref_scene* s, int cam, int* width, int* height, int* samples);
/* PhotonCountPerIteration, NumberOfIterations, MaxRecursionDepth (PPM/src/Scene.cpp:388-430) */
int ppmref_settings(const ppmref_scene* s, int* per_iteration, int* iterations, int* max_depth);

/* reset_hash_grid + eye_trace_lines over every row (Scene.cpp:46, 250-285). */
int ppmref_eye_pass(ppmref_scene* s, int cam, unsigned long long seed, ppmref_stats* st);
/* build_hash_grid (Scene.cpp:53-93).  info6 (may be NULL): initial radius, hash scale,
 * bbox min xyz ... written as doubles: {r0, scale, minx, miny, minz, maxx, maxy, maxz}. */
int ppmref_build_hash_grid(ppmref_scene* s, int width, int height, double* info8);
int ppmref_num_hit_points(const ppmref_scene* s);
/* 16 floats per hit point, ppm_harness `hitpoints` layout: position, normal, w_o,
 * attenuation, pixel, pixel_weight, radius_squared, material_type. */
int ppmref_hit_points(const ppmref_scene* s, float* out16);
/* 5 floats per hit point: flux xyz, radius_squared, n. */
int ppmref_hit_state(const ppmref_scene* s, float* out5);
/* Photons [first, first+count) of the photon sequence (trace_n_photons, Scene.cpp:95-104). */
int ppmref_trace_photons(ppmref_scene* s, unsigned long long seed, long long first,
                         long long count, ppmref_stats* st);
/* analysis only (tools/ppm_list_study.py): the same photons, logging deposits and updates */
long long ppmref_trace_photons_logged(ppmref_scene* s, unsigned long long seed, long long first,
                                      long long count, float* dep8, long long dep_cap,
                                      long long* upd2, long long upd_cap, long long* n_upd);
/* density_estimation (Scene.cpp:363-371) + Pixel::get_color: out w*h*3. */
int ppmref_density(const ppmref_scene* s, long long total_num_of_photons, float* out_rgb);

/* main.cpp:30-104 for one camera, as the reference run on `threads` host threads would
 * count: traces threads*(P/threads)*I photons and normalises by P*(P/threads)*threads. */
int ppmref_render(ppmref_scene* s, int cam, unsigned long long seed, int threads,
                  float* out_rgb, ppmref_stats* st);

/* ppm_math pieces, exported for the accuracy test against libm. */
float ppmref_sinf(float x);
float ppmref_cosf(float x);
float ppmref_asinf(float x);
float ppmref_powf(float x, float y);

#ifdef __cplusplus
}
#endif
#endif
