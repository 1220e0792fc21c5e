// ORACLE TEST INFRASTRUCTURE — never shipped, never measured as the product.
//
// Probe harness linked against the UNMODIFIED reference PPM sources, compiled where they lie
// under /root/reference/PPM by oracle/Makefile (`make ref-ppm`, output oracle/_ref/ppm_harness).
// It drives only the public reference API, in the order PPM/src/main.cpp:21-107 does for one
// camera:
//   Scene::Scene(xml)                                   PPM/src/Scene.cpp:373
//   reset_hash_grid / eye_trace_lines (T threads)       Scene.cpp:46, 250; main.cpp:36-52
//   build_hash_grid(w, h)                               Scene.cpp:53; main.cpp:61
//   trace_n_photons(P/T, I) on T threads                Scene.cpp:95; main.cpp:72-90
//   density_estimation(pixels, P*(P/T)*T)               Scene.cpp:363; main.cpp:93-95
//   Pixel::get_color                                    PPM/include/Pixel.h:19-28
//
// Commands:
//   render    <xml> <cam> <out.f32> <threads> [iterations] [photons_per_iteration]
//             float RGB (get_color), w*h*3; prints one JSON line (phase times, counts)
//   hitpoints <xml> <cam> <out.f32>
//             single-threaded eye pass + build_hash_grid; per hit point 16 floats
//             {position, normal, w_o, attenuation, pixel, pixel_weight, radius_squared,
//              material_type}; prints one JSON line (count, hash scale, grid bbox)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <thread>
#include <vector>

#include "Pixel.h"
#include "Scene.h"

static double seconds_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

static void write_floats(const char* path, const std::vector<float>& v) {
  std::ofstream f(path, std::ios::binary);
  f.write(reinterpret_cast<const char*>(v.data()), v.size() * sizeof(float));
}

int main(int argc, char** argv) {
  if (argc < 5) {
    std::cerr << "usage: ppm_harness render|hitpoints <xml> <cam> <out> ..." << std::endl;
    return 2;
  }
  const std::string cmd = argv[1];
  std::streambuf* saved = std::cout.rdbuf();
  std::ostringstream quiet;  // the loader prints progress lines; keep stdout for our JSON
  std::cout.rdbuf(quiet.rdbuf());
  Scene scene(argv[2]);
  std::cout.rdbuf(saved);
  const int cam = std::atoi(argv[3]);
  const Camera& camera = scene.cameras[cam];
  const int width = camera.get_image_plane().width;
  const int height = camera.get_image_plane().height;
  scene.reset_hash_grid();

  if (cmd == "hitpoints") {
    scene.eye_trace_lines(cam, 0, 1);
    scene.build_hash_grid(width, height);
    std::vector<float> out;
    for (const Hit_point* h : scene.hit_points) {
      const float rec[16] = {h->position.x, h->position.y, h->position.z, h->normal.x,
                             h->normal.y, h->normal.z, h->w_o.x, h->w_o.y, h->w_o.z,
                             h->attenuation.x, h->attenuation.y, h->attenuation.z,
                             (float)h->pixel, h->pixel_weight, h->radius_squared,
                             (float)h->material.material_type};
      out.insert(out.end(), rec, rec + 16);
    }
    write_floats(argv[4], out);
    const Bounding_box& b = scene.hit_point_bbox;
    std::printf("{\"hit_points\": %zu, \"num_hash\": %u, \"hash_scale\": %.9g, "
                "\"bbox_min\": [%.9g, %.9g, %.9g], \"bbox_max\": [%.9g, %.9g, %.9g]}\n",
                scene.hit_points.size(), scene.num_hash, scene.hash_scale, b.min_corner.x,
                b.min_corner.y, b.min_corner.z, b.max_corner.x, b.max_corner.y,
                b.max_corner.z);
    return 0;
  }
  if (cmd != "render" || argc < 6) return 2;
  const int thread_count = std::max(1, std::atoi(argv[5]));
  if (argc > 6 && std::atoi(argv[6]) > 0) scene.number_of_iterations = std::atoi(argv[6]);
  if (argc > 7 && std::atoi(argv[7]) > 0) scene.photon_count_per_iteration = std::atoi(argv[7]);

  auto t0 = std::chrono::steady_clock::now();
  if (height < thread_count) {
    scene.eye_trace_lines(cam, 0, 1);
  } else {
    std::vector<std::thread> pool;
    for (int i = 0; i < thread_count; i++)
      pool.emplace_back(&Scene::eye_trace_lines, &scene, cam, i, thread_count);
    for (auto& t : pool) t.join();
  }
  const double eye_s = seconds_since(t0);

  t0 = std::chrono::steady_clock::now();
  scene.build_hash_grid(width, height);
  const double grid_s = seconds_since(t0);

  const int iterations = scene.number_of_iterations;
  const int per_iteration = scene.photon_count_per_iteration;
  const int photons_per_thread = per_iteration / thread_count;
  long long traced = 0;
  t0 = std::chrono::steady_clock::now();
  if (height < thread_count) {
    scene.trace_n_photons(per_iteration, iterations);
    traced = (long long)per_iteration * iterations;
  } else {
    std::vector<std::thread> pool;
    for (int i = 0; i < thread_count; i++)
      pool.emplace_back(&Scene::trace_n_photons, &scene, photons_per_thread, iterations);
    for (auto& t : pool) t.join();
    traced = (long long)photons_per_thread * iterations * thread_count;
  }
  const double photon_s = seconds_since(t0);

  std::vector<Pixel> pixels((size_t)width * height);
  const int normalizer = per_iteration * photons_per_thread * thread_count;
  t0 = std::chrono::steady_clock::now();
  scene.density_estimation(pixels.data(), normalizer);
  const double density_s = seconds_since(t0);

  std::vector<float> out((size_t)width * height * 3);
  for (size_t i = 0; i < pixels.size(); i++) {
    const Vector3 c = pixels[i].get_color();
    out[3 * i] = c.x;
    out[3 * i + 1] = c.y;
    out[3 * i + 2] = c.z;
  }
  write_floats(argv[4], out);
  std::printf("{\"threads\": %d, \"photons_traced\": %lld, \"normalizer\": %d, "
              "\"hit_points\": %zu, \"eye_s\": %.6f, \"grid_s\": %.6f, \"photon_s\": %.6f, "
              "\"density_s\": %.6f, \"photons_per_s\": %.1f}\n",
              thread_count, traced, normalizer, scene.hit_points.size(), eye_s, grid_s,
              photon_s, density_s, traced / photon_s);
  return 0;
}
