// `ppm_render [--gpus N] <scene.xml> [threads]` — the host driver of PPM/src/main.cpp:21-160 on
// top of the photon-mapping C ABI: for every <Camera>, the eye pass, hash grid, photon pass and
// density estimation (with the photon budget and normaliser the reference uses on `threads` host
// threads, default 8), then the default tone curve and <ImageName> (extension replaced by .png).
// --gpus N: one multi-device scene over GPUs 0..N-1 (update pass sharded by hit point).
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/ceng795_ppm.h"

int main(int argc, char** argv) {
  int gpus = 0, arg = 1;
  if (argc > 2 && std::string(argv[1]) == "--gpus") {
    gpus = std::atoi(argv[2]);
    arg = 3;
  }
  if (argc <= arg) {
    std::fprintf(stderr, "Please provide scene file as argument\n");
    return 1;
  }
  const int threads = argc > arg + 1 ? std::atoi(argv[arg + 1]) : 8;
  ppm_scene* scene = nullptr;
  std::vector<int> devices;
  for (int d = 0; d < gpus; d++) devices.push_back(d);
  const int rc = gpus > 0 ? ppm_scene_load_xml_multi(argv[arg], gpus, devices.data(), &scene)
                          : ppm_scene_load_xml(argv[arg], 0, &scene);
  if (rc != RT_OK) {
    std::fprintf(stderr, "%s\n", ppm_last_error());
    return 1;
  }
  std::printf("Scene is parsed\n");
  int status = 0;
  for (int c = 0; c < ppm_num_cameras(scene); c++) {
    int w, h, n;
    ppm_camera_info(scene, c, &w, &h, &n);
    std::vector<float> rgb((size_t)w * h * 3);
    ppm_stats st;
    if (ppm_render(scene, c, threads, rgb.data(), &st) != RT_OK) {
      std::fprintf(stderr, "render failed: %s\n", ppm_last_error());
      status = 1;
      continue;
    }
    std::printf("Eye pass is completed in: %.3f ms\n", st.eye_ms);
    std::printf("Building hash grid is completed in: %.3f ms\n", st.grid_ms);
    std::printf("Tracing photon rays is completed in: %.3f ms (%lld photons, %.1f Mphotons/s)\n",
                st.photon_ms, st.photons, st.photons / (st.photon_ms * 1e3));
    std::printf("Density estimation is completed in: %.3f ms\n", st.density_ms);
    std::string name = ppm_image_name(scene, c);
    name = name.substr(0, name.find_last_of('.')) + ".png";  // main.cpp:108-110
    if (ppm_write_png(name.c_str(), rgb.data(), w, h) != RT_OK) {
      std::printf("encoder error: %s\n", ppm_last_error());
      status = 1;
    } else {
      std::printf("Saved png file. [ %s ]\n", name.c_str());
    }
  }
  ppm_scene_destroy(scene);
  return status;
}
