// `raytracer [--gpus N] [--reference-traversal] <scene.xml>` — the host driver of
// HW2/main.cpp:10-70 on top of the C ABI: parse the scene, then for every <Camera> render
// (timed), quantise and write <ImageName>.  The reference spawns hardware_concurrency()
// threads on render_image (main.cpp:33-36); here one rt_render call renders every row on the
// GPU, or with --gpus N on N GPUs of the node (rt_scene_load_xml_multi: tiles dealt over the
// devices, RCCL gather onto the first).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/ceng795_rt.h"

int main(int argc, char** argv) {
  int mode = RT_TRAVERSAL_FAST, gpus = 0;
  const char* xml = nullptr;
  for (int i = 1; i < argc; i++) {
    const std::string a = argv[i];
    if (a == "--reference-traversal") {
      mode = RT_TRAVERSAL_REFERENCE;
    } else if (a == "--gpus" && i + 1 < argc) {
      gpus = std::atoi(argv[++i]);
    } else {
      xml = argv[i];
    }
  }
  if (!xml) {
    std::fprintf(stderr, "Please provide scene file as argument\n");
    return 1;
  }
  rt_scene* scene = nullptr;
  const int rc = gpus > 0 ? rt_scene_load_xml_multi(xml, gpus, nullptr, &scene)
                          : rt_scene_load_xml(xml, -1, &scene);
  if (rc != RT_OK) {
    std::fprintf(stderr, "%s\n", rt_last_error());
    return 1;
  }
  rt_set_traversal(scene, mode);
  std::printf("Scene is parsed\n");
  const int cameras = rt_scene_num_cameras(scene);
  int status = 0;
  for (int c = 0; c < cameras; c++) {
    rt_camera cam;
    rt_scene_camera(scene, c, &cam);
    std::vector<float> rgb((size_t)cam.width * cam.height * 3, 0.0f);
    std::printf("Starting rendering on %d GPU(s)\n", rt_scene_device_count(scene));
    const auto t0 = std::chrono::steady_clock::now();
    rt_stats st;
    if (rt_render(scene, c, 0, 1, rgb.data(), &st) != RT_OK) {
      std::fprintf(stderr, "render failed: %s\n", rt_last_error());
      status = 1;
      continue;
    }
    const auto t1 = std::chrono::steady_clock::now();
    const std::string name = rt_scene_image_name(scene, c);
    if (rt_write_png(name.c_str(), rgb.data(), cam.width, cam.height) != RT_OK) {
      std::printf("encoder error: %s\n", rt_last_error());
      status = 1;
    }
    const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    std::printf("%s(%dx%d) is saved in: %.3f ms (kernel %.3f ms, %.1f Mrays/s)\n", name.c_str(),
                cam.width, cam.height, ms, st.kernel_ms,
                (st.primary_rays + st.shadow_rays + st.secondary_rays) / (st.kernel_ms * 1e3));
  }
  rt_scene_destroy(scene);
  return status;
}
