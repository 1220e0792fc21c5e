// `raytracer <scene.xml>` — the host driver of HW2/main.cpp:10-70 on top of the C ABI:
// parse the scene, then for every <Camera> render (timed), quantise and write <ImageName>.
// The reference spawns hardware_concurrency() threads on render_image (main.cpp:33-36); here
// one rt_render call renders every row on the GPU.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/ceng795_rt.h"

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "Please provide scene file as argument\n");
    return 1;
  }
  const int mode = (argc > 2 && std::string(argv[2]) == "--reference-traversal")
                       ? RT_TRAVERSAL_REFERENCE
                       : RT_TRAVERSAL_FAST;
  rt_scene* scene = nullptr;
  if (rt_scene_load_xml(argv[1], -1, &scene) != RT_OK) {
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
    std::printf("Starting rendering on the GPU\n");
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
