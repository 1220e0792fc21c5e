// ORACLE TEST INFRASTRUCTURE — the reference-side binding of INTEGRATION.md §2, compiled and
// run (oracle/Makefile target `binding`).  This is the file a maintainer would add to HW2 as
// HW2/Scene_gpu.cpp: it keeps the reference's own Scene (cameras, image names, the Pixel array
// and the PNG step of HW2/main.cpp) and renders through libceng795_rt.so instead of
// Scene::render_image (HW2/Scene.h:34-35, HW2/Scene.cpp:16-31).
#include <stdexcept>
#include <vector>

#include "Pixel.h"
#include "Scene.h"
#include "ceng795_rt.h"

// Loaded once next to the reference Scene (same XML file).  devices > 1: the same scene on
// that many GPUs of this process (rt_scene_load_xml_multi).
static rt_scene* g_rt = nullptr;

void gpu_scene_open(const char* xml, int devices) {
  const int rc = devices > 1 ? rt_scene_load_xml_multi(xml, devices, nullptr, &g_rt)
                             : rt_scene_load_xml(xml, /*device=*/-1, &g_rt);
  if (rc != RT_OK) throw std::runtime_error(rt_last_error());
}

void gpu_scene_close() {
  rt_scene_destroy(g_rt);
  g_rt = nullptr;
}

// Same contract as Scene::render_image: rows starting_row, starting_row + height_increase, ...
// of `result` receive Pixel::add_color(color, 1) (HW2/Scene.cpp:25-31, Pixel.h:12-16).
void render_image_gpu(const Scene& scene, int camera_index, Pixel* result, int starting_row,
                      int height_increase) {
  const Image_plane& ip = scene.cameras[camera_index].get_image_plane();
  std::vector<float> rgb((size_t)ip.width * ip.height * 3);
  if (rt_render(g_rt, camera_index, starting_row, height_increase, rgb.data(), nullptr) != RT_OK)
    throw std::runtime_error(rt_last_error());
  for (int j = starting_row; j < ip.height; j += height_increase)
    for (int i = 0; i < ip.width; i++) {
      const float* c = &rgb[3 * ((size_t)j * ip.width + i)];
      result[j * ip.width + i].add_color(Vector3(c[0], c[1], c[2]), 1);
    }
}
