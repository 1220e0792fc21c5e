// ORACLE TEST INFRASTRUCTURE — HW2's driver with the two-line patch of INTEGRATION.md §2:
// the reference's Scene parses the XML and builds its BVH, gpu_scene_open hands that Scene (its
// objects and its own BVH, walked through public members) to libceng795_rt.so, render_image_gpu
// (oracle/ref/Scene_gpu.cpp) fills the reference's Pixel array, and the reference's own Pixel::get_color +
// lodepng::encode write the PNG named by <ImageName> (HW2/main.cpp:17-57).  Linked against the
// UNMODIFIED reference HW2 sources by oracle/Makefile (`make -C oracle binding`).
//
//   hw2_gpu <scene.xml> [--threads T] [--gpus N] [--dump PREFIX]
//
// --threads T: T host threads, thread i on rows i, i+T, ... (HW2/main.cpp:33-36 kept: the
// library call is reentrant); default 1 call on every row.  --gpus N: the scene over N GPUs of
// this process.  --dump PREFIX: also writes each camera's Pixel::color as fp32 RGB, row-major
// (PREFIX_cam<i>.f32), for the tests' comparison with the reference's frame hashes.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <thread>
#include <vector>

#include "Pixel.h"
#include "Scene.h"
#include "lodepng/lodepng.h"

void gpu_scene_open(const Scene& scene, const char* xml, int devices);
void gpu_scene_close();
void render_image_gpu(const Scene& scene, int camera_index, Pixel* result, int starting_row,
                      int height_increase);

int main(int argc, char* argv[]) {
  if (argc < 2) {
    std::cerr << "usage: hw2_gpu <scene.xml> [--threads T] [--gpus N] [--dump PREFIX]\n";
    return 1;
  }
  int threads = 1, gpus = 1;
  std::string dump;
  for (int a = 2; a + 1 < argc; a += 2) {
    if (!std::strcmp(argv[a], "--threads")) threads = std::atoi(argv[a + 1]);
    else if (!std::strcmp(argv[a], "--gpus")) gpus = std::atoi(argv[a + 1]);
    else if (!std::strcmp(argv[a], "--dump")) dump = argv[a + 1];
  }
  try {
    Scene scene(argv[1]);
    gpu_scene_open(scene, argv[1], gpus);
    for (size_t cam = 0; cam < scene.cameras.size(); cam++) {
      const Camera& camera = scene.cameras[cam];
      const int w = camera.get_image_plane().width, h = camera.get_image_plane().height;
      std::vector<Pixel> pixels((size_t)w * h);
      const auto t0 = std::chrono::steady_clock::now();
      if (threads <= 1 || h < threads) {
        render_image_gpu(scene, (int)cam, pixels.data(), 0, 1);
      } else {
        std::vector<std::thread> pool;
        for (int i = 0; i < threads; i++)
          pool.emplace_back(render_image_gpu, std::cref(scene), (int)cam, pixels.data(), i, threads);
        for (auto& t : pool) t.join();
      }
      const double ms = std::chrono::duration<double, std::milli>(
                            std::chrono::steady_clock::now() - t0).count();
      if (!dump.empty()) {
        const std::string path = dump + "_cam" + std::to_string(cam) + ".f32";
        FILE* f = std::fopen(path.c_str(), "wb");
        if (!f) throw std::runtime_error("cannot write " + path);
        for (const Pixel& p : pixels) std::fwrite(&p.color.x, sizeof(float), 3, f);
        std::fclose(f);
      }
      // HW2/main.cpp:43-57: Pixel::get_color (truncate, clamp), alpha 255, lodepng::encode
      std::vector<unsigned char> rgba((size_t)w * h * 4);
      for (size_t k = 0; k < pixels.size(); k++) {
        const Vector3i c = pixels[k].get_color();
        rgba[4 * k] = (unsigned char)c.x;
        rgba[4 * k + 1] = (unsigned char)c.y;
        rgba[4 * k + 2] = (unsigned char)c.z;
        rgba[4 * k + 3] = 255;
      }
      const unsigned err = lodepng::encode(camera.get_filename().c_str(), rgba.data(), w, h);
      if (err) {
        std::cerr << "encoder error " << err << ": " << lodepng_error_text(err) << "\n";
        return 2;
      }
      std::cout << camera.get_filename() << " (" << w << "x" << h << ") in " << ms << " ms\n";
    }
    gpu_scene_close();
  } catch (const std::exception& e) {
    std::cerr << "error: " << e.what() << "\n";
    return 3;
  }
  return 0;
}
