// ORACLE TEST INFRASTRUCTURE — never shipped, never measured as the product.
//
// Probe harness linked against the UNMODIFIED reference HW2 sources, compiled where they
// lie under /root/reference/HW2 by oracle/Makefile (output: oracle/_ref/ref_harness).
// It only drives public reference API:
//   * Scene::Scene(xml)                        HW2/Scene.cpp:198
//   * Scene::render_image(cam, Pixel*, s, k)   HW2/Scene.cpp:16 (row-interleaved, as main.cpp:33-36)
//   * Pixel::color (public fp32 radiance)      HW2/Pixel.h:10
//   * BVH::left/right/bounding_box, Mesh::bvh, Triangle::index_*, Sphere::center/radius
//     (HW2/Bounding_volume_hierarchy.h:39-41, Mesh.h:12, Triangle.h:12-14, Sphere.h:12-14)
//   * Camera::calculate_ray_at + scene.bvh->intersect for hit / ray counts (Camera.h:30).
//
// Commands:
//   render <xml> <cam> <out.f32> [threads]          float RGB, w*h*3, row-major, top row first
//   resolved <xml> <cam> <out.f32> [threads]        Pixel::color / Pixel::weight (what
//                                                   get_color truncates; MSAA cameras)
//   bvh    <xml> <out.txt>                          preorder BVH topology, floats as hex bits
//   rays   <xml> <cam> <out.bin>                    per-pixel primary hit: t, normal (hex) + hit flag
//   time   <xml> <cam> <threads> <reps> <row_step> [warm]  median wall time of render_image
//          over rows, after `warm` untimed renders
//                                                   j = 0 (mod row_step); prints one JSON line
//   png    <xml> <cam> <out.png> [threads]          the reference's own output file: Pixel::
//                                                   get_color() + alpha 255 -> lodepng::encode
//                                                   (HW2/main.cpp:43-57, HW2/lodepng 20180114)
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <thread>
#include <vector>

#include "Bounding_volume_hierarchy.h"
#include "lodepng/lodepng.h"
#include "Mesh.h"
#include "Pixel.h"
#include "Scene.h"
#include "Sphere.h"
#include "Triangle.h"

static unsigned bits(float f) {
  unsigned u;
  std::memcpy(&u, &f, 4);
  return u;
}

static void render_rows(const Scene& scene, int cam, Pixel* px, int first_row, int row_step,
                        int threads) {
  const int h = scene.cameras[cam].get_image_plane().height;
  const int stride = row_step * threads;
  if (threads <= 1 || h < threads) {
    scene.render_image(cam, px, first_row, row_step);
    return;
  }
  std::vector<std::thread> pool;
  for (int i = 0; i < threads; i++)
    pool.emplace_back(&Scene::render_image, &scene, cam, px, first_row + i * row_step, stride);
  for (auto& t : pool) t.join();
}

static void dump_shape(const Shape* s, std::ostream& os) {
  if (const BVH* b = dynamic_cast<const BVH*>(s)) {
    const Bounding_box& bb = b->bounding_box;
    char buf[160];
    std::snprintf(buf, sizeof buf, "N %08x %08x %08x %08x %08x %08x\n", bits(bb.min_corner.x),
                  bits(bb.min_corner.y), bits(bb.min_corner.z), bits(bb.max_corner.x),
                  bits(bb.max_corner.y), bits(bb.max_corner.z));
    os << buf;
    dump_shape(b->left, os);
    dump_shape(b->right, os);
  } else if (const Mesh* m = dynamic_cast<const Mesh*>(s)) {
    os << "M\n";
    dump_shape(m->bvh, os);
  } else if (const Triangle* t = dynamic_cast<const Triangle*>(s)) {
    os << "T " << t->index_0 << " " << t->index_1 << " " << t->index_2 << " "
       << t->get_material_id() << "\n";
  } else if (const Sphere* sp = dynamic_cast<const Sphere*>(s)) {
    char buf[160];
    std::snprintf(buf, sizeof buf, "S %08x %08x %08x %08x %d\n", bits(sp->center.x),
                  bits(sp->center.y), bits(sp->center.z), bits(sp->radius),
                  sp->get_material_id());
    os << buf;
  } else {
    os << "?\n";
  }
}

// rays = W*H primary + one shadow ray per light for every primary hit (depth-0 scenes),
// counted over the rows j = first (mod step).  Matches SURVEY §8(d)'s definition.
static long long count_rays(const Scene& scene, int cam, int first_row, int row_step) {
  const Camera& c = scene.cameras[cam];
  const int w = c.get_image_plane().width, h = c.get_image_plane().height;
  long long rays = 0;
  for (int j = first_row; j < h; j += row_step)
    for (int i = 0; i < w; i++) {
      Hit_data hd;
      hd.t = std::numeric_limits<float>::infinity();
      hd.shape = NULL;
      rays++;
      if (scene.bvh->intersect(c.calculate_ray_at(i, j), hd))
        rays += (long long)scene.point_lights.size();
    }
  return rays;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::cerr << "usage: ref_harness render|bvh|rays|time ..." << std::endl;
    return 2;
  }
  const std::string cmd = argv[1];
  Scene scene(argv[2]);
  if (cmd == "render" || cmd == "resolved") {
    const int cam = std::atoi(argv[3]);
    const int threads = argc > 5 ? std::atoi(argv[5]) : (int)std::thread::hardware_concurrency();
    const Image_plane& ip = scene.cameras[cam].get_image_plane();
    const int w = ip.width, h = ip.height;
    Pixel* px = new Pixel[(size_t)w * h];
    render_rows(scene, cam, px, 0, 1, threads);
    std::vector<float> out((size_t)w * h * 3);
    for (size_t i = 0; i < (size_t)w * h; i++) {
      const float w = cmd == "resolved" ? px[i].weight : 1.0f;
      out[3 * i + 0] = cmd == "resolved" ? px[i].color.x / w : px[i].color.x;
      out[3 * i + 1] = cmd == "resolved" ? px[i].color.y / w : px[i].color.y;
      out[3 * i + 2] = cmd == "resolved" ? px[i].color.z / w : px[i].color.z;
    }
    std::ofstream f(argv[4], std::ios::binary);
    f.write(reinterpret_cast<const char*>(out.data()), out.size() * sizeof(float));
    delete[] px;
  } else if (cmd == "png") {
    const int cam = std::atoi(argv[3]);
    const int threads = argc > 5 ? std::atoi(argv[5]) : (int)std::thread::hardware_concurrency();
    const Image_plane& ip = scene.cameras[cam].get_image_plane();
    const int w = ip.width, h = ip.height;
    Pixel* px = new Pixel[(size_t)w * h];
    render_rows(scene, cam, px, 0, 1, threads);
    std::vector<unsigned char> image((size_t)w * h * 4);
    size_t idx = 0;
    for (int j = 0; j < h; j++)
      for (int i = 0; i < w; i++) {
        const Vector3i p = px[(size_t)j * w + i].get_color();
        image[idx++] = (unsigned char)p.x;
        image[idx++] = (unsigned char)p.y;
        image[idx++] = (unsigned char)p.z;
        image[idx++] = 255;
      }
    delete[] px;
    const unsigned err = lodepng::encode(argv[4], image.data(), (unsigned)w, (unsigned)h);
    if (err) {
      std::cerr << "lodepng error " << err << std::endl;
      return 1;
    }
  } else if (cmd == "bvh") {
    std::ofstream f(argv[3]);
    dump_shape(scene.bvh, f);
  } else if (cmd == "rays") {
    const int cam = std::atoi(argv[3]);
    const Camera& c = scene.cameras[cam];
    const int w = c.get_image_plane().width, h = c.get_image_plane().height;
    std::ofstream f(argv[4], std::ios::binary);
    for (int j = 0; j < h; j++)
      for (int i = 0; i < w; i++) {
        Hit_data hd;
        hd.t = std::numeric_limits<float>::infinity();
        hd.shape = NULL;
        const Ray r = c.calculate_ray_at(i, j);
        const bool hit = scene.bvh->intersect(r, hd);
        float rec[8] = {r.d.x, r.d.y, r.d.z, hit ? hd.t : 0.f, hit ? hd.normal.x : 0.f,
                        hit ? hd.normal.y : 0.f, hit ? hd.normal.z : 0.f, hit ? 1.f : 0.f};
        f.write(reinterpret_cast<const char*>(rec), sizeof rec);
      }
  } else if (cmd == "time") {
    const int cam = std::atoi(argv[3]);
    const int threads = std::atoi(argv[4]);
    const int reps = std::atoi(argv[5]);
    const int row_step = std::atoi(argv[6]);
    const Image_plane& ip = scene.cameras[cam].get_image_plane();
    const int w = ip.width, h = ip.height;
    const int warm = argc > 7 ? std::atoi(argv[7]) : 0;  // untimed warm renders first
    std::vector<double> times;
    for (int r = 0; r < warm + reps; r++) {
      Pixel* px = new Pixel[(size_t)w * h];
      auto t0 = std::chrono::steady_clock::now();
      render_rows(scene, cam, px, 0, row_step, threads);
      auto t1 = std::chrono::steady_clock::now();
      if (r >= warm) times.push_back(std::chrono::duration<double>(t1 - t0).count());
      delete[] px;
    }
    std::sort(times.begin(), times.end());
    const long long rays = count_rays(scene, cam, 0, row_step);
    std::printf("{\"seconds_median\": %.6f, \"seconds_min\": %.6f, \"rays\": %lld, "
                "\"threads\": %d, \"row_step\": %d, \"width\": %d, \"height\": %d}\n",
                times[times.size() / 2], times[0], rays, threads, row_step, w, h);
  } else {
    std::cerr << "unknown command " << cmd << std::endl;
    return 2;
  }
  return 0;
}
