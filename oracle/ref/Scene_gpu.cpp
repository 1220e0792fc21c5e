// ORACLE TEST INFRASTRUCTURE — the reference-side binding of INTEGRATION.md §2, compiled and
// run (oracle/Makefile target `binding`).  This is the file a maintainer would add to HW2 as
// HW2/Scene_gpu.cpp: the reference's own Scene (parsed by its tinyxml2 loader, its objects and
// its BVH built by BVH::create_bvh) is handed to libceng795_rt.so as an rt_scene_desc with the
// reference's BVH walked through its public members (ABI 7: bvh_*), and render_image_gpu
// replaces Scene::render_image (HW2/Scene.h:34-35, HW2/Scene.cpp:16-31).  The library's own XML
// loader is not used.
//
// What the Scene does not expose: Camera keeps e / top_left / s_u / s_v private
// (HW2/Camera.h:56-62), so each camera's Position / Gaze / Up are read from the same XML with the
// reference's tinyxml2 and the reference's stream semantics (HW2/Scene.cpp:239-283), and
// rt_camera_from_view applies Camera.h:19-28; everything else of the camera (image plane,
// per-axis sample count) comes from the Camera object.
#include <algorithm>
#include <array>
#include <cstring>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "Pixel.h"
#include "Scene.h"
#include "ceng795_rt.h"
#include "tinyxml2.h"

static rt_scene* g_rt = nullptr;
// One page-locked frame buffer, the size of the largest camera, allocated with the scene
// (rt_host_alloc, outside the reference's timed region like the Scene ctor): rt_render writes it
// from the frame kernel directly, with no device-to-host copy; the reference's threads render
// disjoint rows of it.
static float* g_frame = nullptr;

namespace {

void put3(float* d, const Vector3& v) {
  d[0] = v.x;
  d[1] = v.y;
  d[2] = v.z;
}

// The reference's BVH in DFS preorder (left first), Mesh wrappers spliced out
// (Mesh::intersect delegates to its bvh, HW2/Mesh.h:13-15).
struct TreeWalk {
  const Scene& scene;
  std::vector<int> children;
  std::vector<float> boxes;
  std::vector<int> leaf_kind, leaf_index;  // 0 triangle / 1 sphere, index in its list
  std::vector<float> leaf_normals;
  std::vector<int> tri_idx, tri_mat, sph_center, sph_mat;
  std::vector<float> sph_radius;

  explicit TreeWalk(const Scene& s) : scene(s) {}

  int vertex_of(const Vector3& c) const {  // the vertex a Sphere's center was copied from
    for (size_t i = 0; i < scene.vertex_data.size(); i++) {
      const Vector3& v = scene.vertex_data[i];
      if (!std::memcmp(&v.x, &c.x, 4) && !std::memcmp(&v.y, &c.y, 4) && !std::memcmp(&v.z, &c.z, 4))
        return (int)i;
    }
    throw std::runtime_error("sphere center is no vertex of the scene");
  }

  int leaf(int kind, int index, const Vector3& n) {
    leaf_kind.push_back(kind);
    leaf_index.push_back(index);
    leaf_normals.insert(leaf_normals.end(), {n.x, n.y, n.z});
    return ~(int)(leaf_kind.size() - 1);
  }

  int visit(const Shape* sh) {
    while (const Mesh* m = dynamic_cast<const Mesh*>(sh)) sh = m->bvh;
    if (const BVH* b = dynamic_cast<const BVH*>(sh)) {
      const int node = (int)(children.size() / 2);
      children.insert(children.end(), {0, 0});
      float box[6];
      put3(box, b->bounding_box.min_corner);
      put3(box + 3, b->bounding_box.max_corner);
      boxes.insert(boxes.end(), box, box + 6);
      const int l = visit(b->left);
      const int r = visit(b->right);
      children[2 * node] = l;
      children[2 * node + 1] = r;
      return node;
    }
    if (const Triangle* t = dynamic_cast<const Triangle*>(sh)) {
      tri_idx.insert(tri_idx.end(), {t->index_0, t->index_1, t->index_2});
      tri_mat.push_back(t->material_id);
      return leaf(0, (int)tri_mat.size() - 1, t->normal);
    }
    if (const Sphere* s = dynamic_cast<const Sphere*>(sh)) {
      sph_center.push_back(vertex_of(s->center));
      sph_radius.push_back(s->radius);
      sph_mat.push_back(s->material_id);
      return leaf(1, (int)sph_mat.size() - 1, Vector3(0.0f));
    }
    throw std::runtime_error("unknown Shape in the reference BVH");
  }
};

// Position / Gaze / Up of every camera, as HW2/Scene.cpp:239-283 reads them.
std::vector<std::array<float, 9>> camera_views(const char* xml) {
  tinyxml2::XMLDocument doc;
  if (doc.LoadFile(xml)) throw std::runtime_error(std::string("cannot parse ") + xml);
  const tinyxml2::XMLNode* root = doc.FirstChild();
  std::vector<std::array<float, 9>> out;
  std::stringstream stream;
  const tinyxml2::XMLElement* e =
      root->FirstChildElement("Cameras")->FirstChildElement("Camera");
  for (; e; e = e->NextSiblingElement("Camera")) {
    std::array<float, 9> v{};
    for (const char* tag : {"Position", "Gaze", "Up"}) stream << e->FirstChildElement(tag)->GetText() << std::endl;
    for (float& x : v) stream >> x;
    out.push_back(v);
  }
  return out;
}

}  // namespace

void gpu_scene_open(const Scene& scene, const char* xml, int devices) {
  rt_scene_desc d;
  std::memset(&d, 0, sizeof d);
  put3(d.background, scene.background_color);
  d.shadow_ray_epsilon = scene.shadow_ray_epsilon;
  d.max_recursion_depth = scene.max_recursion_depth;
  put3(d.ambient_light, scene.ambient_light);
  std::vector<float> verts(3 * scene.vertex_data.size());
  for (size_t i = 0; i < scene.vertex_data.size(); i++) put3(&verts[3 * i], scene.vertex_data[i]);
  d.vertices = verts.data();
  d.num_vertices = (int)scene.vertex_data.size();
  std::vector<rt_material> mats(scene.materials.size());
  for (size_t i = 0; i < mats.size(); i++) {
    const Material& m = scene.materials[i];
    put3(mats[i].ambient, m.ambient);
    put3(mats[i].diffuse, m.diffuse);
    put3(mats[i].specular, m.specular);
    put3(mats[i].mirror, m.mirror);
    put3(mats[i].transparency, m.transparency);
    mats[i].refraction_index = m.refraction_index;
    mats[i].phong_exponent = m.phong_exponent;
  }
  d.materials = mats.data();
  d.num_materials = (int)mats.size();
  std::vector<rt_point_light> lights(scene.point_lights.size());
  for (size_t i = 0; i < lights.size(); i++) {
    put3(lights[i].position, scene.point_lights[i].position);
    put3(lights[i].intensity, scene.point_lights[i].intensity);
  }
  d.lights = lights.data();
  d.num_lights = (int)lights.size();
  const auto views = camera_views(xml);
  if (views.size() != scene.cameras.size()) throw std::runtime_error("camera count mismatch");
  std::vector<rt_camera> cams(scene.cameras.size());
  for (size_t c = 0; c < cams.size(); c++) {
    const Image_plane& ip = scene.cameras[c].get_image_plane();
    const float np[4] = {ip.left, ip.right, ip.bottom, ip.top};
    if (rt_camera_from_view(&views[c][0], &views[c][3], &views[c][6], np, ip.distance, ip.width,
                            ip.height, scene.cameras[c].get_number_of_samples(), &cams[c]) != RT_OK)
      throw std::runtime_error(rt_last_error());
  }
  d.cameras = cams.data();
  d.num_cameras = (int)cams.size();

  TreeWalk w(scene);
  const int root = w.visit(scene.bvh);
  (void)root;  // node 0, or ~0 when the root is one primitive
  d.num_triangles = (int)w.tri_mat.size();
  d.triangle_indices = w.tri_idx.data();
  d.triangle_material = w.tri_mat.data();
  d.num_spheres = (int)w.sph_mat.size();
  d.sphere_center = w.sph_center.data();
  d.sphere_radius = w.sph_radius.data();
  d.sphere_material = w.sph_mat.data();
  std::vector<int> leaf_object(w.leaf_kind.size());
  for (size_t k = 0; k < leaf_object.size(); k++)
    leaf_object[k] = w.leaf_kind[k] == 0 ? w.leaf_index[k] : d.num_triangles + w.leaf_index[k];
  d.bvh_num_nodes = (int)(w.children.size() / 2);
  d.bvh_children = w.children.data();
  d.bvh_boxes = w.boxes.data();
  d.bvh_num_leaves = (int)leaf_object.size();
  d.bvh_leaf_object = leaf_object.data();
  d.bvh_leaf_normals = w.leaf_normals.data();

  const int rc = devices > 1 ? rt_scene_create_multi(&d, devices, nullptr, &g_rt)
                             : rt_scene_create(&d, /*device=*/-1, &g_rt);
  if (rc != RT_OK) throw std::runtime_error(rt_last_error());
  size_t floats = 1;
  for (const rt_camera& c : cams) floats = std::max(floats, (size_t)c.width * c.height * 3);
  g_frame = static_cast<float*>(rt_host_alloc(floats * sizeof(float)));
  if (!g_frame) throw std::runtime_error(rt_last_error());
}

void gpu_scene_close() {
  rt_host_free(g_frame);
  g_frame = nullptr;
  rt_scene_destroy(g_rt);
  g_rt = nullptr;
}

// Same contract as Scene::render_image: rows starting_row, starting_row + height_increase, ...
// of `result` receive Pixel::add_color(color, 1) (HW2/Scene.cpp:25-31, Pixel.h:12-16).
void render_image_gpu(const Scene& scene, int camera_index, Pixel* result, int starting_row,
                      int height_increase) {
  const Image_plane& ip = scene.cameras[camera_index].get_image_plane();
  float* rgb = g_frame;
  if (rt_render(g_rt, camera_index, starting_row, height_increase, rgb, nullptr) != RT_OK)
    throw std::runtime_error(rt_last_error());
  for (int j = starting_row; j < ip.height; j += height_increase)
    for (int i = 0; i < ip.width; i++) {
      const float* c = &rgb[3 * ((size_t)j * ip.width + i)];
      result[j * ip.width + i].add_color(Vector3(c[0], c[1], c[2]), 1);
    }
}
