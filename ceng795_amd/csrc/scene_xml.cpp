// Scene XML ingest — the host side the north star keeps.  Mirrors HW2/Scene.cpp:198-451:
// the same tags, defaults and 1-based index conversion, and — so every fp32 value gets the
// reference's bits — the same parsing mechanism: all text goes through ONE std::stringstream
// and `operator>>` (libstdc++ num_get -> strtof), as the reference does.
//
// The reference parses with tinyxml2 6.1.0 (vendored at HW2/tinyxml2.*); we use our own DOM
// reader (xml_dom.h).
#include <cctype>
#include <cmath>
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>
#include <stdexcept>

#include "host_scene.h"
#include "xml_dom.h"

namespace rt {

void load_scene_xml(const std::string& path, XmlSceneStorage& st, rt_scene_desc& d) {
  const std::unique_ptr<Node> root = parse_xml_file(path);

  std::stringstream ss;  // one shared stream, as HW2/Scene.cpp:200
  auto put = [&](const Node* n, const char* what, const char* fallback) {
    if (n) ss << node_text(n, what) << std::endl;
    else ss << fallback << std::endl;
  };
  float bg[3];
  put(root->first("BackgroundColor"), "BackgroundColor", "0 0 0");
  ss >> bg[0] >> bg[1] >> bg[2];
  float eps;
  put(root->first("ShadowRayEpsilon"), "ShadowRayEpsilon", "0.001");
  ss >> eps;
  int depth;
  put(root->first("MaxRecursionDepth"), "MaxRecursionDepth", "0");
  ss >> depth;

  const Node* cams = root->first("Cameras");
  if (!cams) throw std::runtime_error("scene xml: missing <Cameras>");
  for (const Node* c : cams->each("Camera")) {
    ss << node_text(c->first("Position"), "Position") << std::endl;
    ss << node_text(c->first("Gaze"), "Gaze") << std::endl;
    ss << node_text(c->first("Up"), "Up") << std::endl;
    ss << node_text(c->first("NearPlane"), "NearPlane") << std::endl;
    ss << node_text(c->first("NearDistance"), "NearDistance") << std::endl;
    ss << node_text(c->first("ImageResolution"), "ImageResolution") << std::endl;
    put(c->first("NumSamples"), "NumSamples", "1");
    ss << node_text(c->first("ImageName"), "ImageName") << std::endl;
    float pos[3], gaze[3], up[3], np[4], dist;
    int w, h, ns;
    std::string name;
    ss >> pos[0] >> pos[1] >> pos[2] >> gaze[0] >> gaze[1] >> gaze[2] >> up[0] >> up[1] >> up[2];
    ss >> np[0] >> np[1] >> np[2] >> np[3] >> dist >> w >> h >> ns;
    ns = (int)std::sqrt((double)ns);  // HW2/Scene.cpp:275-276
    if (ns <= 0) ns = 1;
    ss >> name;
    rt_camera cam;
    camera_from_view(pos, gaze, up, np, dist, w, h, ns, cam);
    st.cameras.push_back(cam);
    st.image_names.push_back(name);
  }

  const Node* lights = root->first("Lights");
  if (!lights) throw std::runtime_error("scene xml: missing <Lights>");
  float amb[3];
  ss << node_text(lights->first("AmbientLight"), "AmbientLight") << std::endl;
  ss >> amb[0] >> amb[1] >> amb[2];
  for (const Node* pl : lights->each("PointLight")) {
    ss << node_text(pl->first("Position"), "Position") << std::endl;
    ss << node_text(pl->first("Intensity"), "Intensity") << std::endl;
    rt_point_light L;
    ss >> L.position[0] >> L.position[1] >> L.position[2];
    ss >> L.intensity[0] >> L.intensity[1] >> L.intensity[2];
    st.lights.push_back(L);
  }

  const Node* mats = root->first("Materials");
  if (!mats) throw std::runtime_error("scene xml: missing <Materials>");
  for (const Node* m : mats->each("Material")) {
    put(m->first("AmbientReflectance"), "AmbientReflectance", "0 0 0");
    put(m->first("DiffuseReflectance"), "DiffuseReflectance", "0 0 0");
    put(m->first("SpecularReflectance"), "SpecularReflectance", "0 0 0");
    put(m->first("MirrorReflectance"), "MirrorReflectance", "0 0 0");
    put(m->first("PhongExponent"), "PhongExponent", "1");
    put(m->first("Transparency"), "Transparency", "0 0 0");
    put(m->first("RefractionIndex"), "RefractionIndex", "1.0");
    rt_material M;
    for (float* v : {M.ambient, M.diffuse, M.specular, M.mirror}) ss >> v[0] >> v[1] >> v[2];
    ss >> M.phong_exponent;
    ss >> M.transparency[0] >> M.transparency[1] >> M.transparency[2];
    ss >> M.refraction_index;
    st.materials.push_back(M);
  }

  ss << node_text(root->first("VertexData"), "VertexData") << std::endl;
  float x, y, z;
  while (!(ss >> x).eof()) {  // HW2/Scene.cpp:372-375
    ss >> y >> z;
    st.vertices.insert(st.vertices.end(), {x, y, z});
  }
  ss.clear();

  const Node* objs = root->first("Objects");
  if (!objs) throw std::runtime_error("scene xml: missing <Objects>");
  for (const Node* m : objs->each("Mesh")) {
    int mat;
    ss << node_text(m->first("Material"), "Material") << std::endl;
    ss >> mat;
    ss << node_text(m->first("Faces"), "Faces") << std::endl;
    int a, b, c, count = 0;
    while (!(ss >> a).eof()) {  // HW2/Scene.cpp:394-398
      ss >> b >> c;
      st.mesh_faces.insert(st.mesh_faces.end(), {a - 1, b - 1, c - 1});
      ++count;
    }
    ss.clear();
    st.mesh_material.push_back(mat - 1);
    st.mesh_face_count.push_back(count);
  }
  ss.clear();
  for (const Node* t : objs->each("Triangle")) {
    int mat, a, b, c;
    ss << node_text(t->first("Material"), "Material") << std::endl;
    ss >> mat;
    ss << node_text(t->first("Indices"), "Indices") << std::endl;
    ss >> a >> b >> c;
    st.triangle_indices.insert(st.triangle_indices.end(), {a - 1, b - 1, c - 1});
    st.triangle_material.push_back(mat - 1);
  }
  for (const Node* s : objs->each("Sphere")) {
    int mat, center;
    float radius;
    ss << node_text(s->first("Material"), "Material") << std::endl;
    ss >> mat;
    ss << node_text(s->first("Center"), "Center") << std::endl;
    ss >> center;
    ss << node_text(s->first("Radius"), "Radius") << std::endl;
    ss >> radius;
    st.sphere_material.push_back(mat - 1);
    st.sphere_center.push_back(center - 1);
    st.sphere_radius.push_back(radius);
  }

  d = rt_scene_desc{};
  std::memcpy(d.background, bg, sizeof bg);
  d.shadow_ray_epsilon = eps;
  d.max_recursion_depth = depth;
  std::memcpy(d.ambient_light, amb, sizeof amb);
  d.vertices = st.vertices.data();
  d.num_vertices = (int)(st.vertices.size() / 3);
  d.materials = st.materials.data();
  d.num_materials = (int)st.materials.size();
  d.lights = st.lights.data();
  d.num_lights = (int)st.lights.size();
  d.cameras = st.cameras.data();
  d.num_cameras = (int)st.cameras.size();
  d.num_meshes = (int)st.mesh_material.size();
  d.mesh_material = st.mesh_material.data();
  d.mesh_face_count = st.mesh_face_count.data();
  d.mesh_faces = st.mesh_faces.data();
  d.num_triangles = (int)st.triangle_material.size();
  d.triangle_indices = st.triangle_indices.data();
  d.triangle_material = st.triangle_material.data();
  d.num_spheres = (int)st.sphere_material.size();
  d.sphere_center = st.sphere_center.data();
  d.sphere_radius = st.sphere_radius.data();
  d.sphere_material = st.sphere_material.data();
}

}  // namespace rt
