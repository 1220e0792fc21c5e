// Scene XML ingest — the host side the north star keeps.  Mirrors HW2/Scene.cpp:198-451:
// the same tags, defaults and 1-based index conversion, and — so every fp32 value gets the
// reference's bits — the same parsing mechanism: all text goes through ONE std::stringstream
// and `operator>>` (libstdc++ num_get -> strtof), as the reference does.
//
// The reference parses with tinyxml2 6.1.0 (vendored at HW2/tinyxml2.*); we use our own DOM
// reader (xml_dom.h).
#include <locale.h>

#include <cctype>
#include <cerrno>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>
#include <stdexcept>

#include "host_scene.h"
#include "xml_dom.h"

namespace rt {
namespace {

// ---- fast path for the two bulk lists (VertexData, Faces).  operator>> on a float is
// libstdc++ num_get -> strtof in the "C" locale; on an int, strtol + range check.  For text
// that is nothing but whitespace-separated plain decimal tokens (optional '-', digits, optional
// fraction, optional exponent) in complete triples, the loop `while (!(ss >> x).eof())` reads
// exactly those tokens, so calling strtof_l / strtol directly gives the same bits at a fraction
// of the cost.  Anything else (a '+', "inf", a partial triple, a token strtof would stop
// inside) takes the stream path unchanged.
locale_t c_locale() {
  static locale_t loc = newlocale(LC_ALL_MASK, "C", (locale_t)0);
  return loc;
}
bool is_ws(char c) { return c == ' ' || c == '\n' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }
bool plain_number(const char* b, const char* e, bool integer) {
  const char* p = b;
  if (p < e && *p == '-') p++;
  int digits = 0;
  while (p < e && *p >= '0' && *p <= '9') p++, digits++;
  if (integer) return digits > 0 && p == e;
  if (p < e && *p == '.') {
    p++;
    while (p < e && *p >= '0' && *p <= '9') p++, digits++;
  }
  if (digits == 0) return false;
  if (p < e && (*p == 'e' || *p == 'E')) {
    p++;
    if (p < e && (*p == '+' || *p == '-')) p++;
    int ed = 0;
    while (p < e && *p >= '0' && *p <= '9') p++, ed++;
    if (ed == 0) return false;
  }
  return p == e;
}
// Parses `text` as whitespace-separated numbers; false = not eligible (use the stream).
bool fast_floats(const std::string& text, std::vector<float>& out) {
  std::vector<float> v;
  const char* p = text.c_str();
  const char* end = p + text.size();
  while (true) {
    while (p < end && is_ws(*p)) p++;
    if (p == end) break;
    const char* b = p;
    while (p < end && !is_ws(*p)) p++;
    if (!plain_number(b, p, false)) return false;
    errno = 0;
    char* stop = nullptr;
    const float f = strtof_l(b, &stop, c_locale());
    if (stop != p || errno == ERANGE) return false;
    v.push_back(f);
  }
  if (v.size() % 3) return false;
  out.insert(out.end(), v.begin(), v.end());
  return true;
}
bool fast_ints(const std::string& text, std::vector<int>& out, int delta) {
  std::vector<int> v;
  const char* p = text.c_str();
  const char* end = p + text.size();
  while (true) {
    while (p < end && is_ws(*p)) p++;
    if (p == end) break;
    const char* b = p;
    while (p < end && !is_ws(*p)) p++;
    if (!plain_number(b, p, true) || p - b > 11) return false;
    errno = 0;
    char* stop = nullptr;
    const long x = std::strtol(b, &stop, 10);
    if (stop != p || errno == ERANGE || x < INT_MIN || x > INT_MAX) return false;
    v.push_back((int)x + delta);
  }
  if (v.size() % 3) return false;
  out.insert(out.end(), v.begin(), v.end());
  return true;
}
// The shared stream holds nothing but whitespace before its next read.
bool stream_drained(std::stringstream& ss) {
  const std::streampos g = ss.tellg();
  if (g < 0) return false;
  const std::string& all = ss.str();
  for (size_t i = (size_t)g; i < all.size(); i++)
    if (!is_ws(all[i])) return false;
  return true;
}

// HW7's binary lists (HW7/src/Scene.cpp:1839-1904): int32 N, then N float triples (vertices)
// or N int32 triples (faces).  The path is used as given (fopen, like the reference); a
// relative path that does not open is retried next to the scene file.
FILE* open_beside(const std::string& name, const std::string& scene_path) {
  FILE* f = std::fopen(name.c_str(), "rb");
  if (!f && !name.empty() && name[0] != '/') {
    const size_t slash = scene_path.find_last_of('/');
    if (slash != std::string::npos) f = std::fopen((scene_path.substr(0, slash + 1) + name).c_str(), "rb");
  }
  if (!f) throw std::ios_base::failure("cannot open binary list " + name);
  return f;
}
template <typename T>
void read_binary_triples(const std::string& name, const std::string& scene_path, std::vector<T>& out,
                         T delta) {
  FILE* f = open_beside(name, scene_path);
  int n = 0;
  if (std::fread(&n, sizeof n, 1, f) != 1 || n < 0) {
    std::fclose(f);
    throw std::runtime_error("scene xml: truncated binary list " + name);
  }
  const size_t base = out.size();
  out.resize(base + 3 * (size_t)n);
  const size_t got = std::fread(out.data() + base, sizeof(T), 3 * (size_t)n, f);
  std::fclose(f);
  if (got != 3 * (size_t)n) throw std::runtime_error("scene xml: truncated binary list " + name);
  if (delta != T(0))
    for (size_t i = base; i < out.size(); i++) out[i] += delta;
}

}  // namespace

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

  // <ZeroBasedIndexing>true</ZeroBasedIndexing> applies to binary face lists (HW7 Scene.cpp:515-522)
  bool zero_based = false;
  if (const Node* z = root->first("ZeroBasedIndexing"))
    zero_based = z->has_text && std::string(z->text) == "true";
  const Node* vd = root->first("VertexData");
  if (vd && vd->attr("binaryFile")) {  // HW7 format (f4)
    read_binary_triples<float>(vd->attr("binaryFile"), path, st.vertices, 0.0f);
  } else {
    const char* vtext = node_text(vd, "VertexData");
    if (!(stream_drained(ss) && fast_floats(vtext, st.vertices))) {
      ss << vtext << std::endl;
      float x, y, z;
      while (!(ss >> x).eof()) {  // HW2/Scene.cpp:372-375
        ss >> y >> z;
        st.vertices.insert(st.vertices.end(), {x, y, z});
      }
    }
  }
  ss.clear();

  const Node* objs = root->first("Objects");
  if (!objs) throw std::runtime_error("scene xml: missing <Objects>");
  for (const Node* m : objs->each("Mesh")) {
    int mat;
    ss << node_text(m->first("Material"), "Material") << std::endl;
    ss >> mat;
    const Node* faces = m->first("Faces");
    int count = 0;
    const size_t before = st.mesh_faces.size();
    if (faces && faces->attr("binaryFile")) {  // HW7 format (f4), HW7 Scene.cpp:1866-1904
      const int offset = faces->int_attr("vertexOffset", 0);
      read_binary_triples<int>(faces->attr("binaryFile"), path, st.mesh_faces,
                               (zero_based ? 0 : -1) + offset);
      count = (int)((st.mesh_faces.size() - before) / 3);
    } else {
      const char* ftext = node_text(faces, "Faces");
      if (stream_drained(ss) && fast_ints(ftext, st.mesh_faces, -1)) {
        count = (int)((st.mesh_faces.size() - before) / 3);
      } else {
        ss << ftext << std::endl;
        int a, b, c;
        while (!(ss >> a).eof()) {  // HW2/Scene.cpp:394-398
          ss >> b >> c;
          st.mesh_faces.insert(st.mesh_faces.end(), {a - 1, b - 1, c - 1});
          ++count;
        }
      }
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
