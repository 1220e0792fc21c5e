// Scene XML ingest — the host side the north star keeps.  Mirrors HW2/Scene.cpp:198-451:
// the same tags, defaults and 1-based index conversion, and — so every fp32 value gets the
// reference's bits — the same parsing mechanism: all text goes through ONE std::stringstream
// and `operator>>` (libstdc++ num_get -> strtof), as the reference does.
//
// The reference parses with tinyxml2 6.1.0 (vendored at HW2/tinyxml2.*).  This is a small
// DOM reader of our own covering what the scene files use: elements, attributes (ignored),
// text, CDATA, comments, processing instructions and the five predefined entities plus
// numeric character references.  `GetText()` semantics: the text of an element is its
// first child if that child is text.  Deviation: the reference takes file.FirstChild() as
// the root, so a leading <?xml?> declaration or comment crashes it (appendix B); we skip
// those and use the first element — a strict superset.
#include <cctype>
#include <cmath>
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>
#include <stdexcept>

#include "host_scene.h"

namespace rt {
namespace {

struct Node {
  std::string tag;
  std::string text;
  bool has_text = false;
  std::vector<std::unique_ptr<Node>> children;
  const Node* first(const char* name) const {
    for (const auto& c : children)
      if (c->tag == name) return c.get();
    return nullptr;
  }
  std::vector<const Node*> each(const char* name) const {
    std::vector<const Node*> r;
    for (const auto& c : children)
      if (c->tag == name) r.push_back(c.get());
    return r;
  }
};

class Reader {
 public:
  explicit Reader(std::string doc) : s_(std::move(doc)) {}

  std::unique_ptr<Node> document_root() {
    skip_prolog();
    if (i_ >= s_.size() || s_[i_] != '<') error("no root element");
    return parse_element();
  }

 private:
  std::string s_;
  size_t i_ = 0;

  [[noreturn]] void error(const std::string& what) const {
    throw std::runtime_error("scene xml: " + what + " at byte " + std::to_string(i_));
  }
  bool at(const char* lit) const { return s_.compare(i_, std::strlen(lit), lit) == 0; }
  void skip_to(const char* end) {
    const size_t k = s_.find(end, i_);
    if (k == std::string::npos) error(std::string("missing ") + end);
    i_ = k + std::strlen(end);
  }
  void skip_prolog() {
    for (;;) {
      while (i_ < s_.size() && std::isspace((unsigned char)s_[i_])) ++i_;
      if (at("<?")) skip_to("?>");
      else if (at("<!--")) skip_to("-->");
      else if (at("<!")) skip_to(">");
      else return;
    }
  }
  static std::string unescape(const std::string& raw) {
    std::string out;
    out.reserve(raw.size());
    for (size_t k = 0; k < raw.size(); ++k) {
      if (raw[k] != '&') {
        out.push_back(raw[k]);
        continue;
      }
      const size_t semi = raw.find(';', k);
      if (semi == std::string::npos) {
        out.push_back('&');
        continue;
      }
      const std::string e = raw.substr(k + 1, semi - k - 1);
      if (e == "amp") out.push_back('&');
      else if (e == "lt") out.push_back('<');
      else if (e == "gt") out.push_back('>');
      else if (e == "quot") out.push_back('"');
      else if (e == "apos") out.push_back('\'');
      else if (e.size() > 1 && e[0] == '#') {
        const bool hexa = e[1] == 'x' || e[1] == 'X';
        out.push_back((char)std::strtol(e.c_str() + (hexa ? 2 : 1), nullptr, hexa ? 16 : 10));
      } else {
        out += "&" + e + ";";
      }
      k = semi;
    }
    return out;
  }
  std::unique_ptr<Node> parse_element() {
    ++i_;  // '<'
    const size_t name_begin = i_;
    while (i_ < s_.size() && !std::isspace((unsigned char)s_[i_]) && s_[i_] != '>' &&
           s_[i_] != '/')
      ++i_;
    auto node = std::make_unique<Node>();
    node->tag = s_.substr(name_begin, i_ - name_begin);
    if (node->tag.empty()) error("empty tag name");
    for (;;) {  // attributes: skipped, quotes honoured
      if (i_ >= s_.size()) error("unterminated start tag");
      const char c = s_[i_];
      if (c == '>') {
        ++i_;
        break;
      }
      if (c == '/' && i_ + 1 < s_.size() && s_[i_ + 1] == '>') {
        i_ += 2;
        return node;
      }
      if (c == '"' || c == '\'') {
        const size_t q = s_.find(c, i_ + 1);
        if (q == std::string::npos) error("unterminated attribute");
        i_ = q + 1;
        continue;
      }
      ++i_;
    }
    bool first_child = true;
    for (;;) {
      if (i_ >= s_.size()) error("unterminated element <" + node->tag + ">");
      if (at("</")) {
        skip_to(">");
        return node;
      }
      if (at("<!--")) {
        skip_to("-->");
        first_child = false;
        continue;
      }
      if (at("<![CDATA[")) {
        const size_t begin = i_ + 9;
        skip_to("]]>");
        if (first_child) {
          node->text = s_.substr(begin, i_ - 3 - begin);
          node->has_text = true;
        }
        first_child = false;
        continue;
      }
      if (at("<?")) {
        skip_to("?>");
        first_child = false;
        continue;
      }
      if (s_[i_] == '<') {
        node->children.push_back(parse_element());
        first_child = false;
        continue;
      }
      const size_t end = s_.find('<', i_);
      if (end == std::string::npos) error("text runs to end of file");
      if (first_child) {
        node->text = unescape(s_.substr(i_, end - i_));
        node->has_text = true;
      }
      first_child = false;
      i_ = end;
    }
  }
};

const char* text(const Node* n, const char* what) {
  if (!n) throw std::runtime_error(std::string("scene xml: missing <") + what + ">");
  if (!n->has_text) throw std::runtime_error(std::string("scene xml: <") + what + "> has no text");
  return n->text.c_str();
}

}  // namespace

void load_scene_xml(const std::string& path, XmlSceneStorage& st, rt_scene_desc& d) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::ios_base::failure("Error: The xml file cannot be loaded: " + path);
  std::string doc((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  const std::unique_ptr<Node> root = Reader(std::move(doc)).document_root();

  std::stringstream ss;  // one shared stream, as HW2/Scene.cpp:200
  auto put = [&](const Node* n, const char* what, const char* fallback) {
    if (n) ss << text(n, what) << std::endl;
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
    ss << text(c->first("Position"), "Position") << std::endl;
    ss << text(c->first("Gaze"), "Gaze") << std::endl;
    ss << text(c->first("Up"), "Up") << std::endl;
    ss << text(c->first("NearPlane"), "NearPlane") << std::endl;
    ss << text(c->first("NearDistance"), "NearDistance") << std::endl;
    ss << text(c->first("ImageResolution"), "ImageResolution") << std::endl;
    put(c->first("NumSamples"), "NumSamples", "1");
    ss << text(c->first("ImageName"), "ImageName") << std::endl;
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
  ss << text(lights->first("AmbientLight"), "AmbientLight") << std::endl;
  ss >> amb[0] >> amb[1] >> amb[2];
  for (const Node* pl : lights->each("PointLight")) {
    ss << text(pl->first("Position"), "Position") << std::endl;
    ss << text(pl->first("Intensity"), "Intensity") << std::endl;
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

  ss << text(root->first("VertexData"), "VertexData") << std::endl;
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
    ss << text(m->first("Material"), "Material") << std::endl;
    ss >> mat;
    ss << text(m->first("Faces"), "Faces") << std::endl;
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
    ss << text(t->first("Material"), "Material") << std::endl;
    ss >> mat;
    ss << text(t->first("Indices"), "Indices") << std::endl;
    ss >> a >> b >> c;
    st.triangle_indices.insert(st.triangle_indices.end(), {a - 1, b - 1, c - 1});
    st.triangle_material.push_back(mat - 1);
  }
  for (const Node* s : objs->each("Sphere")) {
    int mat, center;
    float radius;
    ss << text(s->first("Material"), "Material") << std::endl;
    ss >> mat;
    ss << text(s->first("Center"), "Center") << std::endl;
    ss >> center;
    ss << text(s->first("Radius"), "Radius") << std::endl;
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
