// ORACLE TEST INFRASTRUCTURE — CPU restatement of the reference PPM (progressive photon
// mapping) path.  See ppm_ref.h for what it is, what it replaces and how it is pinned.
// Built with -ffp-contract=off on plain x86-64 SSE; fp32 in the reference's operation order,
// the reference's double islands kept where it promotes (M_PI products, 1.0 divisions).
#include "ppm_ref.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../ceng795_amd/csrc/ppm_math.h"
#include "xml_lite.h"

namespace {
using oracle_xml::Elem;
using oracle_xml::XmlParser;

constexpr float kTestEps = 0.0001f;  // intersection_test_epsilon, PPM/include/Vector3.h:10
constexpr float kInf = std::numeric_limits<float>::infinity();
constexpr float kAlpha = 0.7f;       // ALPHA, PPM/src/Scene.cpp:13

// ------------------------------------------------------------------ Vector3 (PPM/include/Vector3.h)
struct V3 {
  float x = 0, y = 0, z = 0;
  V3() = default;
  V3(float a) : x(a), y(a), z(a) {}
  V3(float a, float b, float c) : x(a), y(b), z(c) {}
  float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
  float& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
};
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator*(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline V3 operator+(V3 a, float s) { return {a.x + s, a.y + s, a.z + s}; }
inline V3 operator-(V3 a, float s) { return {a.x - s, a.y - s, a.z - s}; }
inline V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 operator/(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline V3 operator*(float s, V3 a) { return a * s; }  // Vector3.h:125
inline V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
inline bool operator==(V3 a, V3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
inline float dot(V3 a, V3 b) { return (a.x * b.x) + (a.y * b.y) + (a.z * b.z); }
inline V3 cross(V3 a, V3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline float length(V3 a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
inline V3 normalize(V3 a) { return a / length(a); }
inline float smin(float a, float b) { return (b < a) ? b : a; }  // std::min
inline float smax(float a, float b) { return (a < b) ? b : a; }  // std::max

struct Ray {  // PPM/include/Ray.h
  V3 o, d;
  V3 point_at(float t) const { return o + (t * d); }
};

// ------------------------------------------------------------------ Matrix4x4 (PPM/src/Matrix4x4.cpp)
struct M4 {
  float e[4][4];
  explicit M4(bool identity = false) {
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 4; j++) e[i][j] = (identity && i == j) ? 1.0f : 0.0f;
  }
  V3 mul(V3 v, bool is_vector) const {
    V3 r;
    for (int i = 0; i < 3; i++) {
      r[i] = is_vector ? 0.0f : e[i][3];
      for (int j = 0; j < 3; j++) r[i] += e[i][j] * v[j];
    }
    return r;
  }
  M4 operator*(const M4& b) const {
    M4 r;
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 4; j++)
        for (int k = 0; k < 4; k++) r.e[i][j] += e[i][k] * b.e[k][j];
    return r;
  }
  M4 transpose() const {
    M4 t;
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 4; j++) t.e[i][j] = e[j][i];
    return t;
  }
  bool is_identity() const {
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 4; j++)
        if (e[i][j] != (i == j ? 1.0f : 0.0f)) return false;
    return true;
  }
  bool invert(M4& out) const {  // cofactor expansion, Matrix4x4.cpp:97-164
    float m[16], v[16];
    for (int i = 0; i < 16; i++) m[i] = e[i / 4][i % 4];
    v[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] +
           m[9] * m[7] * m[14] + m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
    v[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] -
           m[8] * m[7] * m[14] - m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
    v[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] +
           m[8] * m[7] * m[13] + m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
    v[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] -
            m[8] * m[6] * m[13] - m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
    v[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] -
           m[9] * m[3] * m[14] - m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
    v[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] +
           m[8] * m[3] * m[14] + m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
    v[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] -
           m[8] * m[3] * m[13] - m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
    v[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] +
            m[8] * m[2] * m[13] + m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
    v[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] +
           m[5] * m[3] * m[14] + m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
    v[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] -
           m[4] * m[3] * m[14] - m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
    v[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] +
            m[4] * m[3] * m[13] + m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
    v[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] -
            m[4] * m[2] * m[13] - m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
    v[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] -
           m[5] * m[3] * m[10] - m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
    v[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] +
           m[4] * m[3] * m[10] + m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
    v[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] -
            m[4] * m[3] * m[9] - m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
    v[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] +
            m[4] * m[2] * m[9] + m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
    float det = m[0] * v[0] + m[1] * v[4] + m[2] * v[8] + m[3] * v[12];
    if (det == 0.0f) return false;
    det = 1.0f / det;
    for (int i = 0; i < 16; i++) out.e[i / 4][i % 4] = v[i] * det;
    return true;
  }
};

struct Xform {  // Transformation.h: matrix, inverse, inverse transpose
  M4 m{true}, inv{true}, nrm{true};
};
Xform arbitrary(const M4& m) {  // Arbitrary_transformation, Transformation.cpp:83-91
  Xform t;
  t.m = m;
  if (!m.invert(t.inv)) throw std::runtime_error("NOT INVERTIBLE MATRIX!");
  t.nrm = t.inv.transpose();
  return t;
}

// ------------------------------------------------------------------ scene
struct Box {  // PPM/include/Bounding_box.h
  V3 lo{kInf, kInf, kInf}, hi{-kInf, -kInf, -kInf}, delta, center;
  Box() = default;
  Box(V3 a, V3 b) : lo(a), hi(b), delta(b - a), center((b + a) / 2) {}
  void expand(const Box& o) {  // Bounding_box.cpp:5-17
    lo = V3(smin(lo.x, o.lo.x), smin(lo.y, o.lo.y), smin(lo.z, o.lo.z));
    hi = V3(smax(hi.x, o.hi.x), smax(hi.y, o.hi.y), smax(hi.z, o.hi.z));
    delta = hi - lo;
    center = (hi + lo) / 2.;
  }
  void fit(V3 p) {  // Bounding_box.cpp:19-30
    lo = V3(smin(lo.x, p.x), smin(lo.y, p.y), smin(lo.z, p.z));
    hi = V3(smax(hi.x, p.x), smax(hi.y, p.y), smax(hi.z, p.z));
    delta = hi - lo;
    center = (hi + lo) / 2.;
  }
  float intersect(const Ray& r) const {  // Bounding_box.cpp:32-54
    float tmin = -kInf, tmax = kInf;
    for (int i = 0; i < 3; i++) {
      if (std::fabs(r.d[i]) < kTestEps) continue;
      float t0 = (lo[i] - r.o[i]) / r.d[i];
      float t1 = (hi[i] - r.o[i]) / r.d[i];
      if (r.d[i] < 0) std::swap(t0, t1);
      if (t0 > tmin) tmin = t0;
      if (t1 < tmax) tmax = t1;
      if (tmin > tmax) return kInf;
    }
    return tmin > 0.0f ? tmin : tmax;
  }
};
Box transform_box(const Box& b, const M4& m) {  // Bounding_box.cpp:56-137
  const V3 lo = b.lo, hi = b.hi;
  const V3 c[8] = {m.mul(V3(lo.x, lo.y, lo.z), false), m.mul(V3(lo.x, lo.y, hi.z), false),
                   m.mul(V3(lo.x, hi.y, lo.z), false), m.mul(V3(lo.x, hi.y, hi.z), false),
                   m.mul(V3(hi.x, lo.y, lo.z), false), m.mul(V3(hi.x, lo.y, hi.z), false),
                   m.mul(V3(hi.x, hi.y, lo.z), false), m.mul(V3(hi.x, hi.y, hi.z), false)};
  V3 mn = c[0], mx = c[0];
  for (int k = 1; k < 8; k++) {
    mn = V3(smin(mn.x, c[k].x), smin(mn.y, c[k].y), smin(mn.z, c[k].z));
    mx = V3(smax(mx.x, c[k].x), smax(mx.y, c[k].y), smax(mx.z, c[k].z));
  }
  return Box(mn, mx);
}

enum MatType { kDiffuse = 0, kMirror = 1, kRefractive = 2 };
struct Material {  // PPM/include/Material.h
  V3 diffuse, specular, mirror, transparency;
  int type = kDiffuse;
  int brdf_id = -1;
  float refraction_index = 1.0f, phong = 1.0f;
};

struct Camera {  // PPM/include/Camera.h:28-59
  V3 e, s_u, s_v, top_left;
  int width = 0, height = 0, samples = 1;
  Ray ray_at(float x, float y) const {  // Camera.h:76-84
    const V3 s = top_left + x * s_u - y * s_v;
    return Ray{e, normalize(s - e)};
  }
};

enum Kind { kNode, kTri, kSphere, kInstance };
struct Shape {
  Kind kind;
  Box box;
  int left = -1, right = -1;   // kNode
  int v[3] = {0, 0, 0};        // kTri: absolute vertex indices (index + vertex_offset)
  V3 normal;                   // kTri: flat normal
  bool smooth = false;
  V3 center;                   // kSphere
  float radius = 0;
  Xform xf;                    // kSphere / kInstance
  int mesh = -1;               // kInstance: mesh id
  bool refractive = false;     // kInstance
  int material = -1;           // kSphere / kInstance
};
struct Mesh {
  int root = -1;  // shape id of the mesh BVH root (node or single triangle)
  int material = -1;
  M4 base{true};
};

struct Isect {  // PPM/include/Intersection.h
  float t = kInf;
  int shape = -1;
  V3 normal{0.0f};
};

struct HitPoint {  // PPM/include/Hit_point.h
  int material;
  V3 attenuation, w_o, normal, position, flux;
  float radius_squared = 0;
  unsigned n = 0;
  int pixel;
  float pixel_weight;
};

struct Scene {
  float eps = 0.001f;
  int per_iteration = 8000, iterations = 1000, max_depth = 20;
  std::vector<Camera> cameras;
  std::vector<Material> materials;
  std::vector<V3> vpos, vnormal;
  std::vector<std::pair<V3, V3>> lights;  // position, intensity
  std::vector<Shape> shapes;
  std::vector<Mesh> meshes;
  int root = -1;
  // PPM state
  std::vector<HitPoint> hps;
  std::vector<std::vector<int>> grid;
  Box hp_box;
  float hash_scale = 0, r0 = 0;
  unsigned num_hash = 0;
  int eye_cam = -1;  // camera of the last eye pass (sizes density_estimation's image)
  // analysis log (ppmref_trace_photons_logged, tools/ppm_list_study.py): per deposit x, normal,
  // photon index; per update (hit point, deposit number)
  std::vector<float>* log_dep = nullptr;
  std::vector<long long>* log_upd = nullptr;
  long long log_photon = 0;

  // ---------------------------------------------------------------- intersection
  bool tri_intersect(const Shape& s, const Ray& r, Isect& h, bool culling) const {
    // Mesh_triangle.cpp:57-111
    const V3 p0 = vpos[s.v[0]], p1 = vpos[s.v[1]], p2 = vpos[s.v[2]];
    const V3 a1 = p0 - p1, a2 = p0 - p2, a3 = r.d;
    if (culling && dot(a3, s.normal) > 0.0f) return false;
    auto det = [](V3 c1, V3 c2, V3 c3) {
      return c1.x * (c2.y * c3.z - c3.y * c2.z) + c2.x * (c3.y * c1.z - c1.y * c3.z) +
             c3.x * (c1.y * c2.z - c2.y * c1.z);
    };
    const float det_a = det(a1, a2, a3);
    if (det_a == 0.0f) return false;
    const V3 b = (p0 - r.o) / det_a;
    const float beta = det(b, a2, a3);
    if (beta < -kTestEps) return false;
    const float gamma = det(a1, b, a3);
    if (gamma < -kTestEps || beta + gamma > 1.0f + kTestEps) return false;
    const float t = det(a1, a2, b);
    if (t > -kTestEps) {
      h.t = t;
      h.normal = s.smooth ? normalize((1 - beta - gamma) * vnormal[s.v[0]] +
                                      beta * vnormal[s.v[1]] + gamma * vnormal[s.v[2]])
                          : s.normal;
      return true;
    }
    return false;
  }
  bool sphere_intersect(const Shape& s, const Ray& r, Isect& h) const {  // Sphere.cpp:26-64
    const Ray rl{s.xf.inv.mul(r.o, false), s.xf.inv.mul(r.d, true)};
    const V3 co = rl.o - s.center;
    const float a = dot(rl.d, rl.d);
    const float b = 2 * dot(rl.d, co);
    const float c = dot(co, co) - s.radius * s.radius;
    const float disc = b * b - 4 * a * c;
    if (disc < -kTestEps) return false;
    if (disc < kTestEps) {
      h.t = -b / (2 * a);
    } else {
      const float sq = std::sqrt(disc);
      const float t1 = (-b + sq) / (2 * a);
      const float t2 = (-b - sq) / (2 * a);
      h.t = t2 < 0.0f ? t1 : t2;
    }
    const V3 local = rl.point_at(h.t) - s.center;
    h.normal = normalize(s.xf.nrm.mul(normalize(local), true));
    return true;
  }
  bool intersect(int id, const Ray& r, Isect& h, bool culling, long long& boxes) const {
    const Shape& s = shapes[id];
    switch (s.kind) {
      case kTri:
        if (tri_intersect(s, r, h, culling)) {
          h.shape = id;
          return true;
        }
        return false;
      case kSphere:
        if (sphere_intersect(s, r, h)) {
          h.shape = id;
          return true;
        }
        return false;
      case kInstance: {  // Mesh_instance::intersect, Mesh.h:70-93
        boxes++;
        const float bt = s.box.intersect(r);
        if (bt < 0.0f || bt == kInf) return false;
        const bool cull = s.refractive ? false : culling;
        const Ray rl{s.xf.inv.mul(r.o, false), s.xf.inv.mul(r.d, true)};
        if (intersect(meshes[s.mesh].root, rl, h, cull, boxes)) {
          h.normal = normalize(s.xf.nrm.mul(h.normal, true));
          h.shape = id;
          return true;
        }
        return false;
      }
      case kNode: {  // BVH::intersect, Bounding_volume_hierarchy.cpp:30-52
        boxes++;
        const float bt = s.box.intersect(r);
        if (bt < 0.0f || bt == kInf) return false;
        bool any = false;
        Isect lh;
        if (intersect(s.left, r, lh, culling, boxes) && lh.t > 0.0f && lh.t < h.t) {
          h = lh;
          any = true;
        }
        Isect rh;
        if (intersect(s.right, r, rh, culling, boxes) && rh.t > 0.0f && rh.t < h.t) {
          any = true;
          h = rh;
        }
        return any;
      }
    }
    return false;
  }
  bool closest(const Ray& r, Isect& h) const {
    long long boxes = 0;
    if (root < 0) return false;
    return intersect(root, r, h, true, boxes);
  }
  const Material& material_of(const Isect& h) const {
    return materials[shapes[h.shape].material];
  }

  // ---------------------------------------------------------------- BVH build (BVH.cpp:3-28)
  int build(std::vector<int>& objs, int start, int end, int dim) {
    Box box;
    for (int i = start; i < end; i++) box.expand(shapes[objs[i]].box);
    const float center = box.center[dim];
    int mid = start;
    for (int i = start; i < end; i++)
      if (shapes[objs[i]].box.center[dim] < center) std::swap(objs[i], objs[mid++]);
    if (mid == start || mid == end) mid = start + ((end - start) / 2);
    Shape n;
    n.kind = kNode;
    n.box = box;
    const int id = (int)shapes.size();
    shapes.push_back(n);
    const int l = (start + 1 == mid) ? objs[start] : build(objs, start, mid, (dim + 1) % 3);
    const int r = (mid + 1 == end) ? objs[mid] : build(objs, mid, end, (dim + 1) % 3);
    shapes[id].left = l;
    shapes[id].right = r;
    return id;
  }
  int create_bvh(std::vector<int>& objs) {  // Bounding_volume_hierarchy.h:9-18
    if (objs.empty()) return -1;
    if (objs.size() == 1) return objs[0];
    return build(objs, 0, (int)objs.size(), 0);
  }
  const Box& box_of(int id) const { return shapes[id].box; }
};

// ------------------------------------------------------------------ XML ingest
const char* text_of(const Elem* e, const char* what) {
  if (!e || !e->has_text) throw std::runtime_error(std::string("missing <") + what + ">");
  return e->text.c_str();
}
int int_attr(const Elem* e, const char* name, int dflt) {  // tinyxml2 IntAttribute
  const char* a = e->attr(name);
  if (!a) return dflt;
  int v = dflt;
  std::sscanf(a, "%d", &v);
  return v;
}
bool bool_attr(const Elem* e, const char* name, bool dflt) {  // tinyxml2 BoolAttribute
  const char* a = e->attr(name);
  if (!a) return dflt;
  std::string s(a);
  if (s == "true" || s == "1") return true;
  if (s == "false" || s == "0") return false;
  int v;
  if (std::sscanf(a, "%d", &v) == 1) return v != 0;
  return dflt;
}

struct Transforms {
  std::vector<Xform> scaling, translation, rotation;
};

// "s1 t2 r1" lists (Mesh.cpp:38-63, Sphere.cpp:111-136): left-multiplied in order.
M4 apply_list(std::stringstream& stream, const Elem* child, const Transforms& T, M4 m) {
  if (!child) return m;
  char type;
  int index;
  stream.clear();
  stream << text_of(child, "Transformations") << std::endl;
  while (!(stream >> type).eof()) {
    stream >> index;
    index--;
    const std::vector<Xform>* v = type == 's' ? &T.scaling
                                  : type == 't' ? &T.translation
                                  : type == 'r' ? &T.rotation : nullptr;
    if (v) {
      if (index < 0 || index >= (int)v->size()) throw std::runtime_error("bad transform index");
      m = (*v)[index].m * m;
    }
    if (stream.fail() && !stream.eof()) throw std::runtime_error("bad transformation list");
  }
  stream.clear();
  return m;
}

Camera make_camera(V3 up, V3 gaze, V3 pos, int samples, float l, float r, float b, float t,
                   float dist, int w, int h, bool left_handed) {  // Camera.h:28-45
  Camera c;
  c.e = pos;
  c.samples = samples;
  c.width = w;
  c.height = h;
  const V3 W = -(normalize(gaze));
  V3 U, V;
  if (left_handed) {
    U = normalize(cross(W, normalize(up)));
    V = normalize(cross(U, W));
  } else {
    U = normalize(cross(normalize(up), W));
    V = normalize(cross(W, U));
  }
  c.top_left = c.e - W * dist + l * U + t * V;
  c.s_u = ((r - l) / w) * U;
  c.s_v = ((t - b) / h) * V;
  return c;
}

void load(Scene& sc, const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("Error: The xml file cannot be loaded.");
  std::stringstream buf;
  buf << f.rdbuf();
  const std::string txt = buf.str();
  XmlParser xp(txt);
  xp.skip_misc();
  std::unique_ptr<Elem> root = xp.element();
  std::stringstream stream;  // Scene.cpp:377 (scalars + VertexData)

  auto scalar = [&](const char* tag, const char* dflt) {
    const Elem* e = root->child(tag);
    stream << (e ? text_of(e, tag) : dflt) << std::endl;
  };
  scalar("ShadowRayEpsilon", "0.001");
  stream >> sc.eps;
  scalar("PhotonCountPerIteration", "8000");
  stream >> sc.per_iteration;
  scalar("NumberOfIterations", "1000");
  stream >> sc.iterations;
  scalar("MaxRecursionDepth", "20");
  stream >> sc.max_depth;
  if (sc.max_depth > 20) sc.max_depth = 20;

  if (const Elem* cams = root->child("Cameras")) {  // Camera.cpp:4-99
    std::stringstream cs;
    constexpr float d2r = M_PI / 180.0f;
    for (const Elem* e : cams->all("Camera")) {
      V3 pos, up, gaze;
      float dist, l, r, b, t;
      int w, h, ns;
      std::string name;
      cs << text_of(e->child("Position"), "Position") << std::endl;
      cs << text_of(e->child("Up"), "Up") << std::endl;
      cs << text_of(e->child("NearDistance"), "NearDistance") << std::endl;
      cs << text_of(e->child("ImageResolution"), "ImageResolution") << std::endl;
      if (const Elem* n = e->child("NumSamples")) cs << text_of(n, "NumSamples") << std::endl;
      else cs << 1 << std::endl;
      cs << text_of(e->child("ImageName"), "ImageName") << std::endl;
      cs >> pos.x >> pos.y >> pos.z >> up.x >> up.y >> up.z >> dist >> w >> h >> ns;
      ns = (int)std::sqrt(ns);
      if (ns <= 0) ns = 1;
      cs >> name;
      const char* type = e->attr("type");
      const Elem* g = e->child("Gaze");
      if (!g) g = e->child("GazePoint");
      if (type && std::string(type) == "simple") {
        cs << text_of(g, "Gaze") << std::endl;
        cs << text_of(e->child("FovY"), "FovY") << std::endl;
        V3 gp;
        float fovy;
        cs >> gp.x >> gp.y >> gp.z >> fovy;
        const float half = d2r * fovy / 2;
        t = tanf(half) * dist;
        const float aspect = 1.0f * w / h;
        b = -1.0f * t;
        r = t * aspect;
        l = -1.0f * r;
        gaze = normalize(gp - pos);
      } else {
        cs << text_of(g, "Gaze") << std::endl;
        cs << text_of(e->child("NearPlane"), "NearPlane") << std::endl;
        cs >> gaze.x >> gaze.y >> gaze.z >> l >> r >> b >> t;
      }
      if (const Elem* tm = e->child("Tonemap")) {  // options consumed from the stream
        const Elem* tmo = tm->child("TMO");
        if (tmo && std::string(text_of(tmo, "TMO")) == "Photographic") {
          float k, sp, sat;
          cs << text_of(tm->child("TMOOptions"), "TMOOptions") << std::endl;
          cs << text_of(tm->child("Saturation"), "Saturation") << std::endl;
          cs >> k >> sp >> sat;
        }
      }
      const char* hand = e->attr("handedness");
      const bool left = hand && std::string(hand) == "left";
      sc.cameras.push_back(make_camera(up, gaze, pos, ns, l, r, b, t, dist, w, h, left));
    }
  }

  if (const Elem* mats = root->child("Materials")) {  // Material.cpp:3-75
    std::stringstream ms;
    Material m;
    for (const Elem* e : mats->all("Material")) {
      auto put = [&](const char* tag, const char* dflt) {
        const Elem* c = e->child(tag);
        ms << (c ? text_of(c, tag) : dflt) << std::endl;
      };
      put("DiffuseReflectance", "0 0 0");
      put("SpecularReflectance", "0 0 0");
      put("MirrorReflectance", "0 0 0");
      put("PhongExponent", "1");
      put("Transparency", "0 0 0");
      put("RefractionIndex", "1.0");
      m.brdf_id = int_attr(e, "BRDF", 0) - 1;
      ms >> m.diffuse.x >> m.diffuse.y >> m.diffuse.z;
      ms >> m.specular.x >> m.specular.y >> m.specular.z;
      ms >> m.mirror.x >> m.mirror.y >> m.mirror.z;
      ms >> m.phong;
      ms >> m.transparency.x >> m.transparency.y >> m.transparency.z;
      ms >> m.refraction_index;
      if (!(m.mirror == V3(0.0f))) m.type = kMirror;
      else if (!(m.transparency == V3(0.0f))) m.type = kRefractive;
      else m.type = kDiffuse;
      if (bool_attr(e, "degamma", false)) {
        for (int k = 0; k < 3; k++) {
          m.diffuse[k] = (float)::pow((double)m.diffuse[k], (double)2.2f);  // double pow
          m.specular[k] = (float)::pow((double)m.specular[k], (double)2.2f);
        }
      }
      sc.materials.push_back(m);
    }
  }

  Transforms T;
  if (const Elem* tr = root->child("Transformations")) {  // Transformation.cpp:93-134
    std::stringstream ts;
    for (const Elem* e : tr->all("Translation")) {
      float x, y, z;
      ts << text_of(e, "Translation") << std::endl;
      ts >> x >> y >> z;
      Xform t;
      t.m = M4(true);
      t.m.e[0][3] = x;
      t.m.e[1][3] = y;
      t.m.e[2][3] = z;
      t.inv = M4(true);
      t.inv.e[0][3] = -x;
      t.inv.e[1][3] = -y;
      t.inv.e[2][3] = -z;
      t.nrm = t.inv.transpose();
      T.translation.push_back(t);
    }
    std::stringstream ss;
    for (const Elem* e : tr->all("Scaling")) {
      float x, y, z;
      ss << text_of(e, "Scaling") << std::endl;
      ss >> x >> y >> z;
      Xform t;
      t.m = M4(false);
      t.m.e[0][0] = x;
      t.m.e[1][1] = y;
      t.m.e[2][2] = z;
      t.m.e[3][3] = 1.0f;
      t.inv = M4(false);
      t.inv.e[0][0] = 1.0f / x;
      t.inv.e[1][1] = 1.0f / y;
      t.inv.e[2][2] = 1.0f / z;
      t.inv.e[3][3] = 1.0f;
      t.nrm = t.inv.transpose();
      T.scaling.push_back(t);
    }
    std::stringstream rs;
    constexpr float d2r = M_PI / 180.0f;
    for (const Elem* e : tr->all("Rotation")) {
      float angle, x, y, z;
      rs << text_of(e, "Rotation") << std::endl;
      rs >> angle >> x >> y >> z;
      angle = angle * d2r;
      const V3 u = normalize(V3(x, y, z));  // Transformation.cpp:34-75
      const V3 v = normalize((x != 0.0f || y != 0.0f) ? V3(-u.y, u.x, 0.0f) : V3(0.0f, 1.0f, 0.0f));
      const V3 w = cross(u, v);
      M4 m;
      m.e[0][0] = u.x; m.e[0][1] = u.y; m.e[0][2] = u.z;
      m.e[1][0] = v.x; m.e[1][1] = v.y; m.e[1][2] = v.z;
      m.e[2][0] = w.x; m.e[2][1] = w.y; m.e[2][2] = w.z;
      m.e[3][3] = 1.0f;
      M4 rot;
      rot.e[0][0] = 1.0f;
      rot.e[1][1] = std::cos(angle);
      rot.e[1][2] = -std::sin(angle);
      rot.e[2][1] = -rot.e[1][2];
      rot.e[2][2] = rot.e[1][1];
      rot.e[3][3] = 1.0f;
      M4 irot;
      irot.e[0][0] = 1.0f;
      irot.e[1][1] = std::cos(-angle);
      irot.e[1][2] = -std::sin(-angle);
      irot.e[2][1] = -irot.e[1][2];
      irot.e[2][2] = irot.e[1][1];
      irot.e[3][3] = 1.0f;
      const M4 mt = m.transpose();
      Xform t;
      t.m = mt * (rot * m);
      t.inv = mt * (irot * m);
      t.nrm = t.inv.transpose();
      T.rotation.push_back(t);
    }
  }

  if (const Elem* vd = root->child("VertexData")) {  // Scene.cpp:452-470
    if (!vd->attr("binaryFile")) {
      stream << text_of(vd, "VertexData") << std::endl;
      V3 v;
      while (!(stream >> v.x).eof()) {
        stream >> v.y >> v.z;
        if (stream.fail()) throw std::runtime_error("bad VertexData");
        sc.vpos.push_back(v);
      }
    }
  }
  stream.clear();
  sc.vnormal.assign(sc.vpos.size(), V3(0.0f));
  std::vector<bool> has_normal(sc.vpos.size(), false);

  if (const Elem* ls = root->child("Lights")) {  // Point_light.cpp:32-51
    std::stringstream lsr;
    for (const Elem* e : ls->all("PointLight")) {
      V3 p, i;
      lsr << text_of(e->child("Position"), "Position") << std::endl;
      lsr << text_of(e->child("Intensity"), "Intensity") << std::endl;
      lsr >> p.x >> p.y >> p.z >> i.x >> i.y >> i.z;
      sc.lights.push_back({p, i});
    }
  }

  std::vector<int> objects;
  auto vertex = [&](int i) -> V3 {
    if (i < 0 || i >= (int)sc.vpos.size()) throw std::runtime_error("vertex index out of range");
    return sc.vpos[i];
  };
  auto check_mat = [&](int m) {
    if (m < 0 || m >= (int)sc.materials.size()) throw std::runtime_error("material out of range");
  };
  if (const Elem* objs = root->child("Objects")) {
    {  // spheres, Sphere.cpp:84-144
      std::stringstream ss;
      for (const Elem* e : objs->all("Sphere")) {
        int mat, center;
        float radius;
        ss << text_of(e->child("Material"), "Material") << std::endl;
        ss >> mat;
        mat--;
        ss << text_of(e->child("Center"), "Center") << std::endl;
        ss >> center;
        const V3 c = vertex(center - 1);
        ss << text_of(e->child("Radius"), "Radius") << std::endl;
        ss >> radius;
        M4 m = apply_list(ss, e->child("Transformations"), T, M4(true));
        ss.clear();
        if (const Elem* tx = e->child("Texture")) {
          int tid;
          ss << text_of(tx, "Texture") << std::endl;
          ss >> tid;
        }
        ss.clear();
        check_mat(mat);
        Shape s;
        s.kind = kSphere;
        s.center = c;
        s.radius = radius;
        s.material = mat;
        s.xf = arbitrary(m);
        const V3 delta(radius);
        s.box = s.xf.m.is_identity() ? Box(c - delta, c + delta)
                                     : transform_box(Box(c - delta, c + delta), s.xf.m);
        objects.push_back((int)sc.shapes.size());
        sc.shapes.push_back(s);
      }
    }
    {  // meshes, Mesh.cpp:5-111
      std::stringstream ms;
      for (const Elem* e : objs->all("Mesh")) {
        int mat;
        ms << text_of(e->child("Material"), "Material") << std::endl;
        ms >> mat;
        mat--;
        const char* sm = e->attr("shadingMode");
        const bool smooth = sm && std::string(sm) == "smooth";
        M4 m = apply_list(ms, e->child("Transformations"), T, M4(true));
        ms.clear();
        if (const Elem* tx = e->child("Texture")) {
          int tid;
          ms << text_of(tx, "Texture") << std::endl;
          ms >> tid;
        }
        ms.clear();
        std::vector<int> tris;
        const Elem* faces = e->child("Faces");
        if (!faces) throw std::runtime_error("mesh without <Faces>");
        if (!faces->attr("plyFile") && !faces->attr("binaryFile")) {
          const int offset = int_attr(faces, "vertexOffset", 0);
          ms << text_of(faces, "Faces") << std::endl;
          int a, b, c;
          while (!(ms >> a).eof()) {
            ms >> b >> c;
            if (ms.fail()) throw std::runtime_error("bad Faces");
            a--, b--, c--;
            Shape t;
            t.kind = kTri;
            t.v[0] = a + offset;
            t.v[1] = b + offset;
            t.v[2] = c + offset;
            const V3 p0 = vertex(t.v[0]), p1 = vertex(t.v[1]), p2 = vertex(t.v[2]);
            t.normal = normalize(cross(p1 - p0, p2 - p0));  // Mesh_triangle.cpp:23
            t.smooth = smooth;
            V3 mn = p0, mx = p0;
            mn = V3(smin(mn.x, p1.x), smin(mn.y, p1.y), smin(mn.z, p1.z));
            mx = V3(smax(mx.x, p1.x), smax(mx.y, p1.y), smax(mx.z, p1.z));
            mn = V3(smin(mn.x, p2.x), smin(mn.y, p2.y), smin(mn.z, p2.z));
            mx = V3(smax(mx.x, p2.x), smax(mx.y, p2.y), smax(mx.z, p2.z));
            t.box = Box(mn, mx);
            t.material = mat;
            const float area = length(cross(p1 - p0, p2 - p0)) / 2;  // get_surface_area
            for (int k = 0; k < 3; k++) {
              sc.vnormal[t.v[k]] = sc.vnormal[t.v[k]] + t.normal * area;
              has_normal[t.v[k]] = true;
            }
            tris.push_back((int)sc.shapes.size());
            sc.shapes.push_back(t);
          }
        }
        ms.clear();
        Mesh mesh;
        mesh.material = mat;
        mesh.base = m;
        mesh.root = sc.create_bvh(tris);
        if (mesh.root < 0) throw std::runtime_error("mesh without triangles");
        sc.meshes.push_back(mesh);
      }
    }
    auto add_instance = [&](int mesh_id, int mat, const M4& m) {  // Mesh.h:104-112
      check_mat(mat);
      Shape s;
      s.kind = kInstance;
      s.mesh = mesh_id;
      s.material = mat;
      s.xf = arbitrary(m);
      s.refractive = sc.materials[mat].type == kRefractive;
      s.box = transform_box(sc.box_of(sc.meshes[mesh_id].root), s.xf.m);
      objects.push_back((int)sc.shapes.size());
      sc.shapes.push_back(s);
    };
    for (int k = 0; k < (int)sc.meshes.size(); k++)  // Mesh.cpp:113-125
      add_instance(k, sc.meshes[k].material, arbitrary(sc.meshes[k].base).m);
    std::stringstream is;
    for (const Elem* e : objs->all("MeshInstance")) {  // Mesh.cpp:126-206
      const int base = int_attr(e, "baseMeshId", 0) - 1;
      if (base < 0 || base >= (int)sc.meshes.size()) throw std::runtime_error("bad baseMeshId");
      int mat;
      is << text_of(e->child("Material"), "Material") << std::endl;
      is >> mat;
      mat--;
      M4 m = sc.meshes[base].base;
      const char* reset = e->attr("resetTransform");
      if (reset && std::string(reset) == "true") m = M4(true);
      m = apply_list(is, e->child("Transformations"), T, m);
      is.clear();
      if (const Elem* mb = e->child("MotionBlur")) {
        float vx, vy, vz;
        is << text_of(mb, "MotionBlur") << std::endl;
        is >> vx >> vy >> vz;
      }
      is.clear();
      add_instance(base, mat, m);
    }
  }
  for (size_t k = 0; k < sc.vnormal.size(); k++)  // Vertex::finalize_normal
    sc.vnormal[k] = normalize(sc.vnormal[k]);
  sc.root = sc.create_bvh(objects);
}

// ------------------------------------------------------------------ PPM passes
// Shared refraction setup of photon_trace / eye_trace (Scene.cpp:225-245, 330-352).
struct Refraction {
  bool tir, into;
  Ray reflection, refraction;
  float fresnel;
};
Refraction refract_setup(const Scene& sc, const Ray& ray, V3 x, V3 normal, const Material& m) {
  Refraction R;
  const V3 nl = dot(normal, ray.d) < 0.0f ? normal : normal * -1;
  const V3 w_o = normalize(ray.o - x);
  const V3 w_r = normalize((2.0f * dot(normal, w_o) * normal) - w_o);
  R.reflection = Ray{x + (w_r * sc.eps), w_r};
  R.into = dot(normal, nl) > 0.0f;
  const float air = 1.0f;
  const float nnt = R.into ? air / m.refraction_index : m.refraction_index / air;
  const float ddn = dot(ray.d, nl);
  const float cos2t = 1 - nnt * nnt * (1 - ddn * ddn);
  R.tir = cos2t < 0.0f;
  if (R.tir) return R;
  const V3 dir = normalize(ray.d * nnt - normal * ((R.into ? 1 : -1) * (ddn * nnt + std::sqrt(cos2t))));
  const float a = m.refraction_index - air, b = m.refraction_index + air;
  const float r0 = a * a / (b * b);
  const float cosa = R.into ? -ddn : dot(dir, normal);
  const float c = 1 - cosa;
  R.fresnel = r0 + (1 - r0) * c * c * c * c * c;
  R.refraction = Ray{x + (dir * sc.eps), dir};
  return R;
}

struct EyeItem {
  Ray ray;
  int depth;
  V3 attenuation;
};

// eye_trace (Scene.cpp:286-361) for one primary ray, depth first with an explicit stack
// (children pushed in reverse so the reflection subtree completes before the refraction one).
void eye_trace(Scene& sc, const Ray& primary, int pixel, ppmref_stats* st) {
  std::vector<EyeItem> stack;
  stack.push_back({primary, 0, V3(1.0f)});
  while (!stack.empty()) {
    const EyeItem it = stack.back();
    stack.pop_back();
    Isect h;
    if (st) st->eye_rays++;
    if (!sc.closest(it.ray, h)) continue;
    const V3 x = it.ray.point_at(h.t);
    const V3 normal = h.normal;
    const Material& m = sc.material_of(h);
    if (m.type == kDiffuse) {
      HitPoint hp;
      hp.material = sc.shapes[h.shape].material;
      hp.attenuation = it.attenuation;
      hp.w_o = normalize(it.ray.o - x);
      hp.normal = normal;
      hp.position = x;
      hp.pixel = pixel;
      hp.pixel_weight = 1.0f;
      sc.hps.push_back(hp);
    } else if (it.depth >= sc.max_depth) {
      continue;
    } else if (m.type == kMirror) {
      const V3 w_o = normalize(it.ray.o - x);
      const V3 w_r = normalize((2.0f * dot(normal, w_o) * normal) - w_o);
      stack.push_back({Ray{x + (w_r * sc.eps), w_r}, it.depth + 1, m.mirror * it.attenuation});
    } else {
      const Refraction R = refract_setup(sc, it.ray, x, normal, m);
      if (R.tir) {
        stack.push_back({R.reflection, it.depth + 1, m.transparency * it.attenuation});
        continue;
      }
      const V3 attenuated = m.transparency * it.attenuation;
      if (R.into) {
        stack.push_back({R.refraction, it.depth + 1, (1.0f - R.fresnel) * attenuated});
        stack.push_back({R.reflection, it.depth + 1, R.fresnel * it.attenuation});
      } else {
        stack.push_back({R.refraction, it.depth + 1, attenuated});
      }
    }
  }
}

unsigned hash3(const Scene& sc, int ix, int iy, int iz) {  // Scene.h:65-68 (int32 wrap)
  const unsigned a = (unsigned)ix * 73856093u, b = (unsigned)iy * 19349663u,
                 c = (unsigned)iz * 83492791u;
  return (a ^ b ^ c) % sc.num_hash;
}

void sample_hemisphere(const V3 w, ppm_math::Rng& rng, V3& d, float& p) {  // Scene.cpp:15-44
  const float e1 = rng.uniform01();
  const float e2 = rng.uniform01();
  const V3 u = normalize((w.x != 0.0f || w.y != 0.0f) ? V3(-w.y, w.x, 0.0f) : V3(0.0f, 1.0f, 0.0f));
  const V3 v = cross(w, u);
  const float phi = 2 * M_PI * e1;
  const float theta = ppm_math::asinf_ieee(std::sqrt(e2));
  float st, ct, sp, cp;
  ppm_math::sincosf_ieee(theta, st, ct);
  ppm_math::sincosf_ieee(phi, sp, cp);
  d = normalize(w * ct + v * st * cp + u * st * sp);
  p = smax(0.0f, dot(w, d)) / M_PI;
}

void generate_photon(const Scene& sc, ppm_math::Rng& rng, Ray& ray, V3& flux) {
  // Point_light::generate_photon, Point_light.cpp:7-30 (theta = 2 pi e2: not uniform on S^2)
  const V3 pos = sc.lights[0].first, I = sc.lights[0].second;
  flux = I * (M_PI * 4.0f);
  const float e1 = rng.uniform01();
  const float e2 = rng.uniform01();
  const V3 w(0.0f, 1.0f, 0.0f);
  const V3 u = normalize((w.x != 0.0f || w.y != 0.0f) ? V3(-w.y, w.x, 0.0f) : V3(0.0f, 1.0f, 0.0f));
  const V3 v = cross(w, u);
  const float phi = 2 * M_PI * e1;
  const float theta = 2 * M_PI * e2;
  float st, ct, sp, cp;
  ppm_math::sincosf_ieee(theta, st, ct);
  ppm_math::sincosf_ieee(phi, sp, cp);
  ray.d = normalize(w * ct + v * st * cp + u * st * sp);
  ray.o = pos;
}

// photon_trace (Scene.cpp:106-249): the recursion is a chain, so a loop.
void photon_trace(Scene& sc, Ray ray, V3 flux, ppm_math::Rng& rng, ppmref_stats* st) {
  int depth = 0;
  for (;;) {
    depth++;
    if (depth >= sc.max_depth) return;
    Isect h;
    if (st) st->photon_rays++;
    if (!sc.closest(ray, h)) return;
    const V3 x = ray.point_at(h.t);
    const V3 normal = h.normal;
    const V3 nl = dot(normal, ray.d) < 0 ? normal : normal * -1;
    const Material& m = sc.material_of(h);
    if (m.type == kDiffuse) {
      if (st) st->deposits++;
      if (sc.log_dep) {
        const float rec[8] = {x.x, x.y, x.z, normal.x, normal.y, normal.z, (float)sc.log_photon, 0.0f};
        sc.log_dep->insert(sc.log_dep->end(), rec, rec + 8);
      }
      if (sc.num_hash) {
        const V3 hh = (x - sc.hp_box.lo) * sc.hash_scale;
        const int ix = std::abs(int(hh.x)), iy = std::abs(int(hh.y)), iz = std::abs(int(hh.z));
        const V3 w_i = -normalize(ray.d);
        for (int id : sc.grid[hash3(sc, ix, iy, iz)]) {
          HitPoint& hp = sc.hps[id];
          const V3 v = hp.position - x;
          if ((dot(hp.normal, normal) > 1e-3f) && (dot(v, v) <= hp.radius_squared)) {
            const float rr = (hp.n * kAlpha + kAlpha) / (hp.n * kAlpha + 1.0);
            hp.radius_squared = hp.radius_squared * rr;
            hp.n++;
            if (st) st->updates++;
            if (sc.log_upd) {
              sc.log_upd->push_back(id);
              sc.log_upd->push_back((long long)(sc.log_dep->size() / 8) - 1);
            }
            V3 color(0.0f);
            const Material& hm = sc.materials[hp.material];
            if (hm.brdf_id == -1) {
              const float cos_i = dot(hp.normal, w_i);
              if (cos_i > 1.0f || cos_i <= 0.0f) {
                color = 0.0f;
              } else {
                const float sc_ = smax(0.0f, dot(hp.normal, normalize(hp.w_o + w_i)));
                color = (hm.diffuse + hm.specular * ppm_math::powf_ieee(sc_, hm.phong) / cos_i) *
                        hp.attenuation;
              }
            }
            hp.flux = (hp.flux + color * flux) * rr;
          }
        }
      }
      float prob;
      V3 d;
      sample_hemisphere(normal, rng, d, prob);
      V3 base(0.0f);
      const V3 w_i = -normalize(ray.d);
      const float cos_i = smax(0.0f, dot(normal, w_i));
      const V3 w_o = d;
      if (m.brdf_id == -1) {
        if (cos_i > 1.0f || cos_i <= 0.0f) {
          base = 0.0f;
        } else {
          const float sc_ = smax(0.0f, dot(nl, normalize(w_o + w_i)));
          base = (m.diffuse + (m.specular * ppm_math::powf_ieee(sc_, m.phong) / cos_i));
        }
      }
      const float cos_o = smax(0.0f, dot(normal, w_o));
      base = base * cos_o;
      if (rng.uniform01() < prob) {
        ray = Ray{x + (d * sc.eps), d};
        flux = (base * flux) / prob;
        continue;
      }
      return;
    } else if (m.type == kMirror) {
      const V3 w_o = normalize(ray.o - x);
      const V3 w_r = normalize((2.0f * dot(normal, w_o) * normal) - w_o);
      ray = Ray{x + (w_r * sc.eps), w_r};
      flux = m.mirror * flux;
    } else {
      const Refraction R = refract_setup(sc, ray, x, normal, m);
      if (R.tir) {
        ray = R.reflection;
        continue;
      }
      if (R.into) {
        ray = rng.uniform01() < R.fresnel ? R.reflection : R.refraction;
      } else {
        ray = R.refraction;
      }
    }
  }
}

}  // namespace

struct ppmref_scene {
  Scene sc;
};

extern "C" {

ppmref_scene* ppmref_load(const char* xml_path, char* err, int errlen) {
  auto s = std::make_unique<ppmref_scene>();
  try {
    load(s->sc, xml_path);
  } catch (const std::exception& e) {
    if (err && errlen > 0) std::snprintf(err, errlen, "%s", e.what());
    return nullptr;
  }
  return s.release();
}
void ppmref_free(ppmref_scene* s) { delete s; }
int ppmref_num_cameras(const ppmref_scene* s) { return (int)s->sc.cameras.size(); }
int ppmref_camera_info(const ppmref_scene* s, int cam, int* w, int* h, int* n) {
  if (cam < 0 || cam >= (int)s->sc.cameras.size()) return -1;
  const Camera& c = s->sc.cameras[cam];
  *w = c.width;
  *h = c.height;
  *n = c.samples;
  return 0;
}
int ppmref_settings(const ppmref_scene* s, int* per_iteration, int* iterations, int* max_depth) {
  *per_iteration = s->sc.per_iteration;
  *iterations = s->sc.iterations;
  *max_depth = s->sc.max_depth;
  return 0;
}

int ppmref_eye_pass(ppmref_scene* s, int cam, unsigned long long seed, ppmref_stats* st) {
  Scene& sc = s->sc;
  if (cam < 0 || cam >= (int)sc.cameras.size()) return -1;
  sc.hps.clear();  // reset_hash_grid
  sc.grid.clear();
  sc.eye_cam = cam;
  const Camera& c = sc.cameras[cam];
  if (c.samples == 1) {  // Scene.cpp:257-263
    for (int j = 0; j < c.height; j++)
      for (int i = 0; i < c.width; i++)
        eye_trace(sc, c.ray_at(i + 0.5f, j + 0.5f), j * c.width + i, st);
  } else {  // Scene.cpp:264-284: at most 2x2 jittered samples, each its own hit points
    const int n = std::min(2, c.samples);
    for (int j = 0; j < c.height; j++)
      for (int i = 0; i < c.width; i++) {
        ppm_math::Rng rng(seed, ppm_math::kEyeStream | (unsigned long long)(j * c.width + i));
        for (int x = 0; x < n; x++)
          for (int y = 0; y < n; y++) {
            const float ex = rng.uniform01();
            const float ey = rng.uniform01();
            const float sx = (x + ex) / n;
            const float sy = (y + ey) / n;
            eye_trace(sc, c.ray_at(i + sx, j + sy), j * c.width + i, st);
          }
      }
  }
  if (st) st->hit_points = (long long)sc.hps.size();
  return 0;
}

int ppmref_build_hash_grid(ppmref_scene* s, int width, int height, double* info) {
  Scene& sc = s->sc;  // Scene.cpp:53-93
  Box b;
  for (const HitPoint& h : sc.hps) b.fit(h.position);
  const V3 size = b.delta;
  const float r = ((size.x + size.y + size.z) / 3.0f) / ((width + height) / 2.0f) * 2.0f * 4.0f;
  sc.hp_box = Box();
  sc.num_hash = (unsigned)sc.hps.size();
  for (HitPoint& h : sc.hps) {
    h.radius_squared = r * r;
    h.n = 0;
    h.flux = V3(0.0f);
    sc.hp_box.fit(h.position - r);
    sc.hp_box.fit(h.position + r);
  }
  sc.hash_scale = 1.0 / (r * 2.0);
  sc.r0 = r;
  sc.grid.assign(sc.num_hash, {});
  for (int id = 0; id < (int)sc.hps.size(); id++) {
    const HitPoint& h = sc.hps[id];
    const V3 bmin = ((h.position - r) - sc.hp_box.lo) * sc.hash_scale;
    const V3 bmax = ((h.position + r) - sc.hp_box.lo) * sc.hash_scale;
    for (int iz = std::abs(int(bmin.z)); iz <= std::abs(int(bmax.z)); iz++)
      for (int iy = std::abs(int(bmin.y)); iy <= std::abs(int(bmax.y)); iy++)
        for (int ix = std::abs(int(bmin.x)); ix <= std::abs(int(bmax.x)); ix++)
          sc.grid[hash3(sc, ix, iy, iz)].push_back(id);
  }
  if (info) {
    const double v[8] = {r, sc.hash_scale, sc.hp_box.lo.x, sc.hp_box.lo.y, sc.hp_box.lo.z,
                         sc.hp_box.hi.x, sc.hp_box.hi.y, sc.hp_box.hi.z};
    std::memcpy(info, v, sizeof v);
  }
  return 0;
}

int ppmref_num_hit_points(const ppmref_scene* s) { return (int)s->sc.hps.size(); }

int ppmref_hit_points(const ppmref_scene* s, float* out) {
  for (const HitPoint& h : s->sc.hps) {
    const float rec[16] = {h.position.x, h.position.y, h.position.z, h.normal.x, h.normal.y,
                           h.normal.z, h.w_o.x, h.w_o.y, h.w_o.z, h.attenuation.x,
                           h.attenuation.y, h.attenuation.z, (float)h.pixel, h.pixel_weight,
                           h.radius_squared, (float)s->sc.materials[h.material].type};
    std::memcpy(out, rec, sizeof rec);
    out += 16;
  }
  return 0;
}

int ppmref_hit_state(const ppmref_scene* s, float* out) {
  for (const HitPoint& h : s->sc.hps) {
    out[0] = h.flux.x;
    out[1] = h.flux.y;
    out[2] = h.flux.z;
    out[3] = h.radius_squared;
    out[4] = (float)h.n;
    out += 5;
  }
  return 0;
}

int ppmref_trace_photons(ppmref_scene* s, unsigned long long seed, long long first,
                         long long count, ppmref_stats* st) {
  Scene& sc = s->sc;
  if (sc.lights.empty()) return -1;
  for (long long p = first; p < first + count; p++) {
    ppm_math::Rng rng(seed, (unsigned long long)p);
    Ray ray;
    V3 flux;
    generate_photon(sc, rng, ray, flux);
    if (st) st->photons++;
    photon_trace(sc, ray, flux, rng, st);
  }
  return 0;
}

// Analysis only (tools/ppm_list_study.py): ppmref_trace_photons that also logs every deposit
// (x, normal, photon index: 8 floats) and every update (hit point, deposit number).  Returns the
// deposit count; *n_upd = the update count; outputs truncated to their capacities.
long long ppmref_trace_photons_logged(ppmref_scene* s, unsigned long long seed, long long first,
                                      long long count, float* dep8, long long dep_cap,
                                      long long* upd2, long long upd_cap, long long* n_upd) {
  Scene& sc = s->sc;
  if (sc.lights.empty()) return -1;
  std::vector<float> dep;
  std::vector<long long> upd;
  sc.log_dep = &dep;
  sc.log_upd = &upd;
  for (long long p = first; p < first + count; p++) {
    ppm_math::Rng rng(seed, (unsigned long long)p);
    Ray ray;
    V3 flux;
    generate_photon(sc, rng, ray, flux);
    sc.log_photon = p;
    photon_trace(sc, ray, flux, rng, nullptr);
  }
  sc.log_dep = nullptr;
  sc.log_upd = nullptr;
  const long long nd = (long long)dep.size() / 8, nu = (long long)upd.size() / 2;
  std::copy(dep.begin(), dep.begin() + 8 * std::min(nd, dep_cap), dep8);
  std::copy(upd.begin(), upd.begin() + 2 * std::min(nu, upd_cap), upd2);
  *n_upd = nu;
  return nd;
}

int ppmref_density(const ppmref_scene* s, long long total, float* out) {
  const Scene& sc = s->sc;  // Scene.cpp:363-371 + Pixel::add_color / get_color
  if (sc.eye_cam < 0) return -1;
  const size_t npix = (size_t)sc.cameras[sc.eye_cam].width * sc.cameras[sc.eye_cam].height;
  std::vector<V3> col(npix, V3(0.0f));
  std::vector<float> wt(npix, 0.0f);
  for (const HitPoint& hp : sc.hps) {
    const float k = 1.0f / (M_PI * hp.radius_squared * (double)total);
    const V3 c = hp.flux * k;
    col[hp.pixel] = col[hp.pixel] + c * hp.pixel_weight;
    wt[hp.pixel] = wt[hp.pixel] + hp.pixel_weight;
  }
  for (size_t p = 0; p < npix; p++) {
    const V3 c = wt[p] == 0 ? V3(0.0f) : col[p] / wt[p];
    out[3 * p] = c.x;
    out[3 * p + 1] = c.y;
    out[3 * p + 2] = c.z;
  }
  return 0;
}

int ppmref_render(ppmref_scene* s, int cam, unsigned long long seed, int threads, float* out,
                  ppmref_stats* st) {
  Scene& sc = s->sc;
  if (cam < 0 || cam >= (int)sc.cameras.size() || threads < 1) return -1;
  if (st) std::memset(st, 0, sizeof *st);
  const Camera& c = sc.cameras[cam];
  int rc = ppmref_eye_pass(s, cam, seed, st);
  if (rc) return rc;
  ppmref_build_hash_grid(s, c.width, c.height, nullptr);
  const long long P = sc.per_iteration, I = sc.iterations;
  const long long per_thread = P / threads;
  // main.cpp:72-90: height < T runs one thread with all P photons per iteration
  const long long traced = c.height < threads ? P * I : per_thread * I * threads;
  rc = ppmref_trace_photons(s, seed, 0, traced, st);
  if (rc) return rc;
  const int normalizer = (int)(P * per_thread * threads);  // main.cpp:94 (int arithmetic)
  return ppmref_density(s, normalizer, out);
}

float ppmref_sinf(float x) { return ppm_math::sinf_ieee(x); }
float ppmref_cosf(float x) { return ppm_math::cosf_ieee(x); }
float ppmref_asinf(float x) { return ppm_math::asinf_ieee(x); }
float ppmref_powf(float x, float y) { return ppm_math::powf_ieee(x, y); }

}  // extern "C"
