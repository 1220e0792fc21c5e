// ORACLE TEST INFRASTRUCTURE — CPU restatement of the reference HW2 render path.
// Not product code: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
// it, as the checker / CPU baseline.  See cpu_ref.h for the pinning story.
//
// Every function restates one piece of /root/reference/HW2 with the same floating-point
// operation order: fp32 everywhere, no FMA (built with
// -ffp-contract=off on x86-64 SSE), IEEE division and sqrtf, and the double-precision
// islands of libm (pow, exp, log, sqrt) exactly where the reference calls the double
// overloads.
#include "cpu_ref.h"
#include "xml_lite.h"

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace {
using oracle_xml::Elem;
using oracle_xml::XmlParser;

constexpr float kEps = 0.000001f;  // HW2/Vector3.h:7
constexpr float kInf = std::numeric_limits<float>::infinity();

// ------------------------------------------------------------------ value types (Vector3.h)
struct V3 {
  float x, y, z;
};
inline V3 mk(float a) { return {a, a, a}; }
inline V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 mul(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline V3 muls(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }  // Vector3*float
inline V3 divs(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }  // Vector3/float :65
inline V3 neg(V3 a) { return {-a.x, -a.y, -a.z}; }
inline float dot(V3 a, V3 b) { return (a.x * b.x) + (a.y * b.y) + (a.z * b.z); }  // :106
inline V3 cross(V3 a, V3 b) {                                                     // :109
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline float length(V3 a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }  // sqrtf
inline V3 normalize(V3 a) { return divs(a, length(a)); }                             // :114
inline bool is_zero(V3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }
inline float comp(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

struct Ray {  // HW2/Ray.h:5-13
  V3 o, d;
  bool in_medium;
};
inline V3 point_at(const Ray& r, float t) { return add(r.o, muls(r.d, t)); }  // o + (t*d)

struct Box {  // HW2/Bounding_box.h
  V3 lo{kInf, kInf, kInf}, hi{-kInf, -kInf, -kInf}, center{0, 0, 0};
};
inline Box box_from(V3 lo, V3 hi) {  // Bounding_box(min, max): center((max+min)/2)
  Box b;
  b.lo = lo;
  b.hi = hi;
  b.center = divs(add(hi, lo), 2.0f);
  return b;
}
inline void expand(Box& b, const Box& o) {  // HW2/bounding_box.cpp:2-13
  b.lo = {std::fmin(b.lo.x, o.lo.x), std::fmin(b.lo.y, o.lo.y), std::fmin(b.lo.z, o.lo.z)};
  b.hi = {std::fmax(b.hi.x, o.hi.x), std::fmax(b.hi.y, o.hi.y), std::fmax(b.hi.z, o.hi.z)};
  b.center = divs(add(b.hi, b.lo), 2.0f);
}
// HW2/bounding_box.cpp:15-35: slab test with true division and the |d_i| < 1e-6 axis skip.
inline float box_intersect(const Box& b, const Ray& r) {
  float tmin = -kInf, tmax = kInf;
  for (int i = 0; i < 3; i++) {
    const float d = comp(r.d, i), o = comp(r.o, i);
    if (std::fabs(d) < kEps) continue;
    float t0 = (comp(b.lo, i) - o) / d;
    float t1 = (comp(b.hi, i) - o) / d;
    if (d < 0) std::swap(t0, t1);
    if (t0 > tmin) tmin = t0;
    if (t1 < tmax) tmax = t1;
    if (tmin > tmax) return kInf;
  }
  return tmin > 0.0f ? tmin : tmax;
}

struct Material {  // HW2/Material.h
  V3 ambient, diffuse, specular, mirror, transparency;
  float refraction_index, phong_exponent;
};
struct Light {
  V3 position, intensity;
};
struct Camera {  // HW2/Camera.h:10-35
  V3 e, u, v, w, s_u, s_v, top_left;
  int width, height, samples;
};

// ------------------------------------------------------------------ shapes + BVH
enum Kind { kBVH, kMesh, kTri, kSphere };
struct Shape {
  Kind kind;
  Box box;
  int left = -1, right = -1;  // kBVH children; kMesh: left = its bvh root
  int i0 = 0, i1 = 0, i2 = 0;  // kTri vertex indices (0-based)
  V3 normal{0, 0, 0};          // kTri flat normal
  V3 center{0, 0, 0};          // kSphere
  float radius = 0;
  int material = -1;
};

struct Hit {
  float t;
  int shape;
  V3 normal;
};

struct Counters {
  long long box = 0, prim = 0;
};

struct Scene {
  V3 background{0, 0, 0};
  float shadow_eps = 0.001f;
  int max_depth = 0;
  V3 ambient{0, 0, 0};
  std::vector<Camera> cameras;
  std::vector<Light> lights;
  std::vector<Material> materials;
  std::vector<V3> verts;
  std::vector<Shape> shapes;
  int root = -1;

  // HW2/Triangle.cpp:35-65 (Cramer's rule; determinant = Triangle.h:33-38)
  static float det3(V3 c1, V3 c2, V3 c3) {
    return c1.x * (c2.y * c3.z - c3.y * c2.z) + c2.x * (c3.y * c1.z - c1.y * c3.z) +
           c3.x * (c1.y * c2.z - c2.y * c1.z);
  }
  bool tri_intersect(const Shape& s, int id, const Ray& r, Hit& h) const {
    const V3 v0 = verts[s.i0], v1 = verts[s.i1], v2 = verts[s.i2];
    const V3 a1 = sub(v0, v1), a2 = sub(v0, v2);
    const float det = det3(a1, a2, r.d);
    if (det == 0.0f) return false;
    const V3 b = divs(sub(v0, r.o), det);
    const float beta = det3(b, a2, r.d);
    if (beta < 0.0f || beta > 1.0f) return false;
    const float gamma = det3(a1, b, r.d);
    if (gamma < 0.0f || beta + gamma > 1.0f) return false;
    const float t = det3(a1, a2, b);
    if (t > 0.0f) {
      h.t = t;
      h.shape = id;
      h.normal = s.normal;
      return true;
    }
    return false;
  }
  // HW2/Sphere.h:26-52 — returns true even for a negative root.
  static bool sphere_intersect(const Shape& s, int id, const Ray& r, Hit& h) {
    const V3 co = sub(r.o, s.center);
    const float a = dot(r.d, r.d);
    const float b = 2 * dot(r.d, co);
    const float c = dot(co, co) - s.radius * s.radius;
    const float disc = b * b - 4 * a * c;
    if (disc < -kEps) return false;
    if (disc < kEps) {
      h.t = -b / (2 * a);
    } else {
      const float sq = (float)::sqrt((double)disc);
      const float t1 = (-b + sq) / (2 * a);
      const float t2 = (-b - sq) / (2 * a);
      h.t = t2 < .0 ? t1 : t2;
    }
    h.normal = normalize(sub(point_at(r, h.t), s.center));
    h.shape = id;
    return true;
  }
  // Shape::intersect dispatch; BVH::intersect = HW2/Bounding_volume_hierarchy.cpp:31-55.
  bool intersect(int id, const Ray& r, Hit& h, Counters& c) const {
    const Shape& s = shapes[id];
    switch (s.kind) {
      case kTri:
        c.prim++;
        return tri_intersect(s, id, r, h);
      case kSphere:
        c.prim++;
        return sphere_intersect(s, id, r, h);
      case kMesh:
        return intersect(s.left, r, h, c);
      case kBVH: {
        c.box++;
        const float bt = box_intersect(s.box, r);
        if (bt < 0.0f || bt == kInf) return false;
        bool any = false;
        Hit lh{kInf, -1, {0, 0, 0}};
        if (intersect(s.left, r, lh, c) && lh.t > 0.0f && lh.t < h.t) {
          h = lh;
          any = true;
        }
        Hit rh{kInf, -1, {0, 0, 0}};
        if (intersect(s.right, r, rh, c) && rh.t > 0.0f && rh.t < h.t) {
          any = true;
          h = rh;
        }
        return any;
      }
    }
    return false;
  }

  // HW2/Scene.cpp:72-86
  static bool refract(V3 dir, V3 n, float idx, V3& out) {
    const float n_ratio = 1 / idx;
    const float cos_t = dot(neg(dir), n);
    const float delta = 1 - (n_ratio) * (n_ratio) * (1 - (cos_t * cos_t));
    if (delta < 0.0f) return false;
    out = normalize(sub(muls(add(dir, muls(n, cos_t)), n_ratio),
                        muls(n, (float)::sqrt((double)delta))));
    return true;
  }

  // HW2/Scene.cpp:88-196
  V3 trace(const Ray& ray, int depth, Counters* ctr, cpuref_stats* st) const {
    V3 color{0, 0, 0};
    Hit hd{kInf, -1, {0, 0, 0}};
    const int kind = depth == max_depth ? 0 : 2;
    if (!intersect(root, ray, hd, ctr[kind])) {
      if (max_depth == depth) return background;
      return color;
    }
    if (kind == 0) st->primary_hits++;
    const V3 p = point_at(ray, hd.t);
    const Material& m = materials[shapes[hd.shape].material];
    const V3 w0 = normalize(sub(ray.o, p));
    const V3 n = hd.normal;
    if (!ray.in_medium) {
      color = add(color, mul(m.ambient, ambient));
      for (const Light& L : lights) {
        const V3 ld = sub(L.position, p);
        const V3 wi = normalize(ld);
        const float dist = length(ld);
        Ray sr{add(p, muls(wi, shadow_eps)), wi, false};
        Hit sh{kInf, -1, {0, 0, 0}};
        st->shadow_rays++;
        intersect(root, sr, sh, ctr[1]);
        if (sh.t < (dist - shadow_eps) && sh.t > 0.0f) continue;
        const float d2 = dist * dist;
        const float cos_d = dot(n, wi);
        color = add(color, divs(muls(mul(m.diffuse, L.intensity), cos_d), d2));
        const float cos_s = (float)std::fmax(0.0, (double)dot(n, normalize(add(w0, wi))));
        const float pw = (float)::pow((double)cos_s, (double)m.phong_exponent);
        color = add(color, divs(muls(mul(m.specular, L.intensity), pw), d2));
      }
    }
    if (!is_zero(m.mirror) && depth > 0) {  // :141-146
      const V3 wr = normalize(sub(muls(n, 2 * dot(n, w0)), w0));
      Ray mr{add(p, muls(wr, shadow_eps)), wr, false};
      st->secondary_rays++;
      color = add(color, mul(m.mirror, trace(mr, depth - 1, ctr, st)));
    }
    if (!is_zero(m.transparency) && depth > 0) {  // :149-194
      const V3 wr = normalize(sub(muls(n, 2 * dot(n, w0)), w0));
      V3 td{0, 0, 0};
      float cos_t = 0.0f;
      V3 k = mk(0.0f);
      const V3 dn = normalize(ray.d);
      const float idx = m.refraction_index;
      bool tir = false, entering;
      if (dot(dn, n) < 0.0f) {
        refract(dn, n, idx, td);
        cos_t = dot(neg(dn), n);
        k = mk(1.0f);
        entering = true;
      } else {
        const V3 T = m.transparency;
        const float t = hd.t;
        k.x = (float)::exp(-::log((double)T.x) * (double)t);
        k.y = (float)::exp(-::log((double)T.y) * (double)t);
        k.z = (float)::exp(-::log((double)T.z) * (double)t);
        entering = false;
        if (refract(dn, neg(n), 1.0f / idx, td)) {
          cos_t = dot(td, n);
        } else {
          tir = true;
        }
      }
      if (tir) {
        Ray rr{add(p, muls(wr, shadow_eps)), wr, true};
        st->secondary_rays++;
        color = add(color, mul(k, trace(rr, depth - 1, ctr, st)));
      } else {
        const float r0 = (idx - 1) * (idx - 1) / ((idx + 1) * (idx + 1));
        const float r = (float)((double)r0 + (double)(1 - r0) * ::pow((double)(1 - cos_t), 5.0));
        Ray rr{add(p, muls(wr, shadow_eps)), wr, !entering};
        Ray tr{add(p, muls(td, shadow_eps)), td, entering};
        st->secondary_rays += 2;
        const V3 a = muls(trace(rr, depth - 1, ctr, st), r);
        const V3 b = muls(trace(tr, depth - 1, ctr, st), 1 - r);
        color = add(color, mul(k, add(a, b)));
      }
    }
    return color;
  }

  // Camera::calculate_ray_at (HW2/Camera.h:30-35): (x + 0.5) is a double add, narrowed back
  // to float by Vector3 operator*(float, const Vector3&).
  // calculate_ray_at(float x, float y) for an MSAA sample: the caller passes
  // i + sample_x - 0.5 (a double narrowed to the float parameter, HW2/Scene.cpp:47-48).
  Ray primary_f(const Camera& c, float x, float y) const {
    const float fx = (float)((double)x + 0.5);
    const float fy = (float)((double)y + 0.5);
    const V3 s = sub(add(c.top_left, muls(c.s_u, fx)), muls(c.s_v, fy));
    return Ray{c.e, normalize(sub(s, c.e)), false};
  }

  Ray primary(const Camera& c, int x, int y) const {
    const float fx = (float)((double)(float)x + 0.5);
    const float fy = (float)((double)(float)y + 0.5);
    const V3 s = sub(add(c.top_left, muls(c.s_u, fx)), muls(c.s_v, fy));
    return Ray{c.e, normalize(sub(s, c.e)), false};
  }
};

// ------------------------------------------------------------------ BVH build
// HW2/Bounding_volume_hierarchy.cpp:3-29 + create_bvh (Bounding_volume_hierarchy.h:9-18).
int build_bvh(Scene& sc, std::vector<int>& objs) {
  const int n = (int)objs.size();
  if (n == 0) return -1;
  if (n == 1) return objs[0];
  struct Job {
    int start, end, dim, node;
  };
  std::vector<Job> stack;
  auto make_node = [&](int start, int end, int dim) {
    Shape s;
    s.kind = kBVH;
    for (int i = start; i < end; i++) expand(s.box, sc.shapes[objs[i]].box);
    sc.shapes.push_back(s);
    const int id = (int)sc.shapes.size() - 1;
    stack.push_back({start, end, dim, id});
    return id;
  };
  const int root = make_node(0, n, 0);
  while (!stack.empty()) {
    Job j = stack.back();
    stack.pop_back();
    const float center = comp(sc.shapes[j.node].box.center, j.dim);
    int mid = j.start;
    for (int i = j.start; i < j.end; i++)
      if (comp(sc.shapes[objs[i]].box.center, j.dim) < center) std::swap(objs[i], objs[mid++]);
    if (mid == j.start || mid == j.end) mid = j.start + ((j.end - j.start) / 2);
    const int nd = (j.dim + 1) % 3;
    int l, r;
    if (j.start + 1 == mid)
      l = objs[j.start];
    else
      l = make_node(j.start, mid, nd);
    if (mid + 1 == j.end)
      r = objs[mid];
    else
      r = make_node(mid, j.end, nd);
    sc.shapes[j.node].left = l;
    sc.shapes[j.node].right = r;
  }
  return root;
}

// ------------------------------------------------------------------ XML (appendix B)
// oracle/xml_lite.h: Elem + XmlParser (tinyxml2 GetText() semantics).

const char* text_of(const Elem* e, const char* what) {
  if (!e || !e->has_text) throw std::runtime_error(std::string("missing text for ") + what);
  return e->text.c_str();
}

Camera make_camera(V3 up, V3 gaze, V3 pos, int samples, float l, float r, float b, float t,
                   float dist, int w, int h) {
  Camera c;
  c.e = pos;
  c.samples = samples;
  c.width = w;
  c.height = h;
  c.w = neg(normalize(gaze));
  c.u = normalize(cross(normalize(up), c.w));
  c.v = normalize(cross(c.w, c.u));
  // e - w*distance + left*u + top*v, left to right (HW2/Camera.h:23-24)
  c.top_left = add(add(sub(c.e, muls(c.w, dist)), muls(c.u, l)), muls(c.v, t));
  c.s_u = muls(c.u, (r - l) / w);
  c.s_v = muls(c.v, (t - b) / h);
  return c;
}

// HW2/Scene.cpp:198-451, with one shared stringstream as the reference uses.
void load_scene(Scene& sc, const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("Error: The xml file cannot be loaded.");
  std::stringstream buf;
  buf << f.rdbuf();
  const std::string txt = buf.str();
  XmlParser xp(txt);
  xp.skip_misc();
  std::unique_ptr<Elem> root = xp.element();
  std::stringstream st;
  auto feed = [&](const Elem* e, const char* def, const char* what) {
    if (e) st << text_of(e, what) << std::endl;
    else st << def << std::endl;
  };
  feed(root->child("BackgroundColor"), "0 0 0", "BackgroundColor");
  st >> sc.background.x >> sc.background.y >> sc.background.z;
  feed(root->child("ShadowRayEpsilon"), "0.001", "ShadowRayEpsilon");
  st >> sc.shadow_eps;
  feed(root->child("MaxRecursionDepth"), "0", "MaxRecursionDepth");
  st >> sc.max_depth;
  const Elem* cams = root->child("Cameras");
  if (!cams) throw std::runtime_error("missing Cameras");
  for (const Elem* c : cams->all("Camera")) {
    st << text_of(c->child("Position"), "Position") << std::endl;
    st << text_of(c->child("Gaze"), "Gaze") << std::endl;
    st << text_of(c->child("Up"), "Up") << std::endl;
    st << text_of(c->child("NearPlane"), "NearPlane") << std::endl;
    st << text_of(c->child("NearDistance"), "NearDistance") << std::endl;
    st << text_of(c->child("ImageResolution"), "ImageResolution") << std::endl;
    if (c->child("NumSamples")) st << text_of(c->child("NumSamples"), "NumSamples") << std::endl;
    else st << 1 << std::endl;
    st << text_of(c->child("ImageName"), "ImageName") << std::endl;
    V3 pos, up, gaze;
    float nd, l, r, b, t;
    int w, h, ns;
    std::string name;
    st >> pos.x >> pos.y >> pos.z >> gaze.x >> gaze.y >> gaze.z >> up.x >> up.y >> up.z;
    st >> l >> r >> b >> t >> nd >> w >> h >> ns;
    ns = (int)::sqrt((double)ns);
    if (ns <= 0) ns = 1;
    st >> name;
    sc.cameras.push_back(make_camera(up, gaze, pos, ns, l, r, b, t, nd, w, h));
  }
  const Elem* lights = root->child("Lights");
  if (!lights) throw std::runtime_error("missing Lights");
  st << text_of(lights->child("AmbientLight"), "AmbientLight") << std::endl;
  st >> sc.ambient.x >> sc.ambient.y >> sc.ambient.z;
  for (const Elem* pl : lights->all("PointLight")) {
    st << text_of(pl->child("Position"), "Position") << std::endl;
    st << text_of(pl->child("Intensity"), "Intensity") << std::endl;
    Light L;
    st >> L.position.x >> L.position.y >> L.position.z;
    st >> L.intensity.x >> L.intensity.y >> L.intensity.z;
    sc.lights.push_back(L);
  }
  const Elem* mats = root->child("Materials");
  if (!mats) throw std::runtime_error("missing Materials");
  for (const Elem* m : mats->all("Material")) {
    feed(m->child("AmbientReflectance"), "0 0 0", "AmbientReflectance");
    feed(m->child("DiffuseReflectance"), "0 0 0", "DiffuseReflectance");
    feed(m->child("SpecularReflectance"), "0 0 0", "SpecularReflectance");
    feed(m->child("MirrorReflectance"), "0 0 0", "MirrorReflectance");
    feed(m->child("PhongExponent"), "1", "PhongExponent");
    feed(m->child("Transparency"), "0 0 0", "Transparency");
    feed(m->child("RefractionIndex"), "1.0", "RefractionIndex");
    Material M;
    st >> M.ambient.x >> M.ambient.y >> M.ambient.z >> M.diffuse.x >> M.diffuse.y >>
        M.diffuse.z >> M.specular.x >> M.specular.y >> M.specular.z >> M.mirror.x >>
        M.mirror.y >> M.mirror.z >> M.phong_exponent >> M.transparency.x >>
        M.transparency.y >> M.transparency.z >> M.refraction_index;
    sc.materials.push_back(M);
  }
  st << text_of(root->child("VertexData"), "VertexData") << std::endl;
  V3 v;
  while (!(st >> v.x).eof()) {
    st >> v.y >> v.z;
    sc.verts.push_back(v);
  }
  st.clear();
  const Elem* objects = root->child("Objects");
  if (!objects) throw std::runtime_error("missing Objects");
  auto check_mat = [&](int m) {
    if (m < 0 || m >= (int)sc.materials.size()) throw std::runtime_error("bad material id");
  };
  auto check_v = [&](int i) {
    if (i < 0 || i >= (int)sc.verts.size()) throw std::runtime_error("bad vertex index");
  };
  auto add_tri = [&](int a, int b, int c, int mat) {  // HW2/Triangle.cpp:4-34
    check_v(a);
    check_v(b);
    check_v(c);
    Shape s;
    s.kind = kTri;
    s.i0 = a;
    s.i1 = b;
    s.i2 = c;
    s.material = mat;
    const V3 v0 = sc.verts[a], v1 = sc.verts[b], v2 = sc.verts[c];
    s.normal = normalize(cross(sub(v1, v0), sub(v2, v0)));
    V3 lo = v0, hi = v0;
    lo = {std::fmin(lo.x, v1.x), std::fmin(lo.y, v1.y), std::fmin(lo.z, v1.z)};
    hi = {std::fmax(hi.x, v1.x), std::fmax(hi.y, v1.y), std::fmax(hi.z, v1.z)};
    lo = {std::fmin(lo.x, v2.x), std::fmin(lo.y, v2.y), std::fmin(lo.z, v2.z)};
    hi = {std::fmax(hi.x, v2.x), std::fmax(hi.y, v2.y), std::fmax(hi.z, v2.z)};
    s.box = box_from(lo, hi);
    sc.shapes.push_back(s);
    return (int)sc.shapes.size() - 1;
  };
  std::vector<int> top;
  for (const Elem* m : objects->all("Mesh")) {
    st << text_of(m->child("Material"), "Material") << std::endl;
    int mat;
    st >> mat;
    mat--;
    check_mat(mat);
    st << text_of(m->child("Faces"), "Faces") << std::endl;
    std::vector<int> tris;
    int a, b, c;
    while (!(st >> a).eof()) {
      st >> b >> c;
      tris.push_back(add_tri(a - 1, b - 1, c - 1, mat));
    }
    st.clear();
    if (tris.empty()) throw std::runtime_error("mesh without faces");
    const int bvh = build_bvh(sc, tris);
    Shape ms;
    ms.kind = kMesh;
    ms.left = bvh;
    ms.material = mat;
    ms.box = sc.shapes[bvh].box;
    sc.shapes.push_back(ms);
    top.push_back((int)sc.shapes.size() - 1);
  }
  st.clear();
  for (const Elem* t : objects->all("Triangle")) {
    int mat, a, b, c;
    st << text_of(t->child("Material"), "Material") << std::endl;
    st >> mat;
    mat--;
    check_mat(mat);
    st << text_of(t->child("Indices"), "Indices") << std::endl;
    st >> a >> b >> c;
    top.push_back(add_tri(a - 1, b - 1, c - 1, mat));
  }
  for (const Elem* s : objects->all("Sphere")) {
    int mat, ci;
    float rad;
    st << text_of(s->child("Material"), "Material") << std::endl;
    st >> mat;
    mat--;
    check_mat(mat);
    st << text_of(s->child("Center"), "Center") << std::endl;
    st >> ci;
    check_v(ci - 1);
    st << text_of(s->child("Radius"), "Radius") << std::endl;
    st >> rad;
    Shape sp;
    sp.kind = kSphere;
    sp.center = sc.verts[ci - 1];
    sp.radius = rad;
    sp.material = mat;
    sp.box = box_from(sub(sp.center, mk(rad)), add(sp.center, mk(rad)));
    sc.shapes.push_back(sp);
    top.push_back((int)sc.shapes.size() - 1);
  }
  if (top.empty()) throw std::runtime_error("scene has no objects");
  sc.root = build_bvh(sc, top);
}

unsigned fbits(float f) {
  unsigned u;
  std::memcpy(&u, &f, 4);
  return u;
}

void dump(const Scene& sc, int id, FILE* f) {
  const Shape& s = sc.shapes[id];
  switch (s.kind) {
    case kBVH:
      std::fprintf(f, "N %08x %08x %08x %08x %08x %08x\n", fbits(s.box.lo.x), fbits(s.box.lo.y),
                   fbits(s.box.lo.z), fbits(s.box.hi.x), fbits(s.box.hi.y), fbits(s.box.hi.z));
      dump(sc, s.left, f);
      dump(sc, s.right, f);
      break;
    case kMesh:
      std::fprintf(f, "M\n");
      dump(sc, s.left, f);
      break;
    case kTri:
      std::fprintf(f, "T %d %d %d %d\n", s.i0, s.i1, s.i2, s.material);
      break;
    case kSphere:
      std::fprintf(f, "S %08x %08x %08x %08x %d\n", fbits(s.center.x), fbits(s.center.y),
                   fbits(s.center.z), fbits(s.radius), s.material);
      break;
  }
}

}  // namespace

// ------------------------------------------------------------------ MSAA (HW2/Scene.cpp:32-69)
// std::default_random_engine is libstdc++'s minstd_rand0 (x <- 16807 x mod 2^31-1); the
// reference seeds it per pixel from system_clock (non-deterministic), we from msaa_seed().
// uniform_real_distribution<float>(0, 1) = generate_canonical<float, 24> with one draw:
// float(u - 1) / float(2147483646.0L) (= 2^31), clamped below 1.
constexpr uint64_t kMinstdM = 2147483647ull;

uint64_t msaa_seed(uint64_t base, uint64_t pixel) {  // splitmix64 of (base, pixel)
  uint64_t z = base + 0x9E3779B97F4A7C15ull * (pixel + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Minstd {
  uint64_t x;
  explicit Minstd(uint64_t seed) {
    x = seed % kMinstdM;
    if (x == 0) x = 1;
  }
  uint64_t next() {
    x = (x * 16807ull) % kMinstdM;
    return x;
  }
  float uniform01() {
    const float sum = (float)(next() - 1) * 1.0f;
    const float tmp = (float)(1.0L * (2147483646.0L));
    float r = sum / tmp;
    if (r >= 1.0f) r = std::nextafter(1.0f, 0.0f);
    return r * (1.0f - 0.0f) + 0.0f;
  }
};

inline float gaussian_filter(float x, float y, float sigma) {  // HW2/Scene.cpp:12-14
  return (float)(::exp((double)(-(x * x + y * y) / (2 * sigma * sigma))) / (2 * M_PI * sigma));
}

struct cpuref_scene {
  Scene sc;
};

extern "C" {

cpuref_scene* cpuref_load(const char* xml_path, char* err, int errlen) {
  auto* s = new cpuref_scene;
  try {
    load_scene(s->sc, xml_path);
  } catch (const std::exception& e) {
    if (err && errlen > 0) std::snprintf(err, (size_t)errlen, "%s", e.what());
    delete s;
    return nullptr;
  }
  return s;
}

void cpuref_free(cpuref_scene* s) { delete s; }

int cpuref_num_cameras(const cpuref_scene* s) { return (int)s->sc.cameras.size(); }
int cpuref_num_lights(const cpuref_scene* s) { return (int)s->sc.lights.size(); }

int cpuref_camera_info(const cpuref_scene* s, int cam, int* w, int* h, int* ns) {
  if (cam < 0 || cam >= (int)s->sc.cameras.size()) return -1;
  const Camera& c = s->sc.cameras[cam];
  if (w) *w = c.width;
  if (h) *h = c.height;
  if (ns) *ns = c.samples;
  return 0;
}

int cpuref_render(const cpuref_scene* s, int cam, int starting_row, int row_stride, int threads,
                  float* out, cpuref_stats* stats) {
  if (cam < 0 || cam >= (int)s->sc.cameras.size() || row_stride < 1 || starting_row < 0)
    return -1;
  const Scene& sc = s->sc;
  const Camera& c = sc.cameras[cam];
  if (c.samples != 1) return -2;  // MSAA: cpuref_render_msaa
  if (threads < 1) threads = 1;
  if (c.height < threads) threads = 1;
  std::vector<cpuref_stats> st(threads);
  std::vector<Counters> ctr(threads * 3);
  auto work = [&](int ti, int first, int step) {
    cpuref_stats& S = st[ti];
    std::memset(&S, 0, sizeof S);
    Counters* C = &ctr[ti * 3];
    for (int j = first; j < c.height; j += step)
      for (int i = 0; i < c.width; i++) {
        const V3 col = sc.trace(sc.primary(c, i, j), sc.max_depth, C, &S);
        S.primary_rays++;
        // Pixel::add_color(color, 1) on a zeroed pixel (HW2/Pixel.h:12-16)
        float* o = out + 3 * ((size_t)j * c.width + i);
        o[0] = 0.0f + col.x * 1.0f;
        o[1] = 0.0f + col.y * 1.0f;
        o[2] = 0.0f + col.z * 1.0f;
      }
  };
  if (threads == 1) {
    work(0, starting_row, row_stride);
  } else {
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; t++)
      pool.emplace_back(work, t, starting_row + t * row_stride, row_stride * threads);
    for (auto& t : pool) t.join();
  }
  if (stats) {
    std::memset(stats, 0, sizeof *stats);
    for (int t = 0; t < threads; t++) {
      stats->primary_rays += st[t].primary_rays;
      stats->shadow_rays += st[t].shadow_rays;
      stats->secondary_rays += st[t].secondary_rays;
      stats->primary_hits += st[t].primary_hits;
      for (int k = 0; k < 3; k++) {
        stats->box_tests[k] += ctr[t * 3 + k].box;
        stats->prim_tests[k] += ctr[t * 3 + k].prim;
      }
    }
  }
  return 0;
}

int cpuref_render_msaa(const cpuref_scene* s, int cam, unsigned long long seed, int threads,
                       float* out, cpuref_stats* stats) {
  if (cam < 0 || cam >= (int)s->sc.cameras.size()) return -1;
  const Scene& sc = s->sc;
  const Camera& c = sc.cameras[cam];
  const int n = c.samples, W = c.width, H = c.height, S = n * n;
  if (threads < 1) threads = 1;
  // phase 1: every sample's colour (order-free), phase 2: the splat in the single-threaded
  // reference order (source rows, source columns, samples x-major; neighbours j-1..j+1,
  // i-1..i+1), so the per-pixel float sums are deterministic.
  std::vector<float> col((size_t)W * H * S * 3), sx((size_t)W * H * S), sy((size_t)W * H * S);
  std::vector<cpuref_stats> st(threads);
  std::vector<Counters> ctr(threads * 3);
  auto work = [&](int ti) {
    cpuref_stats& St = st[ti];
    std::memset(&St, 0, sizeof St);
    Counters* C = &ctr[ti * 3];
    for (int j = ti; j < H; j += threads)
      for (int i = 0; i < W; i++) {
        const size_t pix = (size_t)j * W + i;
        Minstd gen(msaa_seed(seed, pix));
        for (int x = 0; x < n; x++)
          for (int y = 0; y < n; y++) {
            const float ex = gen.uniform01();
            const float ey = gen.uniform01();
            const float smx = (x + ex) / n;
            const float smy = (y + ey) / n;
            const V3 color = sc.trace(sc.primary_f(c, (float)((double)(i + smx) - 0.5),
                                                   (float)((double)(j + smy) - 0.5)),
                                      sc.max_depth, C, &St);
            St.primary_rays++;
            const size_t k = pix * S + (size_t)(x * n + y);
            col[3 * k] = color.x;
            col[3 * k + 1] = color.y;
            col[3 * k + 2] = color.z;
            sx[k] = smx;
            sy[k] = smy;
          }
      }
  };
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; t++) pool.emplace_back(work, t);
  for (auto& t : pool) t.join();
  std::vector<float> acc((size_t)W * H * 3, 0.0f), wsum((size_t)W * H, 0.0f);
  for (int j = 0; j < H; j++)
    for (int i = 0; i < W; i++)
      for (int k = 0; k < S; k++) {
        const size_t src = ((size_t)j * W + i) * S + k;
        const V3 color{col[3 * src], col[3 * src + 1], col[3 * src + 2]};
        for (int aj = j - 1; aj < j + 2; aj++) {
          if (aj < 0 || aj >= H) continue;
          for (int ai = i - 1; ai < i + 2; ai++) {
            if (ai < 0 || ai >= W) continue;
            const float dx = (i + sx[src]) - (ai + 0.5f);
            const float dy = (j + sy[src]) - (aj + 0.5f);
            const float w = gaussian_filter(dx, dy, 1.0f / 3.0f);
            float* a = &acc[3 * ((size_t)aj * W + ai)];  // Pixel::add_color(color, w)
            const V3 cw = muls(color, w);
            a[0] += cw.x;
            a[1] += cw.y;
            a[2] += cw.z;
            wsum[(size_t)aj * W + ai] += w;
          }
        }
      }
  for (size_t p = 0; p < (size_t)W * H; p++) {  // Pixel::get_color: color / weight
    out[3 * p] = acc[3 * p] / wsum[p];
    out[3 * p + 1] = acc[3 * p + 1] / wsum[p];
    out[3 * p + 2] = acc[3 * p + 2] / wsum[p];
  }
  if (stats) {
    std::memset(stats, 0, sizeof *stats);
    for (int t = 0; t < threads; t++) {
      stats->primary_rays += st[t].primary_rays;
      stats->shadow_rays += st[t].shadow_rays;
      stats->secondary_rays += st[t].secondary_rays;
      stats->primary_hits += st[t].primary_hits;
      for (int k = 0; k < 3; k++) {
        stats->box_tests[k] += ctr[t * 3 + k].box;
        stats->prim_tests[k] += ctr[t * 3 + k].prim;
      }
    }
  }
  return 0;
}

void cpuref_minstd_uniform(unsigned long long seed, int count, float* out) {
  Minstd g(seed);
  for (int k = 0; k < count; k++) out[k] = g.uniform01();
}

unsigned long long cpuref_msaa_seed(unsigned long long base, unsigned long long pixel) {
  return msaa_seed(base, pixel);
}

int cpuref_dump_bvh(const cpuref_scene* s, const char* path) {
  FILE* f = std::fopen(path, "w");
  if (!f) return -1;
  dump(s->sc, s->sc.root, f);
  std::fclose(f);
  return 0;
}

int cpuref_primary_records(const cpuref_scene* s, int cam, float* out8) {
  if (cam < 0 || cam >= (int)s->sc.cameras.size()) return -1;
  const Scene& sc = s->sc;
  const Camera& c = sc.cameras[cam];
  Counters ctr;
  for (int j = 0; j < c.height; j++)
    for (int i = 0; i < c.width; i++) {
      const Ray r = sc.primary(c, i, j);
      Hit h{kInf, -1, {0, 0, 0}};
      const bool hit = sc.intersect(sc.root, r, h, ctr);
      float* o = out8 + 8 * ((size_t)j * c.width + i);
      o[0] = r.d.x;
      o[1] = r.d.y;
      o[2] = r.d.z;
      o[3] = hit ? h.t : 0.f;
      o[4] = hit ? h.normal.x : 0.f;
      o[5] = hit ? h.normal.y : 0.f;
      o[6] = hit ? h.normal.z : 0.f;
      o[7] = hit ? 1.f : 0.f;
    }
  return 0;
}

}  // extern "C"
