// PPM scene ingest + acceleration-structure build (host, untimed).
//
// Mirrors PPM/src/Scene.cpp:373-505 and the loaders it calls (Camera.cpp, Material.cpp,
// Transformation.cpp, Point_light.cpp, Sphere.cpp, Mesh.cpp): the same tags, defaults,
// per-loader std::stringstream parsing (so every float gets libstdc++'s bits), the same
// fp32 matrix arithmetic (Matrix4x4.cpp) and the same median-split BVH (BVH.cpp:3-28), built
// separately per mesh and over the top-level objects (spheres, then one Mesh_instance per
// mesh, then the <MeshInstance>s), then flattened in DFS preorder.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <sstream>
#include <stdexcept>
#include <string>

#include "ppm_host.h"
#include "xml_dom.h"

namespace ppm {
namespace {

using rt::Node;
using rt::node_text;

constexpr float kInf = std::numeric_limits<float>::infinity();

struct Vec {
  float x = 0, y = 0, z = 0;
};
Vec vec(float a, float b, float c) { return Vec{a, b, c}; }
Vec operator+(Vec a, Vec b) { return vec(a.x + b.x, a.y + b.y, a.z + b.z); }
Vec operator-(Vec a, Vec b) { return vec(a.x - b.x, a.y - b.y, a.z - b.z); }
Vec operator*(Vec a, float s) { return vec(a.x * s, a.y * s, a.z * s); }
Vec operator/(Vec a, float s) { return vec(a.x / s, a.y / s, a.z / s); }
Vec cross(Vec a, Vec b) {
  return vec(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
float len(Vec a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
Vec unit(Vec a) { return a / len(a); }
float lo_of(float a, float b) { return (b < a) ? b : a; }  // std::min(a, b)
float hi_of(float a, float b) { return (a < b) ? b : a; }  // std::max(a, b)
float comp(Vec v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }

// ------------------------------------------------------------------ 4x4 matrices (Matrix4x4.cpp)
struct Mat {
  float a[4][4];
  static Mat zero() {
    Mat m;
    std::memset(m.a, 0, sizeof m.a);
    return m;
  }
  static Mat identity() {
    Mat m = zero();
    for (int i = 0; i < 4; i++) m.a[i][i] = 1.0f;
    return m;
  }
  Mat operator*(const Mat& r) const {  // result[i][j] += a[i][k] * r[k][j], k ascending
    Mat o = zero();
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 4; j++)
        for (int k = 0; k < 4; k++) o.a[i][j] += a[i][k] * r.a[k][j];
    return o;
  }
  Mat transposed() const {
    Mat t;
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 4; j++) t.a[i][j] = a[j][i];
    return t;
  }
  Vec point(Vec v) const {  // multiply(v, false)
    float r[3];
    for (int i = 0; i < 3; i++) {
      r[i] = a[i][3];
      r[i] += a[i][0] * v.x;
      r[i] += a[i][1] * v.y;
      r[i] += a[i][2] * v.z;
    }
    return vec(r[0], r[1], r[2]);
  }
  bool identity_p() const {
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 4; j++)
        if (a[i][j] != (i == j ? 1.0f : 0.0f)) return false;
    return true;
  }
  // Matrix4x4::invert_matrix: cofactors as written there, det = 1/det, inv * det.
  bool inverse(Mat& out) const {
    float m[16], c[16];
    for (int k = 0; k < 16; k++) m[k] = a[k / 4][k % 4];
    c[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] +
           m[9] * m[7] * m[14] + m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
    c[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] -
           m[8] * m[7] * m[14] - m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
    c[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] +
           m[8] * m[7] * m[13] + m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
    c[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] -
            m[8] * m[6] * m[13] - m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
    c[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] -
           m[9] * m[3] * m[14] - m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
    c[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] +
           m[8] * m[3] * m[14] + m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
    c[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] -
           m[8] * m[3] * m[13] - m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
    c[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] +
            m[8] * m[2] * m[13] + m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
    c[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] +
           m[5] * m[3] * m[14] + m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
    c[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] -
           m[4] * m[3] * m[14] - m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
    c[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] +
            m[4] * m[3] * m[13] + m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
    c[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] -
            m[4] * m[2] * m[13] - m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
    c[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] -
           m[5] * m[3] * m[10] - m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
    c[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] +
           m[4] * m[3] * m[10] + m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
    c[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] -
            m[4] * m[3] * m[9] - m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
    c[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] +
            m[4] * m[2] * m[9] + m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
    float det = m[0] * c[0] + m[1] * c[4] + m[2] * c[8] + m[3] * c[12];
    if (det == 0.0f) return false;
    det = 1.0f / det;
    for (int k = 0; k < 16; k++) out.a[k / 4][k % 4] = c[k] * det;
    return true;
  }
};

struct Transform {  // Transformation.h: M, M^-1, (M^-1)^T
  Mat m = Mat::identity(), inv = Mat::identity(), nrm = Mat::identity();
};
Transform from_matrix(const Mat& m) {  // Arbitrary_transformation
  Transform t;
  t.m = m;
  if (!m.inverse(t.inv)) throw std::runtime_error("scene xml: transformation is not invertible");
  t.nrm = t.inv.transposed();
  return t;
}

// ------------------------------------------------------------------ boxes (Bounding_box.cpp)
struct BBox {
  Vec lo = vec(kInf, kInf, kInf), hi = vec(-kInf, -kInf, -kInf), center;
  static BBox of(Vec lo, Vec hi) {
    BBox b;
    b.lo = lo;
    b.hi = hi;
    b.center = (hi + lo) / 2;
    return b;
  }
  void expand(const BBox& o) {
    lo = vec(lo_of(lo.x, o.lo.x), lo_of(lo.y, o.lo.y), lo_of(lo.z, o.lo.z));
    hi = vec(hi_of(hi.x, o.hi.x), hi_of(hi.y, o.hi.y), hi_of(hi.z, o.hi.z));
    center = (hi + lo) / 2.;
  }
};
BBox transformed(const BBox& b, const Mat& m) {  // Bounding_box::apply_transform
  const Vec l = b.lo, h = b.hi;
  const Vec corner[8] = {vec(l.x, l.y, l.z), vec(l.x, l.y, h.z), vec(l.x, h.y, l.z),
                         vec(l.x, h.y, h.z), vec(h.x, l.y, l.z), vec(h.x, l.y, h.z),
                         vec(h.x, h.y, l.z), vec(h.x, h.y, h.z)};
  Vec mn = m.point(corner[0]), mx = mn;
  for (int k = 1; k < 8; k++) {
    const Vec p = m.point(corner[k]);
    mn = vec(lo_of(mn.x, p.x), lo_of(mn.y, p.y), lo_of(mn.z, p.z));
    mx = vec(hi_of(mx.x, p.x), hi_of(mx.y, p.y), hi_of(mx.z, p.z));
  }
  return BBox::of(mn, mx);
}

// ------------------------------------------------------------------ BVH (BVH.cpp:3-28)
// Builds over `items` (permuted in place as the reference swaps its Shape* vector) and
// appends DFS-preorder nodes to `nodes`; returns the root (node index, or ~item for one item).
struct Builder {
  const std::vector<BBox>& boxes;
  std::vector<PNode>& nodes;
  int depth = 0;
  int build(std::vector<int>& items, int start, int end, int axis, int level) {
    BBox box;
    for (int k = start; k < end; k++) box.expand(boxes[items[k]]);
    const float split = comp(box.center, axis);
    int mid = start;
    for (int k = start; k < end; k++)
      if (comp(boxes[items[k]].center, axis) < split) std::swap(items[k], items[mid++]);
    if (mid == start || mid == end) mid = start + ((end - start) / 2);
    const int id = (int)nodes.size();
    PNode n;
    n.lo[0] = box.lo.x, n.lo[1] = box.lo.y, n.lo[2] = box.lo.z;
    n.hi[0] = box.hi.x, n.hi[1] = box.hi.y, n.hi[2] = box.hi.z;
    n.child[0] = n.child[1] = 0;
    nodes.push_back(n);
    depth = std::max(depth, level + 1);
    const int l = start + 1 == mid ? ~items[start] : build(items, start, mid, (axis + 1) % 3, level + 1);
    const int r = mid + 1 == end ? ~items[mid] : build(items, mid, end, (axis + 1) % 3, level + 1);
    nodes[id].child[0] = l;
    nodes[id].child[1] = r;
    return id;
  }
  int create(std::vector<int>& items) {  // BVH::create_bvh
    if (items.empty()) return std::numeric_limits<int>::min();
    if (items.size() == 1) return ~items[0];
    return build(items, 0, (int)items.size(), 0, 0);
  }
};

// ------------------------------------------------------------------ loaders
struct TransformLists {
  std::vector<Transform> scaling, translation, rotation;
};

// "<Transformations>s1 t2 r1</Transformations>": each left-multiplies (Mesh.cpp:38-63).
Mat apply_transformations(std::stringstream& ss, const Node* n, const TransformLists& T, Mat m) {
  if (!n) return m;
  ss.clear();
  ss << node_text(n, "Transformations") << std::endl;
  char type;
  int index;
  while (!(ss >> type).eof()) {
    ss >> index;
    if (ss.fail()) throw std::runtime_error("scene xml: bad <Transformations> list");
    --index;
    const std::vector<Transform>* list = type == 's'   ? &T.scaling
                                         : type == 't' ? &T.translation
                                         : type == 'r' ? &T.rotation
                                                       : nullptr;
    if (!list) continue;
    if (index < 0 || index >= (int)list->size())
      throw std::runtime_error("scene xml: transformation index out of range");
    m = (*list)[index].m * m;
  }
  ss.clear();
  return m;
}

void put3(float* dst, Vec v) {
  dst[0] = v.x;
  dst[1] = v.y;
  dst[2] = v.z;
}

PCamera make_camera(Vec up, Vec gaze, Vec pos, int samples, float l, float r, float b,
                    float t, float dist, int w, int h, bool left_handed) {  // Camera.h:28-45
  const Vec W = unit(gaze) * -1.0f;
  Vec U, V;
  if (left_handed) {
    U = unit(cross(W, unit(up)));
    V = unit(cross(U, W));
  } else {
    U = unit(cross(unit(up), W));
    V = unit(cross(W, U));
  }
  PCamera c;
  put3(c.e, pos);
  put3(c.top_left, ((pos - W * dist) + U * l) + V * t);
  put3(c.s_u, U * ((r - l) / w));
  put3(c.s_v, V * ((t - b) / h));
  c.width = w;
  c.height = h;
  c.samples = samples;
  return c;
}

}  // namespace

void load_ppm_xml(const std::string& path, HostPPM& S) {
  const std::unique_ptr<Node> root = rt::parse_xml_file(path);
  std::stringstream ss;  // Scene.cpp:377: scalars and VertexData share one stream
  auto scalar = [&](const char* tag, const char* fallback) {
    const Node* n = root->first(tag);
    ss << (n ? node_text(n, tag) : fallback) << std::endl;
  };
  scalar("ShadowRayEpsilon", "0.001");
  ss >> S.eps;
  scalar("PhotonCountPerIteration", "8000");
  ss >> S.per_iteration;
  scalar("NumberOfIterations", "1000");
  ss >> S.iterations;
  scalar("MaxRecursionDepth", "20");
  ss >> S.max_depth;
  if (S.max_depth > 20) S.max_depth = 20;  // Scene.cpp:426-429

  if (const Node* cams = root->first("Cameras")) {  // Camera.cpp:4-99
    std::stringstream cs;
    constexpr float deg = M_PI / 180.0f;
    for (const Node* c : cams->each("Camera")) {
      cs << node_text(c->first("Position"), "Position") << std::endl;
      cs << node_text(c->first("Up"), "Up") << std::endl;
      cs << node_text(c->first("NearDistance"), "NearDistance") << std::endl;
      cs << node_text(c->first("ImageResolution"), "ImageResolution") << std::endl;
      const Node* ns_node = c->first("NumSamples");
      cs << (ns_node ? node_text(ns_node, "NumSamples") : "1") << std::endl;
      cs << node_text(c->first("ImageName"), "ImageName") << std::endl;
      Vec pos, up, gaze;
      float dist, l, r, b, t;
      int w, h, ns;
      HostCamera hc;
      cs >> pos.x >> pos.y >> pos.z >> up.x >> up.y >> up.z >> dist >> w >> h >> ns;
      ns = (int)std::sqrt((double)ns);
      if (ns <= 0) ns = 1;
      cs >> hc.image_name;
      const Node* g = c->first("Gaze");
      if (!g) g = c->first("GazePoint");
      const char* type = c->attr("type");
      if (type && std::string(type) == "simple") {
        cs << node_text(g, "Gaze") << std::endl;
        cs << node_text(c->first("FovY"), "FovY") << std::endl;
        Vec gp;
        float fovy;
        cs >> gp.x >> gp.y >> gp.z >> fovy;
        const float half = deg * fovy / 2;
        t = tanf(half) * dist;
        const float aspect = 1.0f * w / h;
        b = -1.0f * t;
        r = t * aspect;
        l = -1.0f * r;
        gaze = unit(gp - pos);
      } else {
        cs << node_text(g, "Gaze") << std::endl;
        cs << node_text(c->first("NearPlane"), "NearPlane") << std::endl;
        cs >> gaze.x >> gaze.y >> gaze.z >> l >> r >> b >> t;
      }
      if (const Node* tm = c->first("Tonemap")) {
        const Node* tmo = tm->first("TMO");
        if (tmo && std::string(node_text(tmo, "TMO")) == "Photographic") {
          cs << node_text(tm->first("TMOOptions"), "TMOOptions") << std::endl;
          cs << node_text(tm->first("Saturation"), "Saturation") << std::endl;
          cs >> hc.tmo_key >> hc.tmo_saturation_percentage >> hc.tmo_saturation;
          hc.photographic_tmo = true;
        }
      }
      if (w <= 0 || h <= 0) throw std::runtime_error("scene xml: bad <ImageResolution>");
      const char* hand = c->attr("handedness");
      hc.cam = make_camera(up, gaze, pos, ns, l, r, b, t, dist, w, h,
                           hand && std::string(hand) == "left");
      S.cameras.push_back(hc);
    }
  }

  if (const Node* mats = root->first("Materials")) {  // Material.cpp:3-75
    std::stringstream ms;
    for (const Node* m : mats->each("Material")) {
      auto put = [&](const char* tag, const char* fallback) {
        const Node* n = m->first(tag);
        ms << (n ? node_text(n, tag) : fallback) << std::endl;
      };
      put("DiffuseReflectance", "0 0 0");
      put("SpecularReflectance", "0 0 0");
      put("MirrorReflectance", "0 0 0");
      put("PhongExponent", "1");
      put("Transparency", "0 0 0");
      put("RefractionIndex", "1.0");
      PMaterial M;
      M.brdf_id = m->int_attr("BRDF", 0) - 1;
      for (float* v : {M.diffuse, M.specular, M.mirror}) ms >> v[0] >> v[1] >> v[2];
      ms >> M.phong;
      ms >> M.transparency[0] >> M.transparency[1] >> M.transparency[2];
      ms >> M.refraction_index;
      auto nonzero = [](const float* v) { return v[0] != 0.0f || v[1] != 0.0f || v[2] != 0.0f; };
      M.type = nonzero(M.mirror) ? kMatMirror : nonzero(M.transparency) ? kMatRefractive : kMatDiffuse;
      if (m->bool_attr("degamma", false)) {  // double pow(float, 2.2f) (Material.cpp:65-72)
        for (int k = 0; k < 3; k++) {
          M.diffuse[k] = (float)std::pow((double)M.diffuse[k], (double)2.2f);
          M.specular[k] = (float)std::pow((double)M.specular[k], (double)2.2f);
        }
      }
      S.materials.push_back(M);
    }
  }

  TransformLists T;
  if (const Node* tr = root->first("Transformations")) {  // Transformation.cpp:93-134
    std::stringstream ts, sc, rs;
    for (const Node* n : tr->each("Translation")) {
      float x, y, z;
      ts << node_text(n, "Translation") << std::endl;
      ts >> x >> y >> z;
      Transform t;
      t.m.a[0][3] = x, t.m.a[1][3] = y, t.m.a[2][3] = z;
      t.inv.a[0][3] = -x, t.inv.a[1][3] = -y, t.inv.a[2][3] = -z;
      t.nrm = t.inv.transposed();
      T.translation.push_back(t);
    }
    for (const Node* n : tr->each("Scaling")) {
      float x, y, z;
      sc << node_text(n, "Scaling") << std::endl;
      sc >> x >> y >> z;
      Transform t;
      t.m = Mat::zero();
      t.m.a[0][0] = x, t.m.a[1][1] = y, t.m.a[2][2] = z, t.m.a[3][3] = 1.0f;
      t.inv = Mat::zero();
      t.inv.a[0][0] = 1.0f / x, t.inv.a[1][1] = 1.0f / y, t.inv.a[2][2] = 1.0f / z;
      t.inv.a[3][3] = 1.0f;
      t.nrm = t.inv.transposed();
      T.scaling.push_back(t);
    }
    constexpr float deg = M_PI / 180.0f;
    for (const Node* n : tr->each("Rotation")) {  // Transformation.cpp:34-75
      float angle, x, y, z;
      rs << node_text(n, "Rotation") << std::endl;
      rs >> angle >> x >> y >> z;
      angle = angle * deg;
      const Vec u = unit(vec(x, y, z));
      const Vec v = unit((x != 0.0f || y != 0.0f) ? vec(-u.y, u.x, 0.0f) : vec(0.0f, 1.0f, 0.0f));
      const Vec w = cross(u, v);
      Mat basis = Mat::zero();
      put3(basis.a[0], u);
      put3(basis.a[1], v);
      put3(basis.a[2], w);
      basis.a[3][3] = 1.0f;
      auto about_x = [](float ang) {
        Mat r = Mat::zero();
        r.a[0][0] = 1.0f;
        r.a[1][1] = std::cos(ang);
        r.a[1][2] = -std::sin(ang);
        r.a[2][1] = -r.a[1][2];
        r.a[2][2] = r.a[1][1];
        r.a[3][3] = 1.0f;
        return r;
      };
      const Mat bt = basis.transposed();
      Transform t;
      t.m = bt * (about_x(angle) * basis);
      t.inv = bt * (about_x(-angle) * basis);
      t.nrm = t.inv.transposed();
      T.rotation.push_back(t);
    }
  }

  if (const Node* vd = root->first("VertexData")) {  // Scene.cpp:452-470
    if (vd->attr("binaryFile"))
      throw std::domain_error("VertexData binaryFile: the reference PPM loader ignores it");
    ss << node_text(vd, "VertexData") << std::endl;
    float x, y, z;
    while (!(ss >> x).eof()) {
      ss >> y >> z;
      if (ss.fail()) throw std::runtime_error("scene xml: bad <VertexData>");
      S.vpos.insert(S.vpos.end(), {x, y, z});
    }
  }
  ss.clear();
  const int nverts = (int)(S.vpos.size() / 3);
  S.vnormal.assign(S.vpos.size(), 0.0f);
  auto vpos = [&](int i) {
    if (i < 0 || i >= nverts) throw std::runtime_error("scene xml: vertex index out of range");
    return vec(S.vpos[3 * i], S.vpos[3 * i + 1], S.vpos[3 * i + 2]);
  };

  if (const Node* ls = root->first("Lights")) {  // Point_light.cpp:32-51
    std::stringstream lsr;
    for (const Node* pl : ls->each("PointLight")) {
      lsr << node_text(pl->first("Position"), "Position") << std::endl;
      lsr << node_text(pl->first("Intensity"), "Intensity") << std::endl;
      float v[6];
      for (float& f : v) lsr >> f;
      S.lights.insert(S.lights.end(), v, v + 6);
    }
  }

  std::vector<BBox> obj_boxes, tri_boxes;
  std::vector<int> objects;
  auto check_material = [&](int m) {
    if (m < 0 || m >= (int)S.materials.size())
      throw std::runtime_error("scene xml: material index out of range");
  };
  auto add_object = [&](PObject o, const Transform& t, const BBox& box) {
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 4; j++) o.inv[4 * i + j] = t.inv.a[i][j];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) o.nrm[3 * i + j] = t.nrm.a[i][j];
    put3(o.lo, box.lo);
    put3(o.hi, box.hi);
    objects.push_back((int)S.objects.size());
    S.objects.push_back(o);
    obj_boxes.push_back(box);
  };
  std::vector<Mat> mesh_base;
  std::vector<BBox> mesh_box;
  std::vector<int> mesh_material;
  if (const Node* objs = root->first("Objects")) {
    std::stringstream os;
    for (const Node* s : objs->each("Sphere")) {  // Sphere.cpp:84-144
      int mat, center;
      float radius;
      os << node_text(s->first("Material"), "Material") << std::endl;
      os >> mat;
      --mat;
      os << node_text(s->first("Center"), "Center") << std::endl;
      os >> center;
      const Vec c = vpos(center - 1);
      os << node_text(s->first("Radius"), "Radius") << std::endl;
      os >> radius;
      const Mat m = apply_transformations(os, s->first("Transformations"), T, Mat::identity());
      os.clear();
      if (const Node* tx = s->first("Texture")) {
        int tid;
        os << node_text(tx, "Texture") << std::endl;
        os >> tid;
      }
      os.clear();
      check_material(mat);
      const Transform t = from_matrix(m);
      const Vec d = vec(radius, radius, radius);
      const BBox local = BBox::of(c - d, c + d);
      PObject o{};
      o.kind = kObjSphere;
      o.material = mat;
      o.mesh = -1;
      put3(o.center, c);
      o.radius = radius;
      add_object(o, t, t.m.identity_p() ? local : transformed(local, t.m));
    }
    std::stringstream mss;
    for (const Node* mnode : objs->each("Mesh")) {  // Mesh.cpp:5-111
      int mat;
      mss << node_text(mnode->first("Material"), "Material") << std::endl;
      mss >> mat;
      --mat;
      const char* sm = mnode->attr("shadingMode");
      const bool smooth = sm && std::string(sm) == "smooth";
      const Mat m = apply_transformations(mss, mnode->first("Transformations"), T, Mat::identity());
      mss.clear();
      if (const Node* tx = mnode->first("Texture")) {
        int tid;
        mss << node_text(tx, "Texture") << std::endl;
        mss >> tid;
      }
      mss.clear();
      const Node* faces = mnode->first("Faces");
      if (!faces) throw std::runtime_error("scene xml: <Mesh> without <Faces>");
      if (faces->attr("plyFile") || faces->attr("binaryFile"))
        throw std::domain_error("Faces plyFile / binaryFile: the reference PPM loader ignores them");
      const int offset = faces->int_attr("vertexOffset", 0);
      mss << node_text(faces, "Faces") << std::endl;
      std::vector<int> tris;
      int a, b, c;
      while (!(mss >> a).eof()) {
        mss >> b >> c;
        if (mss.fail()) throw std::runtime_error("scene xml: bad <Faces>");
        PTriangle tr{};
        tr.v[0] = a - 1 + offset;
        tr.v[1] = b - 1 + offset;
        tr.v[2] = c - 1 + offset;
        tr.smooth = smooth;
        const Vec p0 = vpos(tr.v[0]), p1 = vpos(tr.v[1]), p2 = vpos(tr.v[2]);
        const Vec n = unit(cross(p1 - p0, p2 - p0));  // Mesh_triangle.cpp:23
        put3(tr.normal, n);
        Vec mn = p0, mx = p0;
        for (Vec p : {p1, p2}) {
          mn = vec(lo_of(mn.x, p.x), lo_of(mn.y, p.y), lo_of(mn.z, p.z));
          mx = vec(hi_of(mx.x, p.x), hi_of(mx.y, p.y), hi_of(mx.z, p.z));
        }
        const float area = len(cross(p1 - p0, p2 - p0)) / 2;  // get_surface_area
        for (int k = 0; k < 3; k++) {                       // Vertex::add_vertex_normal
          float* vn = &S.vnormal[3 * tr.v[k]];
          vn[0] = vn[0] + n.x * area;
          vn[1] = vn[1] + n.y * area;
          vn[2] = vn[2] + n.z * area;
        }
        tris.push_back((int)S.triangles.size());
        S.triangles.push_back(tr);
        tri_boxes.push_back(BBox::of(mn, mx));
      }
      mss.clear();
      if (tris.empty()) throw std::runtime_error("scene xml: <Mesh> without triangles");
      check_material(mat);
      Builder bld{tri_boxes, S.mesh_nodes};
      PMesh pm;
      pm.root = bld.create(tris);
      S.mesh_depth = std::max(S.mesh_depth, bld.depth);
      S.meshes.push_back(pm);
      mesh_base.push_back(m);
      mesh_box.push_back(pm.root >= 0 ? BBox::of(vec(S.mesh_nodes[pm.root].lo[0],
                                                     S.mesh_nodes[pm.root].lo[1],
                                                     S.mesh_nodes[pm.root].lo[2]),
                                                 vec(S.mesh_nodes[pm.root].hi[0],
                                                     S.mesh_nodes[pm.root].hi[1],
                                                     S.mesh_nodes[pm.root].hi[2]))
                                      : tri_boxes[~pm.root]);
      mesh_material.push_back(mat);
    }
    auto add_instance = [&](int mesh, int mat, const Mat& m) {  // Mesh.h:104-112
      check_material(mat);
      const Transform t = from_matrix(m);
      PObject o{};
      o.kind = kObjInstance;
      o.material = mat;
      o.mesh = mesh;
      o.refractive = S.materials[mat].type == kMatRefractive;
      add_object(o, t, transformed(mesh_box[mesh], t.m));
    };
    for (int k = 0; k < (int)S.meshes.size(); k++)  // Mesh.cpp:113-125: one per mesh
      add_instance(k, mesh_material[k], mesh_base[k]);
    std::stringstream is;
    for (const Node* e : objs->each("MeshInstance")) {  // Mesh.cpp:126-206
      const int base = e->int_attr("baseMeshId", 0) - 1;
      if (base < 0 || base >= (int)S.meshes.size())
        throw std::runtime_error("scene xml: bad MeshInstance baseMeshId");
      int mat;
      is << node_text(e->first("Material"), "Material") << std::endl;
      is >> mat;
      --mat;
      Mat m = mesh_base[base];
      const char* reset = e->attr("resetTransform");
      if (reset && std::string(reset) == "true") m = Mat::identity();
      m = apply_transformations(is, e->first("Transformations"), T, m);
      is.clear();
      if (const Node* mb = e->first("MotionBlur")) {  // parsed, unused (as the reference)
        float v[3];
        is << node_text(mb, "MotionBlur") << std::endl;
        is >> v[0] >> v[1] >> v[2];
      }
      is.clear();
      add_instance(base, mat, m);
    }
  }
  for (int k = 0; k < nverts; k++) {  // Vertex::finalize_normal
    const Vec n = unit(vec(S.vnormal[3 * k], S.vnormal[3 * k + 1], S.vnormal[3 * k + 2]));
    put3(&S.vnormal[3 * k], n);
  }
  Builder top{obj_boxes, S.top_nodes};
  S.top_root = top.create(objects);
  S.top_depth = top.depth;
  if (S.top_depth + 1 > kTopStack || S.mesh_depth + 1 > kMeshStack)
    throw std::domain_error("BVH deeper than the traversal stacks (" + std::to_string(kTopStack) +
                            " / " + std::to_string(kMeshStack) + " levels)");
  if (S.lights.empty()) throw std::runtime_error("scene xml: no <PointLight> (photons need one)");
}

}  // namespace ppm
