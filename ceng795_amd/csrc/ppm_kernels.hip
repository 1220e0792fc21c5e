// Photon-mapping (PPM) kernels for gfx950 — the reference's PPM/src/Scene.cpp passes:
//
//   eye_kernel<COUNT|WRITE>  eye_trace_lines + eye_trace (Scene.cpp:250-361): one lane per
//                            pixel walks its eye-ray tree depth first; pass 1 counts hit
//                            points per pixel, a scan gives offsets, pass 2 writes them, so the
//                            hit-point array is in the single-threaded reference order.
//   grid_kernel              build_hash_grid (Scene.cpp:53-93): one block reduces the hit-point
//                            bounding box, derives the initial radius / hash scale and resets
//                            every hit point's (flux, radius^2, n).
//   photon_kernel            generate_photon + photon_trace (Point_light.cpp:7-30,
//                            Scene.cpp:106-249): one lane per photon; every diffuse hit leaves a
//                            deposit {x, n, w_i, flux} in the photon's slot row.
//   deposit_keys_kernel      compacts the deposits in (photon, bounce) order and keys each by
//                            the hash bucket of its cell (Scene.cpp:125-130).
//   expand_* / materialize   every deposit into each hit-point group filed under its bucket
//                            (hit points covering the same cells form a group); a stable
//                            radix sort by group gives each group its deposit list in photon
//                            order, materialised as 16-B position records.
//   group_update_kernel      the radius / flux updates of Scene.cpp:131-168, turned inside out:
//                            one workgroup per tile of a group's hit points streams the list in
//                            windows (superset filter, candidates in photon order, colour
//                            terms), one lane per hit point applies the exact recurrence; long
//                            lists are first compacted segment by segment.
//   density_kernel           density_estimation + Pixel::get_color (Scene.cpp:363-371).
//
// Why the update pass is exact: a photon's path never reads hit-point state, so the reference's
// per-photon updates (under a per-hit-point mutex) are, for each hit point, a sequential
// recurrence over the photons that reach one of its buckets.  Applying that recurrence in
// photon order reproduces a single-threaded reference run exactly (the oracle,
// oracle/ppm_ref.cpp, does literally that), without atomics or locks.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>

#include "ppm_internal.h"
#include "ppm_math.h"

#pragma clang fp contract(off)

namespace ppm {
namespace {

constexpr float kTestEps = 0.0001f;  // intersection_test_epsilon (PPM/include/Vector3.h:10)
constexpr float kInf = __builtin_huge_valf();
constexpr float kAlpha = 0.7f;       // ALPHA (Scene.cpp:13)

typedef float f32x2 __attribute__((ext_vector_type(2)));

struct V {
  float x, y, z;
};
__device__ __forceinline__ V mk(float x, float y, float z) { return V{x, y, z}; }
__device__ __forceinline__ V ld(const float* p) { return V{p[0], p[1], p[2]}; }
__device__ __forceinline__ V operator+(V a, V b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V operator-(V a, V b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V operator*(V a, V b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ V operator*(V a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V operator/(V a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ V operator-(V a, float s) { return mk(a.x - s, a.y - s, a.z - s); }
__device__ __forceinline__ V operator+(V a, float s) { return mk(a.x + s, a.y + s, a.z + s); }
__device__ __forceinline__ V neg(V a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(V a, V b) { return (a.x * b.x) + (a.y * b.y) + (a.z * b.z); }
__device__ __forceinline__ V cross(V a, V b) {
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ V normalize(V a) {
  return a / __builtin_sqrtf(a.x * a.x + a.y * a.y + a.z * a.z);
}
__device__ __forceinline__ float fmax0(float v) { return (0.0f < v) ? v : 0.0f; }  // std::max(0,v)
__device__ __forceinline__ float comp(V v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }

struct Ray {
  V o, d;
};
__device__ __forceinline__ V point_at(const Ray& r, float t) { return r.o + r.d * t; }

// Matrix4x4::multiply (Matrix4x4.cpp:27-45): rows accumulate from 0 (vector) or m[i][3] (point).
__device__ __forceinline__ V mul_vector(const float* m, int stride, V v) {
  float r[3];
#pragma unroll
  for (int i = 0; i < 3; i++) {
    r[i] = 0.0f;
    r[i] += m[stride * i] * v.x;
    r[i] += m[stride * i + 1] * v.y;
    r[i] += m[stride * i + 2] * v.z;
  }
  return mk(r[0], r[1], r[2]);
}
__device__ __forceinline__ V mul_point(const float* m, V v) {  // 3x4 rows
  float r[3];
#pragma unroll
  for (int i = 0; i < 3; i++) {
    r[i] = m[4 * i + 3];
    r[i] += m[4 * i] * v.x;
    r[i] += m[4 * i + 1] * v.y;
    r[i] += m[4 * i + 2] * v.z;
  }
  return mk(r[0], r[1], r[2]);
}

// Bounding_box::intersect + the caller's `t < 0 || t == inf` rejection (Bounding_box.cpp:32-54,
// BVH.cpp:33-35, Mesh.h:72-75), literally: true division, axes with |d| < 1e-4 skipped.
__device__ __forceinline__ bool box_accept(const float* lo, const float* hi, const Ray& r) {
  float tmin = -kInf, tmax = kInf;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const float d = comp(r.d, i), o = comp(r.o, i);
    if (__builtin_fabsf(d) < kTestEps) continue;
    float t0 = (lo[i] - o) / d;
    float t1 = (hi[i] - o) / d;
    if (d < 0) {
      const float s = t0;
      t0 = t1;
      t1 = s;
    }
    if (t0 > tmin) tmin = t0;
    if (t1 < tmax) tmax = t1;
    if (tmin > tmax) return false;  // returns kInf
  }
  const float v = tmin > 0.0f ? tmin : tmax;
  return !(v < 0.0f || v == kInf);
}

__device__ __forceinline__ float det3(V c1, V c2, V c3) {  // Mesh_triangle.h:44-49
  return c1.x * (c2.y * c3.z - c3.y * c2.z) + c2.x * (c3.y * c1.z - c1.y * c3.z) +
         c3.x * (c1.y * c2.z - c2.y * c1.z);
}

// Mesh_triangle::intersect (Mesh_triangle.cpp:57-111) without the normal (computed for the
// winner only).  Returns the raw acceptance (t > -1e-4).
__device__ __forceinline__ bool tri_test(const PScene& S, const PTriangle& tr, const Ray& r,
                                         bool culling, float& t, float& beta, float& gamma) {
  const V p0 = ld(S.vpos + 3 * tr.v[0]), p1 = ld(S.vpos + 3 * tr.v[1]),
          p2 = ld(S.vpos + 3 * tr.v[2]);
  const V a1 = p0 - p1, a2 = p0 - p2;
  if (culling && dot(r.d, ld(tr.normal)) > 0.0f) return false;
  const float det_a = det3(a1, a2, r.d);
  if (det_a == 0.0f) return false;
  const V b = (p0 - r.o) / det_a;
  beta = det3(b, a2, r.d);
  if (beta < -kTestEps) return false;
  gamma = det3(a1, b, r.d);
  if (gamma < -kTestEps || beta + gamma > 1.0f + kTestEps) return false;
  t = det3(a1, a2, b);
  return t > -kTestEps;
}

// Sphere::intersect (Sphere.cpp:26-64): true for any root, the caller filters t > 0.
__device__ __forceinline__ bool sphere_test(const PObject& o, const Ray& r, float& t) {
  const Ray rl{mul_point(o.inv, r.o), mul_vector(o.inv, 4, r.d)};
  const V co = rl.o - ld(o.center);
  const float a = dot(rl.d, rl.d);
  const float b = 2 * dot(rl.d, co);
  const float c = dot(co, co) - o.radius * o.radius;
  const float disc = b * b - 4 * a * c;
  if (disc < -kTestEps) return false;
  if (disc < kTestEps) {
    t = -b / (2 * a);
  } else {
    const float sq = __builtin_sqrtf(disc);
    const float t1 = (-b + sq) / (2 * a);
    const float t2 = (-b - sq) / (2 * a);
    t = t2 < 0.0f ? t1 : t2;
  }
  return true;
}

struct Hit {
  float t;
  int obj;  // top-level object
  int tri;  // triangle (instances), -1 for spheres
  float beta, gamma;
};

// Per-lane traversal stacks.  LDS (the launchers' choice when both BVHs fit kLdsStack levels,
// PScene::lds_stack): thread t's entry d at s[d][t], consecutive threads in consecutive banks,
// 24 KiB per 256-thread workgroup for the top-level and mesh stacks together.  Else a private
// array, which the compiler keeps in scratch (dynamically indexed).  Round 5: the C5 photon pass
// 16.4-16.7 -> 15.9-16.0 ms with LDS stacks (photon kernel scratch 464 -> 60 B per lane).
template <bool LDS, int N, int WHICH>
struct TraceStack {
  int s[N];
  __device__ __forceinline__ int& operator[](int d) { return s[d]; }
};
template <int N, int WHICH>
struct TraceStack<true, N, WHICH> {
  int* base;
  __device__ __forceinline__ TraceStack() {
    __shared__ int s_stk[kLdsStack][kPpmThreads];
    base = &s_stk[0][threadIdx.x];
  }
  __device__ __forceinline__ int& operator[](int d) { return base[d * kPpmThreads]; }
};

// Mesh::intersect -> the mesh's BVH with the local ray (Mesh.h:21-27, BVH.cpp:30-52): the
// first triangle in DFS order with the smallest t > 0.  A one-triangle mesh (create_bvh
// returns the triangle itself) gives the raw test, t > -1e-4 included.
template <bool LDS>
__device__ bool mesh_closest(const PScene& S, int root, const Ray& rl, bool culling, Hit& h) {
  float t, b, g;
  if (root < 0) {
    if (!tri_test(S, S.triangles[~root], rl, culling, t, b, g)) return false;
    h.t = t, h.tri = ~root, h.beta = b, h.gamma = g;
    return true;
  }
  TraceStack<LDS, kMeshStack, 1> stack;
  int sp = 0;
  stack[sp++] = root;
  bool any = false;
  h.t = kInf;
  while (sp > 0) {
    const int e = stack[--sp];
    if (e >= 0) {
      const PNode& n = S.mesh_nodes[e];
      if (!box_accept(n.lo, n.hi, rl)) continue;
      stack[sp++] = n.child[1];  // left child popped (visited) first
      stack[sp++] = n.child[0];
    } else if (tri_test(S, S.triangles[~e], rl, culling, t, b, g) && t > 0.0f && t < h.t) {
      h.t = t, h.tri = ~e, h.beta = b, h.gamma = g;
      any = true;
    }
  }
  return any;
}

// Shape::intersect of a top-level object, unfiltered (the parent BVH node filters t > 0).
template <bool LDS>
__device__ __forceinline__ bool object_test(const PScene& S, int obj, const Ray& r,
                                            bool culling, Hit& h) {
  const PObject& o = S.objects[obj];
  h.obj = obj;
  if (o.kind == kObjSphere) {
    h.tri = -1;
    return sphere_test(o, r, h.t);
  }
  // Mesh_instance::intersect (Mesh.h:70-93): world box, then the mesh with the local ray;
  // refractive instances are never culled.
  if (!box_accept(o.lo, o.hi, r)) return false;
  const Ray rl{mul_point(o.inv, r.o), mul_vector(o.inv, 4, r.d)};
  return mesh_closest<LDS>(S, S.meshes[o.mesh].root, rl, o.refractive ? false : culling, h);
}

// bvh->intersect(ray, intersection, true) at the top level (BVH.cpp:30-52).
template <bool LDS>
__device__ bool closest(const PScene& S, const Ray& r, Hit& best) {
  if (S.top_root == INT_MIN) return false;
  if (S.top_root < 0) return object_test<LDS>(S, ~S.top_root, r, true, best);  // root = one object
  TraceStack<LDS, kTopStack, 0> stack;
  int sp = 0;
  stack[sp++] = S.top_root;
  bool any = false;
  best.t = kInf;
  while (sp > 0) {
    const int e = stack[--sp];
    if (e >= 0) {
      const PNode& n = S.top_nodes[e];
      if (!box_accept(n.lo, n.hi, r)) continue;
      stack[sp++] = n.child[1];
      stack[sp++] = n.child[0];
      continue;
    }
    Hit h;
    if (object_test<LDS>(S, ~e, r, true, h) && h.t > 0.0f && h.t < best.t) {
      best = h;
      any = true;
    }
  }
  return any;
}

// The winner's shading normal, as the winning intersect call computed it: sphere normal from
// the local hit point (Sphere.cpp:55-60), flat or smooth triangle normal (Mesh_triangle.cpp:
// 91-103), then Mesh_instance's normal transform (Mesh.h:84-87).
__device__ V hit_normal(const PScene& S, const Ray& r, const Hit& h) {
  const PObject& o = S.objects[h.obj];
  if (o.kind == kObjSphere) {
    const Ray rl{mul_point(o.inv, r.o), mul_vector(o.inv, 4, r.d)};
    const V local = point_at(rl, h.t) - ld(o.center);
    return normalize(mul_vector(o.nrm, 3, normalize(local)));
  }
  const PTriangle& tr = S.triangles[h.tri];
  V n;
  if (tr.smooth) {
    const float w0 = (1 - h.beta) - h.gamma;
    n = normalize((ld(S.vnormal + 3 * tr.v[0]) * w0 + ld(S.vnormal + 3 * tr.v[1]) * h.beta) +
                  ld(S.vnormal + 3 * tr.v[2]) * h.gamma);
  } else {
    n = ld(tr.normal);
  }
  return normalize(mul_vector(o.nrm, 3, n));
}

// Shared refraction set-up of eye_trace / photon_trace (Scene.cpp:225-245, 330-352).
struct Refraction {
  bool tir, into;
  Ray reflection, refraction;
  float fresnel;
};
__device__ Refraction refract_setup(const PScene& S, const Ray& ray, V x, V normal,
                                    const PMaterial& m) {
  Refraction R;
  const V nl = dot(normal, ray.d) < 0.0f ? normal : normal * -1;
  const V w_o = normalize(ray.o - x);
  const V w_r = normalize((normal * (2.0f * dot(normal, w_o))) - w_o);
  R.reflection = Ray{x + (w_r * S.eps), w_r};
  R.into = dot(normal, nl) > 0.0f;
  const float air = 1.0f;
  const float nnt = R.into ? air / m.refraction_index : m.refraction_index / air;
  const float ddn = dot(ray.d, nl);
  const float cos2t = 1 - nnt * nnt * (1 - ddn * ddn);
  R.tir = cos2t < 0.0f;
  R.fresnel = 0.0f;
  if (R.tir) {
    R.refraction = R.reflection;
    return R;
  }
  const V dir = normalize(ray.d * nnt -
                          normal * ((float)(R.into ? 1 : -1) * (ddn * nnt + __builtin_sqrtf(cos2t))));
  const float a = m.refraction_index - air, b = m.refraction_index + air;
  const float r0 = a * a / (b * b);
  const float cosa = R.into ? -ddn : dot(dir, normal);
  const float c = 1 - cosa;
  R.fresnel = r0 + (1 - r0) * c * c * c * c * c;
  R.refraction = Ray{x + (dir * S.eps), dir};
  return R;
}

__device__ __forceinline__ Ray camera_ray(const PCamera& c, float x, float y) {
  // Camera::calculate_ray_at (PPM/include/Camera.h:76-84): (tl + x*s_u) - y*s_v
  const V s = (ld(c.top_left) + ld(c.s_u) * x) - ld(c.s_v) * y;
  const V e = ld(c.e);
  return Ray{e, normalize(s - e)};
}

struct EyeItem {
  Ray ray;
  V att;
  int depth;
};

// eye_trace (Scene.cpp:286-361) of one primary ray, depth first (reflection subtree before
// the refraction one).  WRITE: store the hit points at out[k++]; always counts them.
template <bool WRITE, bool LDS>
__device__ int eye_trace(const PScene& S, const Ray& primary, int pixel, PHitPoint* out, int k,
                         unsigned long long& rays) {
  EyeItem stack[kEyeStack];
  int sp = 0;
  stack[sp++] = EyeItem{primary, mk(1.0f, 1.0f, 1.0f), 0};
  while (sp > 0) {
    const EyeItem it = stack[--sp];
    Hit h;
    rays++;
    if (!closest<LDS>(S, it.ray, h)) continue;
    const V x = point_at(it.ray, h.t);
    const V normal = hit_normal(S, it.ray, h);
    const int mid = S.objects[h.obj].material;
    const PMaterial& m = S.materials[mid];
    if (m.type == kMatDiffuse) {
      if (WRITE) {
        PHitPoint hp;
        const V w_o = normalize(it.ray.o - x);
        hp.pos[0] = x.x, hp.pos[1] = x.y, hp.pos[2] = x.z;
        hp.normal[0] = normal.x, hp.normal[1] = normal.y, hp.normal[2] = normal.z;
        hp.w_o[0] = w_o.x, hp.w_o[1] = w_o.y, hp.w_o[2] = w_o.z;
        hp.att[0] = it.att.x, hp.att[1] = it.att.y, hp.att[2] = it.att.z;
        hp.material = mid;
        hp.pixel = pixel;
        hp.weight = 1.0f;
        hp.pad = 0.0f;
        out[k] = hp;
      }
      k++;
    } else if (it.depth >= S.max_depth) {
      continue;
    } else if (m.type == kMatMirror) {
      const V w_o = normalize(it.ray.o - x);
      const V w_r = normalize((normal * (2.0f * dot(normal, w_o))) - w_o);
      stack[sp++] = EyeItem{Ray{x + (w_r * S.eps), w_r}, ld(m.mirror) * it.att, it.depth + 1};
    } else {
      const Refraction R = refract_setup(S, it.ray, x, normal, m);
      if (R.tir) {
        stack[sp++] = EyeItem{R.reflection, ld(m.transparency) * it.att, it.depth + 1};
        continue;
      }
      const V attenuated = ld(m.transparency) * it.att;
      if (R.into) {
        stack[sp++] = EyeItem{R.refraction, attenuated * (1.0f - R.fresnel), it.depth + 1};
        stack[sp++] = EyeItem{R.reflection, it.att * R.fresnel, it.depth + 1};
      } else {
        stack[sp++] = EyeItem{R.refraction, attenuated, it.depth + 1};
      }
    }
  }
  return k;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ unsigned bucket_of(const PGrid& G, int ix, int iy, int iz) {
  // Scene::hash (PPM/include/Scene.h:65-68): int products wrap, xor, unsigned % num_hash
  const unsigned a = (unsigned)ix * 73856093u, b = (unsigned)iy * 19349663u,
                 c = (unsigned)iz * 83492791u;
  return (a ^ b ^ c) % G.num_hash;
}
__device__ __forceinline__ int cell(float v) { const int i = (int)v; return i < 0 ? -i : i; }

}  // namespace

// ------------------------------------------------------------------ eye pass
// counts != null: pass 1 (hit points per pixel); else pass 2 writes at offsets[pixel].
template <bool LDS>
__global__ __launch_bounds__(kPpmThreads) void eye_kernel(PScene S, PCamera C,
                                                          unsigned long long seed, int* counts,
                                                          const int* offsets, PHitPoint* out,
                                                          unsigned long long* stats) {
  const int p = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const bool active = p < C.width * C.height;
  unsigned long long rays = 0;
  if (active) {
    const int i = p % C.width, j = p / C.width;
    const bool write = counts == nullptr;
    int k = write ? offsets[p] : 0;
    if (C.samples == 1) {  // Scene.cpp:257-263
      const Ray r = camera_ray(C, i + 0.5f, j + 0.5f);
      k = write ? eye_trace<true, LDS>(S, r, p, out, k, rays)
                : eye_trace<false, LDS>(S, r, p, out, k, rays);
    } else {  // Scene.cpp:264-284: at most 2x2 jittered samples
      const int n = C.samples < 2 ? C.samples : 2;
      ppm_math::Rng rng(seed, ppm_math::kEyeStream | (unsigned long long)p);
      for (int x = 0; x < n; x++)
        for (int y = 0; y < n; y++) {
          const float ex = rng.uniform01();
          const float ey = rng.uniform01();
          const float sx = (x + ex) / n;
          const float sy = (y + ey) / n;
          const Ray r = camera_ray(C, i + sx, j + sy);
          k = write ? eye_trace<true, LDS>(S, r, p, out, k, rays)
                    : eye_trace<false, LDS>(S, r, p, out, k, rays);
        }
    }
    if (!write) counts[p] = k;
  }
  const unsigned long long tot = wave_sum(rays);
  if (stats && (threadIdx.x & 63) == 0 && tot) atomicAdd(&stats[4], tot);
}

// ------------------------------------------------------------------ hash grid
__global__ __launch_bounds__(1024) void grid_kernel(const PHitPoint* hps, int n, int width,
                                                    int height, PGrid* grid, float4* state,
                                                    unsigned* counts) {
  __shared__ float red[6][1024];
  const int t = (int)threadIdx.x;
  float lo[3] = {kInf, kInf, kInf}, hi[3] = {-kInf, -kInf, -kInf};
  for (int k = t; k < n; k += 1024)
    for (int a = 0; a < 3; a++) {  // Bounding_box::fit: std::min / std::max
      const float v = hps[k].pos[a];
      lo[a] = (v < lo[a]) ? v : lo[a];
      hi[a] = (hi[a] < v) ? v : hi[a];
    }
  for (int a = 0; a < 3; a++) red[a][t] = lo[a], red[3 + a][t] = hi[a];
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if (t < s)
      for (int a = 0; a < 3; a++) {
        const float l = red[a][t + s], h = red[3 + a][t + s];
        red[a][t] = (l < red[a][t]) ? l : red[a][t];
        red[3 + a][t] = (red[3 + a][t] < h) ? h : red[3 + a][t];
      }
    __syncthreads();
  }
  // Scene.cpp:59-61: initial radius from the mean bounding-box extent and image size
  const float dx = red[3][0] - red[0][0], dy = red[4][0] - red[1][0], dz = red[5][0] - red[2][0];
  const float r = ((dx + dy + dz) / 3.0f) / ((width + height) / 2.0f) * 2.0f * 4.0f;
  __syncthreads();
  for (int a = 0; a < 3; a++) lo[a] = kInf, hi[a] = -kInf;
  const float r2 = r * r;
  for (int k = t; k < n; k += 1024) {
    for (int a = 0; a < 3; a++) {  // fit(position - r), fit(position + r)
      const float m = hps[k].pos[a] - r, p = hps[k].pos[a] + r;
      lo[a] = (m < lo[a]) ? m : lo[a];
      hi[a] = (hi[a] < m) ? m : hi[a];
      lo[a] = (p < lo[a]) ? p : lo[a];
      hi[a] = (hi[a] < p) ? p : hi[a];
    }
    state[k] = make_float4(0.0f, 0.0f, 0.0f, r2);  // flux = 0, radius^2 (Scene.cpp:64-67)
    counts[k] = 0u;
  }
  for (int a = 0; a < 3; a++) red[a][t] = lo[a], red[3 + a][t] = hi[a];
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if (t < s)
      for (int a = 0; a < 3; a++) {
        const float l = red[a][t + s], h = red[3 + a][t + s];
        red[a][t] = (l < red[a][t]) ? l : red[a][t];
        red[3 + a][t] = (red[3 + a][t] < h) ? h : red[3 + a][t];
      }
    __syncthreads();
  }
  if (t == 0) {
    PGrid G;
    for (int a = 0; a < 3; a++) G.bmin[a] = red[a][0], G.bmax[a] = red[3 + a][0];
    G.radius = r;
    G.hash_scale = (float)(1.0 / ((double)r * 2.0));
    G.num_hash = (unsigned)n;
    G.pad = 0;
    *grid = G;
  }
}

// ------------------------------------------------------------------ photon pass
// Photon first + i traces its chain (photon_trace's recursion never branches) and leaves
// one deposit per diffuse hit in slots[k * count + i], k < K = max(1, MaxRecursionDepth - 1)
// (k-major, so deposit_keys reads the k-th deposits of consecutive photons coalesced).
//
// Lanes are refilled: Russian roulette ends ~2/3 of the chains at every
// diffuse hit (C5: 1.36 segments per photon), so a wave that traced one photon per lane ran
// until its longest chain ended (~4-5 segments) with most lanes idle.  Here each workgroup owns
// a contiguous range of photons; a lane whose chain ends takes the next photon of the range
// (one LDS atomic per wave and round) and the wave runs one segment per round for all its live
// lanes.  Every photon is computed exactly as before (own random stream, same arithmetic, its
// deposits in its own slots), only the lane that computes it changes.
#ifndef PPM_PHOTON_BLOCKS
#define PPM_PHOTON_BLOCKS 4096
#endif
struct PhotonState {
  ppm_math::Rng rng{0, 0};
  Ray ray;
  V flux;
  int depth, k;
};

// Point_light::generate_photon (Point_light.cpp:7-30): theta = 2 pi e2 on purpose
__device__ __forceinline__ void emit_photon(const PScene& S, unsigned long long seed,
                                            long long photon, PhotonState& P) {
  P.rng = ppm_math::Rng(seed, (unsigned long long)photon);
  P.flux = ld(S.light_intensity) * (float)(M_PI * 4.0f);
  const float e1 = P.rng.uniform01();
  const float e2 = P.rng.uniform01();
  const V w = mk(0.0f, 1.0f, 0.0f);
  const V u = normalize((w.x != 0.0f || w.y != 0.0f) ? mk(-w.y, w.x, 0.0f) : mk(0.0f, 1.0f, 0.0f));
  const V v = cross(w, u);
  const float phi = (float)(2 * M_PI * (double)e1);
  const float theta = (float)(2 * M_PI * (double)e2);
  float st, ct, sp, cp;
  ppm_math::sincosf_ieee(theta, st, ct);
  ppm_math::sincosf_ieee(phi, sp, cp);
  P.ray = Ray{ld(S.light_pos), normalize((w * ct + (v * st) * cp) + (u * st) * sp)};
  P.depth = 0;
  P.k = 0;
}

// One segment of photon_trace (Scene.cpp:106-249) for photon i; false when the chain ends.
template <bool LDS>
__device__ __forceinline__ bool photon_segment(const PScene& S, int i, int count, PDeposit* slots,
                                               PhotonState& P, unsigned long long& rays,
                                               unsigned long long& deps) {
  P.depth++;
  if (P.depth >= S.max_depth) return false;
  Hit h;
  rays++;
  const Ray ray = P.ray;
  if (!closest<LDS>(S, ray, h)) return false;
  const V x = point_at(ray, h.t);
  const V normal = hit_normal(S, ray, h);
  const PMaterial& m = S.materials[S.objects[h.obj].material];
  if (m.type == kMatDiffuse) {
    const V w_i = neg(normalize(ray.d));
    PDeposit& d = slots[(size_t)P.k * count + i];
    d.x[0] = x.x, d.x[1] = x.y, d.x[2] = x.z;
    d.normal[0] = normal.x, d.normal[1] = normal.y, d.normal[2] = normal.z;
    d.w_i[0] = w_i.x, d.w_i[1] = w_i.y, d.w_i[2] = w_i.z;
    d.flux[0] = P.flux.x, d.flux[1] = P.flux.y, d.flux[2] = P.flux.z;
    P.k++;
    deps++;
    // sample_hemisphere(normal) (Scene.cpp:15-44), cosine weighted
    const float h1 = P.rng.uniform01();
    const float h2 = P.rng.uniform01();
    const V hu = normalize((normal.x != 0.0f || normal.y != 0.0f) ? mk(-normal.y, normal.x, 0.0f)
                                                                  : mk(0.0f, 1.0f, 0.0f));
    const V hv = cross(normal, hu);
    const float hphi = (float)(2 * M_PI * (double)h1);
    const float htheta = ppm_math::asinf_ieee(__builtin_sqrtf(h2));
    float hst, hct, hsp, hcp;
    ppm_math::sincosf_ieee(htheta, hst, hct);
    ppm_math::sincosf_ieee(hphi, hsp, hcp);
    const V dir = normalize((normal * hct + (hv * hst) * hcp) + (hu * hst) * hsp);
    const float prob = (float)((double)fmax0(dot(normal, dir)) / M_PI);
    // BRDF weight (Scene.cpp:173-194): nl from the incoming ray, as the reference
    const V nl = dot(normal, ray.d) < 0 ? normal : normal * -1;
    V base = mk(0.0f, 0.0f, 0.0f);
    const float cos_i = fmax0(dot(normal, w_i));
    if (m.brdf_id == -1 && !(cos_i > 1.0f || cos_i <= 0.0f)) {
      const float sc = fmax0(dot(nl, normalize(dir + w_i)));
      base = ld(m.diffuse) + (ld(m.specular) * ppm_math::powf_ieee(sc, m.phong)) / cos_i;
    }
    base = base * fmax0(dot(normal, dir));
    if (!(P.rng.uniform01() < prob)) return false;  // Russian roulette (Scene.cpp:196-199)
    P.ray = Ray{x + (dir * S.eps), dir};
    P.flux = (base * P.flux) / prob;
  } else if (m.type == kMatMirror) {
    const V w_o = normalize(ray.o - x);
    const V w_r = normalize((normal * (2.0f * dot(normal, w_o))) - w_o);
    P.ray = Ray{x + (w_r * S.eps), w_r};
    P.flux = ld(m.mirror) * P.flux;
  } else {
    const Refraction R = refract_setup(S, ray, x, normal, m);
    if (R.tir) P.ray = R.reflection;
    else if (R.into) P.ray = P.rng.uniform01() < R.fresnel ? R.reflection : R.refraction;
    else P.ray = R.refraction;
  }
  return true;
}

template <bool LDS>
__global__ __launch_bounds__(kPpmThreads) void photon_kernel(PScene S, unsigned long long seed,
                                                             long long first, int count, int K,
                                                             PDeposit* slots, int* ndep,
                                                             unsigned long long* stats) {
  unsigned long long rays = 0, deps = 0;
  PhotonState P;
  __shared__ int s_next;
  const int per = (int)(((long long)count + gridDim.x - 1) / gridDim.x);
  const int beg = (int)min((long long)blockIdx.x * per, (long long)count);
  const int end = min(count, beg + per);
  if (threadIdx.x == 0) s_next = beg;
  __syncthreads();
  const int lane = (int)(threadIdx.x & 63);
  int i = -1;  // this lane's photon (-1: none)
  for (;;) {
    const unsigned long long need = __ballot(i < 0);
    if (need) {  // refill the idle lanes from the workgroup's range, in lane order
      const int leader = __builtin_ctzll(need);
      int base = 0;
      if (lane == leader) base = atomicAdd(&s_next, __builtin_popcountll(need));
      base = __shfl(base, leader, 64);
      if (i < 0) {
        const int idx = base + __builtin_popcountll(need & ((1ull << lane) - 1ull));
        if (idx < end) {
          i = idx;
          emit_photon(S, seed, first + i, P);
        }
      }
    }
    if (!__ballot(i >= 0)) break;  // range exhausted and every chain ended
    if (i >= 0 && !photon_segment<LDS>(S, i, count, slots, P, rays, deps)) {
      ndep[i] = P.k;
      i = -1;
    }
  }
  const unsigned long long tr = wave_sum(rays), td = wave_sum(deps);
  if (stats && (threadIdx.x & 63) == 0) {
    if (tr) atomicAdd(&stats[1], tr);
    if (td) atomicAdd(&stats[2], td);
  }
}

// Deposit d of photon i -> dense position offsets[i] + d (photon order), with the bucket of
// its cell (Scene.cpp:125-130), and its position alone in dpos (what materialize reads per
// (group, deposit) pair: 16 B instead of a 48-B record's line).
__global__ __launch_bounds__(256) void deposit_keys_kernel(const PDeposit* slots,
                                                           const int* ndep, const int* offsets,
                                                           int count, int K,
                                                           const PGrid* grid, unsigned* bucket,
                                                           PDeposit* dense, float4* dpos) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= count) return;
  const PGrid G = *grid;
  const int n = ndep[i], o = offsets[i];
  for (int k = 0; k < n; k++) {
    const PDeposit d = slots[(size_t)k * count + i];
    const V hh = (ld(d.x) - ld(G.bmin)) * G.hash_scale;
    bucket[o + k] = bucket_of(G, cell(hh.x), cell(hh.y), cell(hh.z));
    dense[o + k] = d;
    dpos[o + k] = make_float4(d.x[0], d.x[1], d.x[2], 0.0f);
  }
}

// Runs of equal (key & mask) in a sorted key array: [start[k], end[k]).
__global__ __launch_bounds__(256) void bucket_bounds_kernel(const unsigned* keys, int n,
                                                            unsigned mask, int* start, int* end) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= n) return;
  const unsigned k = keys[i] & mask;
  if (i == 0 || (keys[i - 1] & mask) != k) start[k] = i;
  if (i == n - 1 || (keys[i + 1] & mask) != k) end[k] = i + 1;
}

// ------------------------------------------------------------------ grouped update pass
// Hit points whose radius boxes cover the same cell range were filed under the same buckets,
// so they see the same deposit stream.  group_key_kernel keys each hit point by its range
// (lower cell corner + extent); a radix sort groups them; group_update_kernel then runs one
// wave per group: it merges the group's bucket runs in photon order through LDS once and
// every lane (hit point) applies the merged stream to its own state.
__global__ __launch_bounds__(256) void group_key_kernel(const PHitPoint* hps, int n,
                                                        const PGrid* grid,
                                                        unsigned long long* keys, int* idx,
                                                        int* error) {
  const int h = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (h >= n) return;
  const PGrid G = *grid;
  const V pos = ld(hps[h].pos);
  const V bmin = ((pos - G.radius) - ld(G.bmin)) * G.hash_scale;
  const V bmax = ((pos + G.radius) - ld(G.bmin)) * G.hash_scale;
  const int x0 = cell(bmin.x), y0 = cell(bmin.y), z0 = cell(bmin.z);
  const int dx = cell(bmax.x) - x0, dy = cell(bmax.y) - y0, dz = cell(bmax.z) - z0;
  if (x0 > 0xffff || y0 > 0xffff || z0 > 0xffff || dx < 0 || dy < 0 || dz < 0 || dx > 31 ||
      dy > 31 || dz > 31 || (dx + 1) * (dy + 1) * (dz + 1) > kMaxCells)
    atomicExch(error, 2);
  keys[h] = (unsigned long long)(x0 & 0xffff) | (unsigned long long)(y0 & 0xffff) << 16 |
            (unsigned long long)(z0 & 0xffff) << 32 | (unsigned long long)(dx & 31) << 48 |
            (unsigned long long)(dy & 31) << 53 | (unsigned long long)(dz & 31) << 58;
  idx[h] = h;
}

__global__ __launch_bounds__(256) void group_flags_kernel(const unsigned long long* keys, int n,
                                                          int* flags) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i < n) flags[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
  if (i == n) flags[n] = 0;
}

__global__ __launch_bounds__(256) void group_starts_kernel(const int* flags, const int* gid,
                                                           int n, int* gstart) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i < n && flags[i]) gstart[gid[i]] = i;
  if (i == n) gstart[gid[n]] = n;  // gid[n] = number of groups
}

#ifndef PPM_TILE
#define PPM_TILE 5  // hit points per update tile (round 3: 5 with 1,024-deposit windows, C5 update 9.58 -> 8.60 ms)
#endif
#ifndef PPM_WIN
#define PPM_WIN 1024
#endif
#ifndef PPM_GATE_B
#define PPM_GATE_B 3
#endif
#ifndef PPM_CHUNK
#define PPM_CHUNK 1024
#endif
#ifndef PPM_WPE
#define PPM_WPE 4
#endif
#ifndef PPM_THREADS
#define PPM_THREADS 512
#endif
constexpr int kTileHP = PPM_TILE;       // hit points per update workgroup
constexpr int kWinMax = PPM_WIN;        // deposits per window
constexpr int kUpdThreads = PPM_THREADS;

// Each group's buckets (Scene.cpp:79-91 for its first hit point; all members share them),
// deduplicated, with multiplicity.
__global__ __launch_bounds__(256) void group_buckets_kernel(const PHitPoint* hps, const int* perm,
                                                            const int* gstart, int groups,
                                                            const PGrid* grid, unsigned* gb,
                                                            int* gm, int* gnb) {
  const int g = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (g > groups) return;
  if (g == groups) {
    gnb[groups] = 0;
    return;
  }
  const PGrid G = *grid;
  const V pos = ld(hps[perm[gstart[g]]].pos);
  const V bmin = ((pos - G.radius) - ld(G.bmin)) * G.hash_scale;
  const V bmax = ((pos + G.radius) - ld(G.bmin)) * G.hash_scale;
  unsigned* b_out = gb + (size_t)g * kMaxCells;
  int* m_out = gm + (size_t)g * kMaxCells;
  int nb = 0;
  for (int iz = cell(bmin.z); iz <= cell(bmax.z); iz++)
    for (int iy = cell(bmin.y); iy <= cell(bmax.y); iy++)
      for (int ix = cell(bmin.x); ix <= cell(bmax.x); ix++) {
        const unsigned b = bucket_of(G, ix, iy, iz);
        int u = 0;
        while (u < nb && b_out[u] != b) u++;
        if (u < nb) m_out[u]++;
        else if (nb < kMaxCells) b_out[nb] = b, m_out[nb] = 1, nb++;
      }
  gnb[g] = nb;
}

// (bucket, group) pairs in group order; a stable sort by bucket makes the bucket -> groups map.
// The value carries the group and, above kGroupBits, its multiplicity for that bucket (how many
// of the group's cells hash there): it rides along in the expansion keys (sorted on the group
// bits only) to the materialised records.
__global__ __launch_bounds__(256) void bucket_group_pairs_kernel(const unsigned* gb,
                                                                 const int* gm, const int* gnb,
                                                                 const int* goff, int groups,
                                                                 unsigned* key, unsigned* val) {
  const int g = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (g >= groups) return;
  for (int u = 0; u < gnb[g]; u++) {
    key[goff[g] + u] = gb[(size_t)g * kMaxCells + u];
    val[goff[g] + u] = (unsigned)g | ((unsigned)gm[(size_t)g * kMaxCells + u] << kGroupBits);
  }
}

// Expansion: every deposit (photon order) into each group filed under its bucket.
__global__ __launch_bounds__(256) void expand_count_kernel(const unsigned* bucket, int n,
                                                           const int* bg_start,
                                                           const int* bg_end, int* count) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i < n) count[i] = bg_end[bucket[i]] - bg_start[bucket[i]];
  if (i == n) count[n] = 0;
}
__global__ __launch_bounds__(256) void expand_write_kernel(const unsigned* bucket, int n,
                                                           const int* bg_start,
                                                           const int* bg_end,
                                                           const unsigned* bg_group,
                                                           const int* off, unsigned* key,
                                                           unsigned* val) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= n) return;
  const unsigned b = bucket[i];
  int o = off[i];
  for (int k = bg_start[b]; k < bg_end[b]; k++, o++) {
    key[o] = bg_group[k];
    val[o] = (unsigned)i;
  }
}

__global__ __launch_bounds__(256) void group_tiles_kernel(const int* gstart, int groups,
                                                          int* ntile) {
  const int g = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (g < groups) ntile[g] = (gstart[g + 1] - gstart[g] + kTileHP - 1) / kTileHP;
  if (g == groups) ntile[groups] = 0;
}

__global__ __launch_bounds__(256) void tile_table_kernel(const int* gstart, const int* tile_off,
                                                         int groups, int2* tiles) {
  const int g = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (g >= groups) return;
  for (int t = tile_off[g]; t < tile_off[g + 1]; t++)
    tiles[t] = make_int2(g, gstart[g] + (t - tile_off[g]) * kTileHP);
}

// Update-pass sharding (ppm_set_update_shard, multi-device scenes): tile t of the group-order
// table belongs to shard t mod shards.  `mine` receives this shard's tiles in table order;
// `owner` (nullable) the shard of every hit point.  Tiles own disjoint hit points, so a shard
// applies the complete photon-order recurrence of each of its hit points.
__global__ __launch_bounds__(256) void tile_shard_kernel(const int2* all, int ntiles, int shard,
                                                         int shards, const int* gstart,
                                                         const int* perm, int2* mine, int* owner) {
  const int t = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (t >= ntiles) return;
  const int2 tile = all[t];
  if (t % shards == shard) mine[t / shards] = tile;
  if (owner) {
    const int e = min(tile.y + kTileHP, gstart[tile.x + 1]);
    for (int k = tile.y; k < e; k++) owner[perm[k]] = t % shards;
  }
}

// Merge of a sharded update pass: hit point h takes (state, count) from the shard that owns
// it; `self`'s own values are already in place, the others' come from `peer` (shards x n).
__global__ __launch_bounds__(256) void merge_state_kernel(const int* owner, int n, int self,
                                                          const float4* peer_state,
                                                          const unsigned* peer_nupd,
                                                          float4* state, unsigned* nupd) {
  const int h = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (h >= n) return;
  const int o = owner[h];
  if (o == self) return;
  state[h] = peer_state[(size_t)o * n + h];
  nupd[h] = peer_nupd[(size_t)o * n + h];
}


// Longest-first launch order for the update pass: a tile's work is its group's deposit-list
// length in this batch; the complemented length sorts the heaviest tiles to the front, so the
// hot groups' serial chains start in the first dispatch round instead of the last.
__global__ __launch_bounds__(256) void tile_work_kernel(const int2* tiles, int ntiles,
                                                        const int* list_start,
                                                        const int* list_end, unsigned* key) {
  const int t = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (t >= ntiles) return;
  const int g = tiles[t].x;
  key[t] = ~(unsigned)(list_end[g] - list_start[g]);
}

// rr(n) of Scene.cpp:139-140, the radius reduction of a hit point's (n+1)-th update:
// (n*ALPHA + ALPHA) / (n*ALPHA + 1.0), a double division rounded to float.  It depends on n
// only, so it is tabulated once (rr_table_kernel) and staged in LDS per window.
__device__ __forceinline__ float radius_reduction(unsigned n) {
  const float nf = (float)n * kAlpha;
  return (float)((double)(nf + kAlpha) / ((double)nf + 1.0));
}

// Tile-list compaction (group_update_kernel phase (0) for long lists): a tile whose group
// list holds at least `min_len` deposits takes it in segments of `seg` (S.compact_seg,
// default 32768) and gets a scratch range of seg >> shift records; per segment the
// kernel copies into it, in photon
// order, the deposits within the radius any of its hit points has at the segment start, and
// streams its windows over that copy (over the segment itself when the copy overflows).
// need[ntiles] = 0 closes the exclusive scan that turns the sizes into offsets.
#ifndef PPM_CPER
#define PPM_CPER 4
#endif
__global__ __launch_bounds__(256) void tile_compact_need_kernel(const int2* tiles, int ntiles,
                                                                const int* list_start,
                                                                const int* list_end,
                                                                long long min_len, int shift,
                                                                int seg, long long* need) {
  const int t = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (t > ntiles) return;
  if (t == ntiles) {
    need[t] = 0;
    return;
  }
  const int g = tiles[t].x;
  const long long L = list_end[g] - list_start[g];
  // (twice that: per-wave scratch regions + the contiguous copy)
  need[t] = L >= min_len ? ((L < seg ? L : (long long)seg) >> shift) * 2 : 0;
}

#ifndef PPM_GATE_RUNS  // gate_round (A1): candidates per accept/reject run pair below which (A2) takes over
#define PPM_GATE_RUNS 16
#endif
#ifndef PPM_GATE_PRIO  // wave priority of the gate waves while they run gate_round
#define PPM_GATE_PRIO 3
#endif
#ifndef PPM_PHASE_TIMERS  // 1: per-phase wall-clock timers for CENG795_PPM_DIAG=2 (tools/ppm_diag.sh)
#define PPM_PHASE_TIMERS 0
#endif

__device__ __forceinline__ float rr_at(const float* rrtab, int nrr, unsigned n) {
  return n < (unsigned)nrr ? rrtab[n] : radius_reduction(n);
}

// The exact recurrence of ONE hit point over its n candidates of a round (Scene.cpp:137-166,
// photon order), run by the hit point's wave; state (fx, fy, fz, r2, cnt) is wave-uniform.
// rec[k] = candidate k's record: color * photon_flux, and in w its distance^2 (negated when
// the deposit's multiplicity exceeds 1, +inf when its normal test failed).
// With a the number of accepts so far, the radius^2 is R(a) = (((r2 * rr(cnt)) * rr(cnt+1))
// ... * rr(cnt+a-1)) — the float products the sequential loop makes, in its order — and R only
// shrinks (rr < 1), so candidate k, tested against R(a_k), is accepted iff a_k <= K_k with
// K_k = max{a : d2_k <= R(a)} (-1: none).  So:
//   (R) lane 0 tabulates R(0..n) — one dependent multiply per entry;
//   (K) every lane binary-searches R for its candidates' K_k (lane l holds k = l + 64u);
//   (A) the acceptance sequence a_{k+1} = a_k + [a_k <= K_k] in RUNS: from k with a accepts,
//       candidates keep being accepted up to the first j with K_j - j < a - k (one ballot per
//       64 candidates finds it), then rejected up to the first j with K_j >= a; a round costs
//       one search per run, not one dependent step per candidate;
//   (C) the accepted records are compacted in order into acc[] (ranks by popcount / mbcnt);
//   (B) flux = (flux + c) * rr(cnt + i) over the i-th accepted record: lanes 0, 1, 2 each run
//       one colour component's chain (two dependent operations per accept).
// Bit-identical to the one-candidate-at-a-time loop, which remains for rounds holding a
// deposit of multiplicity > 1 (lane 0, rr from the table).  rrb[i] = rr(cnt + i), i < n.
[[maybe_unused]] constexpr int kGateK = 6;    // candidates per lane (n <= 64 * kGateK)
[[maybe_unused]] constexpr int kGatePad = 8;  // rr cache / R rows: slack for read-ahead
[[maybe_unused]] constexpr int kGateMinRun = PPM_GATE_RUNS;  // (A1) while runs average this
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// lanes [lo, hi) of a 64-lane chunk as a mask (0 <= lo <= hi <= 64)
__device__ __forceinline__ uint64_t lane_range(int lo, int hi) {
  const uint64_t upto_hi = hi >= 64 ? ~0ull : ((1ull << hi) - 1ull);
  const uint64_t below_lo = lo >= 64 ? ~0ull : ((1ull << lo) - 1ull);
  return upto_hi & ~below_lo;
}
__device__ void gate_round(float4* __restrict__ rec, float4* __restrict__ acc, int n, bool multi,
                           const unsigned* __restrict__ ck, const float* __restrict__ rrtab,
                           int nrr, const float* __restrict__ rrb, float* __restrict__ R,
                           float& fx, float& fy, float& fz, float& r2, unsigned& cnt,
                           unsigned long long* tick) {
  const int lane = (int)__lane_id();
  if (n <= 0) return;
  const unsigned long long t0 = tick ? wall_clock64() : 0;
  if (multi) {  // exact serial loop (multiplicity: retested while inside)
    if (lane == 0) {
      for (int k = 0; k < n; k++) {
        const float4 c = rec[k];
        const float d2 = __builtin_fabsf(c.w);
        const unsigned reps = (__float_as_uint(c.w) >> 31) ? (ck[k] & kRepMask) : 1u;
        for (unsigned i = 0; i < reps && d2 <= r2; i++) {
          const float rr = rr_at(rrtab, nrr, cnt);
          cnt++;
          fx = (fx + c.x) * rr;
          fy = (fy + c.y) * rr;
          fz = (fz + c.z) * rr;
          r2 = r2 * rr;
        }
      }
    }
    fx = __shfl(fx, 0, 64), fy = __shfl(fy, 0, 64), fz = __shfl(fz, 0, 64);
    r2 = __shfl(r2, 0, 64);
    cnt = (unsigned)__shfl((int)cnt, 0, 64);
    return;
  }
  if (lane == 0) {  // (R): the next 4 factors are read before this block's entries are stored
    float r = r2;
    R[0] = r;
    float q0 = rrb[0], q1 = rrb[1], q2 = rrb[2], q3 = rrb[3];
    for (int i = 0; i < n; i += 4) {
      const float p0 = rrb[i + 4], p1 = rrb[i + 5], p2 = rrb[i + 6], p3 = rrb[i + 7];
      r = r * q0;
      R[i + 1] = r;
      r = r * q1;
      R[i + 2] = r;
      r = r * q2;
      R[i + 3] = r;
      r = r * q3;
      R[i + 4] = r;
      q0 = p0, q1 = p1, q2 = p2, q3 = p3;
    }
  }
  wave_sync_lds();
  // (K): #{a : d2 <= R(a)} - 1 (R non-increasing), a lane's candidates searched together
  int K[kGateK];
  {
    int steps = 0;  // ceil(log2(n + 1)): the branch-free search's trip count (uniform)
    while ((1 << steps) < n + 1) steps++;
    float d2[kGateK];
    int len = n + 1;
#pragma unroll
    for (int u = 0; u < kGateK; u++) {
      const int k = lane + 64 * u;
      d2[u] = k < n ? rec[k].w : kInf;
      K[u] = 0;
    }
    for (int t = 0; t < steps; t++) {
      const int half = len >> 1;
#pragma unroll
      for (int u = 0; u < kGateK; u++) K[u] = d2[u] <= R[K[u] + half] ? K[u] + half : K[u];
      len -= half;
    }
#pragma unroll
    for (int u = 0; u < kGateK; u++) K[u] = K[u] + (d2[u] <= R[K[u]] ? 1 : 0) - 1;
  }
  uint64_t accm[kGateK];
#pragma unroll
  for (int u = 0; u < kGateK; u++) accm[u] = 0;
  int a = 0, k = 0;
  // (A1): runs of accepts and of rejects, while they average kGateMinRun candidates or more
  // (high acceptance: the hot hit points); a round whose runs turn out short falls through to
  // (A2) from where it stands
  for (int runs = 0; k < n && (runs < 2 || k >= kGateMinRun * runs); runs++) {
    int j = n;  // first j >= k with K_j - j < a - k
    {
      bool found = false;
#pragma unroll
      for (int u = 0; u < kGateK; u++) {
        if (found || 64 * u + 64 <= k || 64 * u >= n) continue;
        const int kk = 64 * u + lane;
        const uint64_t m = __ballot(kk >= k && kk < n && K[u] - kk < a - k);
        if (m) {
          j = 64 * u + (int)__builtin_ctzll(m);
          found = true;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kGateK; u++) {  // candidates [k, j) are accepted
      const int lo = max(k, 64 * u) - 64 * u, hi = min(j, 64 * u + 64) - 64 * u;
      if (lo < hi) accm[u] |= lane_range(lo, hi);
    }
    a += j - k;
    k = j;
    if (k >= n) break;
    j = n;  // rejected from k up to the first j with K_j >= a
    {
      bool found = false;
#pragma unroll
      for (int u = 0; u < kGateK; u++) {
        if (found || 64 * u + 64 <= k || 64 * u >= n) continue;
        const int kk = 64 * u + lane;
        const uint64_t m = __ballot(kk >= k && kk < n && K[u] >= a);
        if (m) {
          j = 64 * u + (int)__builtin_ctzll(m);
          found = true;
        }
      }
    }
    k = j;
  }
  // (A2): the rest one candidate at a time on the scalar unit (K_k by readlane)
#pragma unroll
  for (int u = 0; u < kGateK; u++) {
    if (64 * u + 64 <= k || 64 * u >= n) continue;
    const int cu = min(64, n - 64 * u);
    uint64_t m = accm[u];
    for (int l = max(k - 64 * u, 0); l < cu; l++) {
      const int Kk = __builtin_amdgcn_readlane(K[u], l);
      const int acc = a <= Kk ? 1 : 0;
      m |= (uint64_t)acc << l;
      a += acc;
    }
    accm[u] = m;
  }
  // (C): the accepted records in order
  {
    int base = 0;
#pragma unroll
    for (int u = 0; u < kGateK; u++) {
      const uint64_t m = accm[u];
      if ((m >> lane) & 1ull) {
        const int below = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
        acc[base + below] = rec[64 * u + lane];
      }
      base += __builtin_popcountll(m);
    }
  }
  wave_sync_lds();
  if (tick) tick[0] += wall_clock64() - t0;  // diag: (R) .. (C)
  // (B): lane c < 3 runs colour component c's chain
  if (lane < 3) {
    float f = lane == 0 ? fx : (lane == 1 ? fy : fz);
    const float* cf = reinterpret_cast<const float*>(acc) + lane;
#pragma unroll 8
    for (int i = 0; i < a; i++) f = (f + cf[4 * i]) * rrb[i];
    if (lane == 0) fx = f;
    if (lane == 1) fy = f;
    if (lane == 2) fz = f;
  }
  fx = __shfl(fx, 0, 64), fy = __shfl(fy, 1, 64), fz = __shfl(fz, 2, 64);
  r2 = R[a];
  cnt += (unsigned)a;
  if (tick) tick[1] += wall_clock64() - t0;
}

__global__ __launch_bounds__(256) void rr_table_kernel(float* rr, int n) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i < n) rr[i] = radius_reduction((unsigned)i);
}

// The expanded (group, deposit) pairs, sorted by group, materialised contiguously as what the
// update pass's filter reads for every pair: 16 B = the deposit's position and one word packing
// its photon-order index (into `dense`, where the candidates' normal, w_i and flux are read)
// with its multiplicity in that group (how many of the group's cells share the deposit's
// bucket, <= kMaxCells < 32).  The host keeps a batch below 2^27 deposits.
__global__ __launch_bounds__(256) void materialize_kernel(const unsigned* pkey, const unsigned* pval,
                                                         int n, const float4* dpos,
                                                         float4* pos) {
  const int p = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (p >= n) return;
  const unsigned i = pval[p];
  const unsigned m = pkey[p] >> kGroupBits;  // the multiplicity rides above the group bits
  const float4 x = dpos[i];
  pos[p] = make_float4(x.x, x.y, x.z, __uint_as_float((i << kRepBits) | m));
}

// One workgroup per (group, tile of <= kTileHP hit points), streaming the group's deposits
// (photon order) in windows of kWinMax.  Per window:
//  (1) every thread tests its deposits against every hit point of the tile with the radius^2
//      the hit point had at the window start — a superset of the deposits that will pass,
//      since the radius only shrinks (normal test and |v|^2 of Scene.cpp:136-137);
//  (2) the candidates are listed per hit point, in photon order;
//  (3) the state-independent term color * photon_flux (Scene.cpp:142-166) is computed for
//      the candidates by all threads;
//  (4) one thread per hit point applies the recurrence exactly, in order: r^2 re-tested with
//      the running value, r^2 *= rr(n), n++, flux = (flux + color * photon_flux) * rr(n) —
//      repeated when two of its cells share the deposit's bucket.
// The next window is fetched (coalesced) while the current one is processed.
// A tile with a compaction range (cofs[t] < cofs[t+1], tile_compact_need_kernel) takes its list
// in segments and first copies each segment's deposits its hit points can reach with their
// radius at the segment start — a superset of what any of its windows' filters passes, by the
// same argument, with the same d2 arithmetic — then runs the windows over that copy (over the
// segment itself if the copy would not fit).
__global__ __launch_bounds__(kUpdThreads) __attribute__((amdgpu_waves_per_eu(PPM_WPE, PPM_WPE))) void group_update_kernel(
    PScene S, const PHitPoint* hps, const int* perm, const int* gstart, const int2* tiles,
    const int* list_start, const int* list_end, const float4* pos, const PDeposit* dense,
    const float* rrtab, int nrr, float4* state, unsigned* nupd, const long long* cofs,
    float4* cbuf, unsigned long long* stats) {
  constexpr int kPer = kWinMax / kUpdThreads;
  constexpr int kWords = kWinMax / 32;
  constexpr int kChunk = PPM_CHUNK;  // candidates per color / apply round
  constexpr int kPerHp = kChunk / kTileHP;  // ... per hit point
  static_assert(kWinMax % kUpdThreads == 0 && kWinMax % 64 == 0, "whole waves per window");
  static_assert(kTileHP * kWords <= kUpdThreads, "one thread per mask word in the scan");
  __shared__ float s_hp[kTileHP][12];  // pos, normal, w_o, attenuation
  __shared__ int s_mat[kTileHP];
  __shared__ float s_r2[kTileHP];
  __shared__ unsigned s_cnt[kTileHP];
  __shared__ unsigned s_mask[kTileHP][kWords];
  __shared__ int s_wc[kTileHP * kWords + 1];
  __shared__ int s_wtot[kUpdThreads / 64];
  __shared__ unsigned s_ck[kTileHP * kWinMax];  // photon-order index << kRepBits | multiplicity
  // color * photon_flux, and in w the candidate's distance^2 for the gate: negated when its
  // multiplicity exceeds 1 (sign bit: the gate's scalar path), +inf when its normal fails
  __shared__ float4 s_ccf[kChunk + 4];  // (+4: gate_round reads two records ahead)
  constexpr int kRRCache = 2 * kPerHp;
  static_assert(kPerHp <= 64 * kGateK, "gate_round: candidates per lane");
  __shared__ float s_grr[kTileHP][kRRCache + kGatePad];  // gate_round: rr(grrb + i), i < kRRCache
  __shared__ float s_gR[kTileHP][kPerHp + 1 + kGatePad];  // gate_round: R(a)
  __shared__ int s_gmulti[kTileHP];  // a candidate of this round has multiplicity > 1
  __shared__ float4 s_gacc[kTileHP][kPerHp + 4];  // gate_round: the accepted records
  const int tid = (int)threadIdx.x, lane = tid & 63;
#if PPM_PHASE_TIMERS
  const unsigned long long t_start = S.diag == 2 ? wall_clock64() : 0;
#endif
  const int2 tile = tiles[blockIdx.x];
  const int g = tile.x, first = tile.y;
  const int nh = min(kTileHP, gstart[g + 1] - first);
  const int h = tid < nh ? perm[first + tid] : -1;
  V flux = mk(0, 0, 0);
  float r2 = 0.0f;
  unsigned cnt = 0;
  if (h >= 0) {
    const PHitPoint hp = hps[h];
    for (int a = 0; a < 3; a++) {
      s_hp[tid][a] = hp.pos[a], s_hp[tid][3 + a] = hp.normal[a];
      s_hp[tid][6 + a] = hp.w_o[a], s_hp[tid][9 + a] = hp.att[a];
    }
    s_mat[tid] = hp.material;
    const float4 st = state[h];
    flux = mk(st.x, st.y, st.z);
    r2 = st.w;
    cnt = nupd[h];
    s_r2[tid] = r2;
    s_cnt[tid] = cnt;
  }
  unsigned long long applied = 0, cands = 0;
  const int list_s = list_start[g], list_e = list_end[g];
  unsigned long long visits = 0, windows = 0;  // 16-B records the filters read; windows run
  __syncthreads();
  // wave j runs hit point j's recurrence (wave_gate) and keeps its state for the whole tile
  const int gw = tid >> 6;
  float gfx = 0.0f, gfy = 0.0f, gfz = 0.0f, gr2 = 0.0f;
  unsigned gcnt = 0;
  if (gw < nh) {
    const int hg = perm[first + gw];
    const float4 st = state[hg];
    gfx = st.x, gfy = st.y, gfz = st.z, gr2 = st.w;
    gcnt = s_cnt[gw];
    if (lane == 0) s_gmulti[gw] = 0;
  }
  unsigned grrb = gcnt;  // the wave's rr cache holds rr(grrb + i), i < kRRCache
#if PPM_PHASE_TIMERS
  unsigned long long gtick[2] = {0, 0};  // diag: wave 0's gate_round ticks, (R)..(C) and total
#endif
  if (gw < nh) {
    for (int i = lane; i < kRRCache; i += 64) s_grr[gw][i] = rr_at(rrtab, nrr, grrb + (unsigned)i);
  }
  const unsigned cnt0 = cnt;  // this thread's hit point's count at the start (tid < nh)
  V tp[kTileHP];
#pragma unroll
  for (int j = 0; j < kTileHP; j++) {
    tp[j] = mk(s_hp[j][0], s_hp[j][1], s_hp[j][2]);
  }
#if PPM_PHASE_TIMERS
  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0}, tp0 = 0, ctick = 0;  // ctick: compaction
#define PPM_PHASE(i)                                              \
  if (S.diag == 2 && tid == 0) {                                  \
    const unsigned long long t1 = wall_clock64();                 \
    ph[i] += t1 - tp0;                                            \
    tp0 = t1;                                                     \
  }
  if (S.diag == 2 && tid == 0) tp0 = wall_clock64();
#else
#define PPM_PHASE(i)
#endif
  // A compacted tile takes its list in segments of S.compact_seg; each segment is first copied,
  // in photon order, down to the deposits within the radius its hit points have at the
  // segment start (its windows' filters could pass no others: the radius only shrinks).
  const bool compact = cofs && cofs[blockIdx.x + 1] > cofs[blockIdx.x];
  const int seg_len = compact ? S.compact_seg : max(1, list_e - list_s);
  for (int seg = list_s; seg < list_e; seg += seg_len) {
  const int seg_e = min(seg + seg_len, list_e);
  int ls = seg, le = seg_e;
  const float4* src = pos;
  visits += (unsigned long long)(seg_e - seg);
  if (compact) {
    // (0) compaction, wave-parallel: wave w streams its own contiguous part of the segment
    // (no barrier until the end), keeping the deposits within any tile hit point's radius at
    // the segment start, in order, in its own scratch region of cap / 2 / waves records; then
    // the waves' runs are copied back to back (in wave order = photon order) into the second
    // half of the tile's range, which the windows read.  A wave whose run would not fit makes
    // the segment fall back to uncompacted windows, as the workgroup-wide version does.
    constexpr int kCW = kUpdThreads / 64;
    constexpr int kCPer = PPM_CPER;
    __shared__ int s_wn[kCW + 1];
    const long long c0 = cofs[blockIdx.x];
    const int half = (int)((cofs[blockIdx.x + 1] - c0) >> 1);
    const int wcap = half / kCW;
    float4* scratch = cbuf + c0;
    float4* dst = cbuf + c0 + half;
    const int wave = tid >> 6;
    float r2c[kTileHP];
#pragma unroll
    for (int j = 0; j < kTileHP; j++) r2c[j] = j < nh ? s_r2[j] : -1.0f;
#if PPM_PHASE_TIMERS
    const unsigned long long t_c0 = S.diag == 2 && tid == 0 ? wall_clock64() : 0;
#endif
    const int per = ((le - ls + kCW - 1) / kCW + 63) & ~63;
    const int wb = min(le, ls + wave * per), we = min(le, wb + per);
    float4* wdst = scratch + (size_t)wave * wcap;
    int n = 0;  // this wave's kept records so far (wave-uniform)
    float4 cd[kCPer];
    auto cfetch = [&](int base) {
#pragma unroll
      for (int q = 0; q < kCPer; q++) {
        const int k = base + lane + q * 64;
        if (k < we) cd[q] = pos[k];
      }
    };
    cfetch(wb);
    for (int base = wb; base < we; base += kCPer * 64) {
      float4 cw[kCPer];
#pragma unroll
      for (int q = 0; q < kCPer; q++) cw[q] = cd[q];
      cfetch(base + kCPer * 64);  // next round in flight
#pragma unroll
      for (int q = 0; q < kCPer; q++) {
        const V x = mk(cw[q].x, cw[q].y, cw[q].z);
        bool kp = false;
#pragma unroll
        for (int j = 0; j < kTileHP; j++) {
          const V v = tp[j] - x;
          kp = kp || (dot(v, v) <= r2c[j]);
        }
        kp = kp && base + lane + q * 64 < we;
        const unsigned long long bal = __ballot(kp);
        const int rank = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
        if (kp && n + rank < wcap) wdst[n + rank] = cw[q];
        n += __builtin_popcountll(bal);
      }
    }
    if (lane == 0) s_wn[wave] = n;
    __syncthreads();
    int kept = 0, off = 0;
    bool fits = true;
#pragma unroll
    for (int w = 0; w < kCW; w++) {
      const int nw = s_wn[w];
      fits = fits && nw <= wcap;
      if (w < wave) off += nw;
      kept += nw;
    }
    if (fits) {  // this wave's run to its place in the contiguous copy
      for (int i = lane; i < n; i += 64) dst[off + i] = wdst[i];
    }
    __syncthreads();  // the copy is read by other threads of the workgroup below
#if PPM_PHASE_TIMERS
    if (S.diag == 2 && tid == 0) ctick += wall_clock64() - t_c0;
#endif
    if (fits) {
      src = dst, ls = 0, le = kept;
      visits += (unsigned long long)kept;
    }
    if (stats && tid == 0) {
      atomicAdd(&stats[fits ? 20 : 21], 1ull);
      atomicAdd(&stats[22], (unsigned long long)kept);
    }
    PPM_PHASE(0)
  }
  windows += (unsigned long long)((le - ls + kWinMax - 1) / kWinMax);
  float4 dep[kPer];  // position, photon-order index << kRepBits | multiplicity
  auto fetch = [&](int base) {
#pragma unroll
    for (int q = 0; q < kPer; q++) {
      const int k = base + tid + q * kUpdThreads;
      if (k < le) dep[q] = src[k];
    }
  };
  fetch(ls);
  for (int base = ls; base < le; base += kWinMax) {
    const int total = min(kWinMax, le - base);
    const int nwords = (total + 31) >> 5;
    // (1) superset filter
    float r2w[kTileHP];
#pragma unroll
    for (int j = 0; j < kTileHP; j++) r2w[j] = s_r2[j];
    float d2r[kPer][kTileHP];
    bool cr[kPer][kTileHP];
    unsigned rp[kPer];  // index | multiplicity words, kept past the next window's fetch
#pragma unroll
    for (int q = 0; q < kPer; q++) {
      const int k = tid + q * kUpdThreads;  // a wave covers 64 consecutive deposits
      const bool live = k < total;
      const V x = mk(dep[q].x, dep[q].y, dep[q].z);
      rp[q] = __float_as_uint(dep[q].w);
#pragma unroll
      for (int j = 0; j < kTileHP; j++) {
        const V v = tp[j] - x;
        d2r[q][j] = dot(v, v);
        // the normal test of Scene.cpp:136 is applied to the candidates (color phase)
        cr[q][j] = live && j < nh && (d2r[q][j] <= r2w[j]);
        const unsigned long long bal = __ballot(cr[q][j]);
        if (lane == 0) {
          s_mask[j][(k - lane) >> 5] = (unsigned)bal;
          s_mask[j][((k - lane) >> 5) + 1] = (unsigned)(bal >> 32);
        }
      }
    }
    fetch(base + kWinMax);  // next window in flight
    __syncthreads();
    PPM_PHASE(0)
    // (2) candidates per hit point, in photon order: exclusive scan of the per-word counts,
    // one word per thread (wave scans, then the wave totals)
    {
      const int n = nh * nwords;
      const int v = tid < n ? __builtin_popcount(s_mask[tid / nwords][tid % nwords]) : 0;
      int x = v;
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      if (lane == 63) s_wtot[tid >> 6] = x;
      __syncthreads();
      PPM_PHASE(1)
      int off = 0;
      for (int w = 0; w < (tid >> 6); w++) off += s_wtot[w];
      if (tid < n) s_wc[tid] = off + x - v;
      if (tid == n - 1) s_wc[n] = off + x;
    }
    __syncthreads();
    PPM_PHASE(2)
#pragma unroll
    for (int q = 0; q < kPer; q++) {
      const int k = tid + q * kUpdThreads;
#pragma unroll
      for (int j = 0; j < kTileHP; j++) {
        if (!cr[q][j]) continue;
        const int w = k >> 5;
        const int idx = s_wc[j * nwords + w] + __builtin_popcount(s_mask[j][w] & ((1u << (k & 31)) - 1u));
        s_ck[idx] = rp[q];
      }
    }
    __syncthreads();
    PPM_PHASE(3)
    const int ncand = s_wc[nh * nwords];
    cands += (unsigned)ncand;
    // Rounds of up to kPerHp candidates of EVERY hit point, so that the gate lanes run side by
    // side however the window's candidates are spread over the tile's hit points.
    int most = 0;
    for (int j = 0; j < nh; j++)
      most = max(most, (j + 1 < nh ? s_wc[(j + 1) * nwords] : ncand) - s_wc[j * nwords]);
    for (int c0 = 0; c0 < most; c0 += kPerHp) {
      // (3) color * photon_flux for candidates [c0, c0 + kPerHp) of each hit point
      for (int x = tid; x < nh * kPerHp; x += kUpdThreads) {
        const int j = x / kPerHp;
        const int e = s_wc[j * nwords] + c0 + (x - j * kPerHp);
        if (e >= (j + 1 < nh ? s_wc[(j + 1) * nwords] : ncand)) continue;
        const PDeposit d = dense[s_ck[e] >> kRepBits];
        const V hn = mk(s_hp[j][3], s_hp[j][4], s_hp[j][5]), w_i = ld(d.w_i), pf = ld(d.flux);
        const PMaterial& m = S.materials[s_mat[j]];
        V color = mk(0.0f, 0.0f, 0.0f);
        // Scene.cpp:136: a deposit whose normal fails the test never updates the hit point
        const bool normal_ok = dot(hn, ld(d.normal)) > 1e-3f;
        if (normal_ok && m.brdf_id == -1) {
          const float cos_i = dot(hn, w_i);
          if (!(cos_i > 1.0f || cos_i <= 0.0f)) {
            const V w_o = mk(s_hp[j][6], s_hp[j][7], s_hp[j][8]);
            const float sc = fmax0(dot(hn, normalize(w_o + w_i)));
            color = (ld(m.diffuse) + (ld(m.specular) * ppm_math::powf_ieee(sc, m.phong)) / cos_i) *
                    mk(s_hp[j][9], s_hp[j][10], s_hp[j][11]);
          }
        }
        const V cf = color * pf;
        // distance^2 as the filter computed it (same operands, same arithmetic)
        const V dv = mk(s_hp[j][0], s_hp[j][1], s_hp[j][2]) - ld(d.x);
        const float d2 = dot(dv, dv);
        const bool multi = normal_ok && (s_ck[e] & kRepMask) > 1u;
        const float d2c = !normal_ok ? kInf : (multi ? -d2 : d2);
        if (multi) s_gmulti[j] = 1;
        s_ccf[x] = make_float4(cf.x, cf.y, cf.z, d2c);
      }
      __syncthreads();
      PPM_PHASE(4)
      // (4) the exact recurrence, in photon order: wave gw applies this round's candidates of
      // its hit point (gate_round: radius table, acceptance runs, flux chains; a candidate of
      // multiplicity > 1 sends the round through the one-at-a-time loop), after sliding its
      // staged rr(n) cache to the hit point's count when the round could run past it
      if (gw < nh && S.diag != 1) {
        const int gb = s_wc[gw * nwords];
        const int ge = gw + 1 < nh ? s_wc[(gw + 1) * nwords] : ncand;
        const int n = min(ge, gb + c0 + kPerHp) - (gb + c0);
        __builtin_amdgcn_s_setprio(PPM_GATE_PRIO);
        if (gcnt + (unsigned)n > grrb + (unsigned)kRRCache) {  // slide the rr cache to cnt
          grrb = gcnt;
          for (int i = lane; i < kRRCache; i += 64) s_grr[gw][i] = rr_at(rrtab, nrr, grrb + (unsigned)i);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        const bool multi = s_gmulti[gw] != 0;
        gate_round(s_ccf + gw * kPerHp, s_gacc[gw], n, multi, s_ck + gb + c0, rrtab, nrr,
                   s_grr[gw] + (gcnt - grrb), s_gR[gw], gfx, gfy, gfz, gr2, gcnt,
#if PPM_PHASE_TIMERS
                   S.diag == 2 && gw == 0 ? gtick : nullptr);
#else
                   nullptr);
#endif
        __builtin_amdgcn_s_setprio(0);
        if (lane == 0) s_r2[gw] = gr2, s_cnt[gw] = gcnt, s_gmulti[gw] = 0;
      }
      __syncthreads();
      PPM_PHASE(5)
    }
    __syncthreads();
    PPM_PHASE(5)
  }
  }  // segments
  if (gw < nh && lane == 0) {
    state[perm[first + gw]] = make_float4(gfx, gfy, gfz, gr2);
    nupd[perm[first + gw]] = gcnt;
  }
  __syncthreads();
  if (h >= 0) applied = s_cnt[tid] - cnt0;
  const unsigned long long tot = wave_sum(applied);
  if (stats && (tid & 63) == 0 && tot) atomicAdd(&stats[3], tot);
  if (stats && tid == 0) {  // the pass's work: (tile, deposit) pairs filtered, candidates
    atomicAdd(&stats[6], visits);
    atomicAdd(&stats[16], cands);
  }
  if (stats && S.diag == 2 && tid == 0) {  // experiment counters: windows, longest tile
    atomicAdd(&stats[5], windows);
#if PPM_PHASE_TIMERS
    const unsigned long long dur = wall_clock64() - t_start;
    atomicMax(&stats[7], dur);  // longest tile, in wall-clock ticks
    atomicAdd(&stats[23], dur);  // sum over tiles, and of each phase (23..29)
    atomicAdd(&stats[30], gtick[0]);  // hit point 0's gate_round: (R)+(K), all phases
    atomicAdd(&stats[31], gtick[1]);
    for (int i = 0; i < 6; i++) atomicAdd(&stats[24 + i], ph[i]);
    atomicAdd(&stats[32], ctick);
    atomicMax(&stats[33], ctick);
    for (int i = 0; i < 6; i++) atomicMax(&stats[8 + i], ph[i]);
#endif
    atomicMax(&stats[17], cands);  // most candidates in one tile
    atomicMax(&stats[19], windows);
  }
  if (stats && S.diag == 2 && (tid & 63) == 0 && tot) atomicMax(&stats[18], tot);  // (per wave)
#undef PPM_PHASE
}

// density_estimation + Pixel::get_color: a pixel's hit points are contiguous, in order.
__global__ __launch_bounds__(256) void density_kernel(const PHitPoint* hps, const float4* state,
                                                      const int* pix_offsets, int npix,
                                                      double total, float* out) {
  const int p = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (p >= npix) return;
  V col = mk(0.0f, 0.0f, 0.0f);
  float wsum = 0.0f;
  for (int k = pix_offsets[p]; k < pix_offsets[p + 1]; k++) {
    const float4 st = state[k];
    const float s = (float)(1.0f / ((M_PI * (double)st.w) * total));
    const float w = hps[k].weight;
    col = col + (mk(st.x, st.y, st.z) * s) * w;
    wsum = wsum + w;
  }
  const V c = wsum == 0 ? mk(0.0f, 0.0f, 0.0f) : col / wsum;
  out[3 * p] = c.x;
  out[3 * p + 1] = c.y;
  out[3 * p + 2] = c.z;
}

// ------------------------------------------------------------------ launchers (ppm_api.hip)
constexpr int kThreads = kPpmThreads;
static int blocks_for(long long n) { return (int)((n + kThreads - 1) / kThreads); }

hipError_t launch_eye(const PScene& S, const PCamera& C, unsigned long long seed, int* counts,
                      const int* offsets, PHitPoint* out, unsigned long long* stats,
                      hipStream_t st) {
  const dim3 grid(blocks_for((long long)C.width * C.height));
  if (S.lds_stack)
    hipLaunchKernelGGL(eye_kernel<true>, grid, dim3(kThreads), 0, st, S, C, seed, counts, offsets,
                       out, stats);
  else
    hipLaunchKernelGGL(eye_kernel<false>, grid, dim3(kThreads), 0, st, S, C, seed, counts,
                       offsets, out, stats);
  return hipGetLastError();
}
hipError_t launch_grid(const PHitPoint* hps, int n, int w, int h, PGrid* grid, float4* state,
                       unsigned* counts, hipStream_t st) {
  hipLaunchKernelGGL(grid_kernel, dim3(1), dim3(1024), 0, st, hps, n, w, h, grid, state, counts);
  return hipGetLastError();
}
hipError_t launch_photons(const PScene& S, unsigned long long seed, long long first, int count,
                          int K, PDeposit* slots, int* ndep, unsigned long long* stats,
                          hipStream_t st) {
  // workgroups of a contiguous photon range each (2048: 3.99 ms, 4096: 3.72 ms on C5)
  const int blocks = std::min(blocks_for(count), PPM_PHOTON_BLOCKS);
  if (blocks <= 0) return hipSuccess;
  if (S.lds_stack)
    hipLaunchKernelGGL(photon_kernel<true>, dim3(blocks), dim3(kThreads), 0, st, S, seed, first,
                       count, K, slots, ndep, stats);
  else
    hipLaunchKernelGGL(photon_kernel<false>, dim3(blocks), dim3(kThreads), 0, st, S, seed, first,
                       count, K, slots, ndep, stats);
  return hipGetLastError();
}
hipError_t launch_deposit_keys(const PDeposit* slots, const int* ndep, const int* offsets,
                               int count, int K, const PGrid* grid, unsigned* bucket,
                               PDeposit* dense, float4* dpos, hipStream_t st) {
  hipLaunchKernelGGL(deposit_keys_kernel, dim3(blocks_for(count)), dim3(kThreads), 0, st, slots,
                     ndep, offsets, count, K, grid, bucket, dense, dpos);
  return hipGetLastError();
}
hipError_t launch_group_buckets(const PHitPoint* hps, const int* perm, const int* gstart,
                                int groups, const PGrid* grid, unsigned* gb, int* gm, int* gnb,
                                hipStream_t st) {
  hipLaunchKernelGGL(group_buckets_kernel, dim3(blocks_for(groups + 1)), dim3(kThreads), 0, st,
                     hps, perm, gstart, groups, grid, gb, gm, gnb);
  return hipGetLastError();
}
hipError_t launch_bucket_group_pairs(const unsigned* gb, const int* gm, const int* gnb,
                                     const int* goff, int groups, unsigned* key, unsigned* val,
                                     hipStream_t st) {
  hipLaunchKernelGGL(bucket_group_pairs_kernel, dim3(blocks_for(groups)), dim3(kThreads), 0, st,
                     gb, gm, gnb, goff, groups, key, val);
  return hipGetLastError();
}
hipError_t launch_expand_count(const unsigned* bucket, int n, const int* bg_start,
                               const int* bg_end, int* count, hipStream_t st) {
  hipLaunchKernelGGL(expand_count_kernel, dim3(blocks_for(n + 1)), dim3(kThreads), 0, st, bucket,
                     n, bg_start, bg_end, count);
  return hipGetLastError();
}
hipError_t launch_expand_write(const unsigned* bucket, int n, const int* bg_start,
                               const int* bg_end, const unsigned* bg_group, const int* off,
                               unsigned* key, unsigned* val, hipStream_t st) {
  hipLaunchKernelGGL(expand_write_kernel, dim3(blocks_for(n)), dim3(kThreads), 0, st, bucket, n,
                     bg_start, bg_end, bg_group, off, key, val);
  return hipGetLastError();
}
hipError_t launch_bucket_bounds(const unsigned* keys, int n, unsigned mask, int* start, int* end,
                                hipStream_t st) {
  hipLaunchKernelGGL(bucket_bounds_kernel, dim3(blocks_for(n)), dim3(kThreads), 0, st, keys, n,
                     mask, start, end);
  return hipGetLastError();
}
hipError_t launch_group_keys(const PHitPoint* hps, int n, const PGrid* grid,
                            unsigned long long* keys, int* idx, int* error, hipStream_t st) {
  hipLaunchKernelGGL(group_key_kernel, dim3(blocks_for(n)), dim3(kThreads), 0, st, hps, n, grid,
                     keys, idx, error);
  return hipGetLastError();
}
hipError_t launch_group_flags(const unsigned long long* keys, int n, int* flags, hipStream_t st) {
  hipLaunchKernelGGL(group_flags_kernel, dim3(blocks_for(n + 1)), dim3(kThreads), 0, st, keys, n,
                     flags);
  return hipGetLastError();
}
hipError_t launch_group_starts(const int* flags, const int* gid, int n, int* gstart,
                               hipStream_t st) {
  hipLaunchKernelGGL(group_starts_kernel, dim3(blocks_for(n + 1)), dim3(kThreads), 0, st, flags,
                     gid, n, gstart);
  return hipGetLastError();
}
hipError_t launch_group_tiles(const int* gstart, int groups, int* ntile, hipStream_t st) {
  hipLaunchKernelGGL(group_tiles_kernel, dim3(blocks_for(groups + 1)), dim3(kThreads), 0, st,
                     gstart, groups, ntile);
  return hipGetLastError();
}
hipError_t launch_tile_table(const int* gstart, const int* tile_off, int groups, int2* tiles,
                             hipStream_t st) {
  hipLaunchKernelGGL(tile_table_kernel, dim3(blocks_for(groups)), dim3(kThreads), 0, st, gstart,
                     tile_off, groups, tiles);
  return hipGetLastError();
}
hipError_t launch_tile_shard(const int2* all, int ntiles, int shard, int shards, const int* gstart,
                             const int* perm, int2* mine, int* owner, hipStream_t st) {
  if (ntiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(tile_shard_kernel, dim3(blocks_for(ntiles)), dim3(kThreads), 0, st, all,
                     ntiles, shard, shards, gstart, perm, mine, owner);
  return hipGetLastError();
}
hipError_t launch_merge_state(const int* owner, int n, int self, const float4* peer_state,
                              const unsigned* peer_nupd, float4* state, unsigned* nupd,
                              hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(merge_state_kernel, dim3(blocks_for(n)), dim3(kThreads), 0, st, owner, n,
                     self, peer_state, peer_nupd, state, nupd);
  return hipGetLastError();
}
hipError_t launch_tile_work(const int2* tiles, int ntiles, const int* list_start,
                           const int* list_end, unsigned* key, hipStream_t st) {
  hipLaunchKernelGGL(tile_work_kernel, dim3(blocks_for(ntiles)), dim3(kThreads), 0, st, tiles,
                     ntiles, list_start, list_end, key);
  return hipGetLastError();
}
hipError_t launch_rr_table(float* rr, int n, hipStream_t st) {
  hipLaunchKernelGGL(rr_table_kernel, dim3(blocks_for(n)), dim3(kThreads), 0, st, rr, n);
  return hipGetLastError();
}
hipError_t launch_materialize(const unsigned* pkey, const unsigned* pval, int n,
                              const float4* dpos, float4* pos, hipStream_t st) {
  hipLaunchKernelGGL(materialize_kernel, dim3(blocks_for(n)), dim3(kThreads), 0, st, pkey, pval,
                     n, dpos, pos);
  return hipGetLastError();
}
hipError_t launch_group_update(const PScene& S, const PHitPoint* hps, const int* perm,
                               const int* gstart, const int2* tiles, int ntiles,
                               const int* list_start, const int* list_end, const float4* pos,
                               const PDeposit* dense, const float* rrtab, int nrr,
                               float4* state, unsigned* nupd, const long long* cofs,
                               float4* cbuf, unsigned long long* stats, hipStream_t st) {
  if (ntiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(group_update_kernel, dim3(ntiles), dim3(kUpdThreads), 0, st, S, hps, perm,
                     gstart, tiles, list_start, list_end, pos, dense, rrtab, nrr, state, nupd,
                     cofs, cbuf, stats);
  return hipGetLastError();
}
hipError_t launch_tile_compact_need(const int2* tiles, int ntiles, const int* list_start,
                                    const int* list_end, long long min_len, int shift, int seg,
                                    long long* need, hipStream_t st) {
  hipLaunchKernelGGL(tile_compact_need_kernel, dim3(blocks_for(ntiles + 1)), dim3(kThreads), 0, st,
                     tiles, ntiles, list_start, list_end, min_len, shift, seg, need);
  return hipGetLastError();
}
hipError_t launch_density(const PHitPoint* hps, const float4* state, const int* pix_offsets,
                          int npix, double total, float* out, hipStream_t st) {
  hipLaunchKernelGGL(density_kernel, dim3(blocks_for(npix)), dim3(kThreads), 0, st, hps, state,
                     pix_offsets, npix, total, out);
  return hipGetLastError();
}

}  // namespace ppm
