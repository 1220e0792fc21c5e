// MI355X (gfx950) render kernels: HW2's Scene::render_image -> trace_ray -> BVH::intersect ->
// Triangle/Sphere::intersect -> Point_light shading + shadow rays, as one fused kernel.
//
// Execution model:
//   * one wavefront = one 8x8 pixel packet; 4 packets per 256-thread workgroup;
//   * the wave walks the BVH TOGETHER: the current node index and the 64-bit lane mask of
//     the rays that accepted every box on the path are wave-uniform (SGPRs), so node and
//     primitive records come in through the scalar cache (s_load) once per wave, not once
//     per lane;
//   * the traversal stack is one entry per VGPR lane (lane-select push, v_readlane pop, 64 deep);
//     trees deeper than that use a per-wave LDS stack (kDeepStack entries);
//   * per-lane masks reproduce the reference's per-ray semantics exactly: a ray tests a node
//     iff it accepted every ancestor's box (HW2/Bounding_volume_hierarchy.cpp:31-55);
//   * closest hit = lexicographic minimum of (t, DFS leaf index) over accepted leaves, which
//     is what the reference's left-first recursion with strict `<` returns (appendix A.5), so
//     any visiting order gives the reference's answer.
//
// Numerics: compiled with -ffp-contract=off and this file's pragma; '/' is the correctly
// rounded fp32 division and sqrtf is correctly rounded on gfx950 (HIP defaults), pow / exp
// / log are the fp64 ocml functions, matching the reference's double libm islands.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "rt_internal.h"

#pragma clang fp contract(off)

namespace rt {

#define RT_INF __builtin_huge_valf()
constexpr float kEps = 0.000001f;  // HW2/Vector3.h:7 kEpsilon
constexpr int kCounterSlots = kCounterRows;
#ifndef RT_RAYS_PER_LANE
#define RT_RAYS_PER_LANE 1
#endif
constexpr int kRaysPerLane = RT_RAYS_PER_LANE;  // tiles per wave in the traversal kernels

#ifdef RT_DIAG
#define DIAG(stmt) stmt
#else
#define DIAG(stmt)
#endif
struct Diag {  // per-wave traversal work (RT_DIAG builds)
  unsigned long long nodes = 0, node_lanes = 0, leaves = 0, leaf_lanes = 0, exact = 0, wide = 0;
};

// ------------------------------------------------------------------ vector helpers
struct V3 {
  float x, y, z;
};
__device__ __forceinline__ V3 v3(float x, float y, float z) { return {x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 operator*(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ V3 operator/(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
__device__ __forceinline__ float dot(V3 a, V3 b) { return (a.x * b.x) + (a.y * b.y) + (a.z * b.z); }
__device__ __forceinline__ float length(V3 a) { return __builtin_sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }
__device__ __forceinline__ V3 normalize(V3 a) { return a / length(a); }
__device__ __forceinline__ V3 ld3(const float* p) { return {p[0], p[1], p[2]}; }

struct LaneRay {
  V3 o, d;
  V3 r;       // v_rcp_f32 reciprocals (<= 1 ulp): the approximate slab test only
  bool skip0, skip1, skip2;  // |d_i| < 1e-6: axis ignored (HW2/bounding_box.cpp:21)
  bool quot;  // origin and scene in the shared-reciprocal range (tri_quotients)
};

__device__ __forceinline__ bool quot_coord(float x) {  // quot_coord_ok of rt_internal.h
  const float a = __builtin_fabsf(x);
  return a == 0.0f || (a >= 0x1p-26f && a <= 0x1p48f);
}

__device__ __forceinline__ LaneRay make_ray(V3 o, V3 d, int scene_quot_ok) {
  LaneRay r;
  r.o = o;
  r.d = d;
  r.r = v3(__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y), __builtin_amdgcn_rcpf(d.z));
  r.skip0 = __builtin_fabsf(d.x) < kEps;
  r.skip1 = __builtin_fabsf(d.y) < kEps;
  r.skip2 = __builtin_fabsf(d.z) < kEps;
  r.quot = scene_quot_ok && quot_coord(o.x) && quot_coord(o.y) && quot_coord(o.z);
  return r;
}

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }

// ------------------------------------------------------------------ slab test
// Literal HW2/bounding_box.cpp:15-35 + the caller's reject rule (BVH.cpp:32-35).  Used when
// the fast test below cannot decide.  Its comparisons are the reference's, so NaN / inf
// inputs behave as there.
__device__ __forceinline__ bool box_exact(const float* b, const LaneRay& r) {
  float tmin = -RT_INF, tmax = RT_INF;
  const float o[3] = {r.o.x, r.o.y, r.o.z};
  const float d[3] = {r.d.x, r.d.y, r.d.z};
#pragma unroll
  for (int i = 0; i < 3; i++) {
    if (__builtin_fabsf(d[i]) < kEps) continue;
    float t0 = (b[i] - o[i]) / d[i];
    float t1 = (b[i + 3] - o[i]) / d[i];
    if (d[i] < 0) {
      const float s = t0;
      t0 = t1;
      t1 = s;
    }
    if (t0 > tmin) tmin = t0;
    if (t1 < tmax) tmax = t1;
    if (tmin > tmax) return false;
  }
  const float bt = tmin > 0.0f ? tmin : tmax;
  return !(bt < 0.0f || bt == RT_INF);
}

#ifdef RT_DIAG
__device__ unsigned long long g_exact_fallbacks;  // lanes that needed box_exact
#endif

// Fast slab test.  With q = RN(RN(m - o) / d) the reference's quotient and q' = RN(RN(m - o)
// * rcp(d)) ours, |q' - q| <= 2^-22 |q| and sign(q') == sign(q) exactly.  The reference
// accepts iff tmin <= tmax and tmax >= 0 (tmin, tmax finite here): the sign test is exact, and
// the order test is decided here only outside a 2^-20 relative band; inside it the lane is
// flagged for box_exact.  Written branch-free: both children of a node are tested together.
// tnear (approximate entry distance) only orders and culls.
template <bool SKIP>
__device__ __forceinline__ void slab_span(const float* b, const LaneRay& r, float& tn, float& tf) {
  const float ax = (b[0] - r.o.x) * r.r.x, bx = (b[3] - r.o.x) * r.r.x;
  const float ay = (b[1] - r.o.y) * r.r.y, by = (b[4] - r.o.y) * r.r.y;
  const float az = (b[2] - r.o.z) * r.r.z, bz = (b[5] - r.o.z) * r.r.z;
  float nx = __builtin_fminf(ax, bx), fx = __builtin_fmaxf(ax, bx);
  float ny = __builtin_fminf(ay, by), fy = __builtin_fmaxf(ay, by);
  float nz = __builtin_fminf(az, bz), fz = __builtin_fmaxf(az, bz);
  if (SKIP) {
    nx = r.skip0 ? -RT_INF : nx;
    fx = r.skip0 ? RT_INF : fx;
    ny = r.skip1 ? -RT_INF : ny;
    fy = r.skip1 ? RT_INF : fy;
    nz = r.skip2 ? -RT_INF : nz;
    fz = r.skip2 ? RT_INF : fz;
  }
  tn = __builtin_fmaxf(__builtin_fmaxf(nx, ny), nz);
  tf = __builtin_fminf(__builtin_fminf(fx, fy), fz);
}

// Two slab spans at once (slots c and c + 1 of a wide node): b - o and * rcp as v_pk_add_f32 /
// v_pk_mul_f32, each element rounded exactly as the scalar op, the min / max per element.
typedef float f32x2v __attribute__((ext_vector_type(2)));
template <bool SKIP>
__device__ __forceinline__ void slab_span2(const float lo[3][4], const float hi[3][4], int c,
                                           const LaneRay& r, float tn[2], float tf[2]) {
  const f32x2v ox = {r.o.x, r.o.x}, oy = {r.o.y, r.o.y}, oz = {r.o.z, r.o.z};
  const f32x2v rx = {r.r.x, r.r.x}, ry = {r.r.y, r.r.y}, rz = {r.r.z, r.r.z};
  const f32x2v ax = (f32x2v{lo[0][c], lo[0][c + 1]} - ox) * rx;
  const f32x2v bx = (f32x2v{hi[0][c], hi[0][c + 1]} - ox) * rx;
  const f32x2v ay = (f32x2v{lo[1][c], lo[1][c + 1]} - oy) * ry;
  const f32x2v by = (f32x2v{hi[1][c], hi[1][c + 1]} - oy) * ry;
  const f32x2v az = (f32x2v{lo[2][c], lo[2][c + 1]} - oz) * rz;
  const f32x2v bz = (f32x2v{hi[2][c], hi[2][c + 1]} - oz) * rz;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    float nx = __builtin_fminf(ax[k], bx[k]), fx = __builtin_fmaxf(ax[k], bx[k]);
    float ny = __builtin_fminf(ay[k], by[k]), fy = __builtin_fmaxf(ay[k], by[k]);
    float nz = __builtin_fminf(az[k], bz[k]), fz = __builtin_fmaxf(az[k], bz[k]);
    if (SKIP) {
      nx = r.skip0 ? -RT_INF : nx;
      fx = r.skip0 ? RT_INF : fx;
      ny = r.skip1 ? -RT_INF : ny;
      fy = r.skip1 ? RT_INF : fy;
      nz = r.skip2 ? -RT_INF : nz;
      fz = r.skip2 ? RT_INF : fz;
    }
    tn[k] = __builtin_fmaxf(__builtin_fmaxf(nx, ny), nz);
    tf[k] = __builtin_fminf(__builtin_fminf(fx, fy), fz);
  }
}

// sure_in: the reference accepts (tf >= 0, and tn <= tf decided outside a 2^-20 relative
// band); sure_out: it rejects.  Neither: box_exact decides (NaN lands here too).  The sign of
// each bound is exact (RN(b - o) * rcp(d) has the sign of the reference's quotient), and
// d = RN(tn - tf) is within 2^-24 of tn - tf, so a decided case keeps a true margin above
// 2^-21 relative.
__device__ __forceinline__ void decide_sure(float tn, float tf, bool& sure_in, bool& sure_out) {
  const float band = __builtin_fmaf(__builtin_fabsf(tn) + __builtin_fabsf(tf), 0x1p-20f, 0x1p-120f);
  const float d = tn - tf;
  sure_in = (d < -band) & (tf >= 0.0f);
  sure_out = (tf < 0.0f) | (d > band);
}

__device__ __forceinline__ void decide_fast(float tn, float tf, bool& accept, bool& undecided) {
  bool out;
  decide_sure(tn, tf, accept, out);
  undecided = !(accept | out);
}

template <bool SKIP>
__device__ __forceinline__ void slab_fast(const float* b, const LaneRay& r, float& tn,
                                          bool& accept, bool& undecided) {
  float tf;
  slab_span<SKIP>(b, r, tn, tf);
  decide_fast(tn, tf, accept, undecided);
}

// Culling-tree boxes (accel_build.cpp) contain every reference box below them.  If the
// reference test accepts a contained box, the exact t-intervals nest and every computed
// bound is within 2^-22 relative of its exact value, so the container is never `sure_out`
// (2^-20 band, same skipped axes): a culling node never drops a treelet the reference would
// enter.  Its test is therefore just !sure_out.
__device__ __forceinline__ bool decide_cull(float tn, float tf) {
  bool in, out;
  decide_sure(tn, tf, in, out);
  return !out;
}

// ------------------------------------------------------------------ primitives
// HW2/Triangle.cpp:35-65 with determinant() = Triangle.h:33-38, v0 - v1 / v0 - v2 precomputed
// on the host with the same fp32 rounding.
__device__ __forceinline__ float det3(V3 c1, V3 c2, V3 c3) {
  return c1.x * (c2.y * c3.z - c3.y * c2.z) + c2.x * (c3.y * c1.z - c1.y * c3.z) +
         c3.x * (c1.y * c2.z - c2.y * c1.z);
}

// det3(a1, a2, c3) with the c3-free minor `cx` = a1.y*a2.z - a2.y*a1.z precomputed (same bits)
__device__ __forceinline__ float det3_cx(V3 c1, V3 c2, V3 c3, float cx) {
  return c1.x * (c2.y * c3.z - c3.y * c2.z) + c2.x * (c3.y * c1.z - c1.y * c3.z) + c3.x * cx;
}

// Correctly rounded n / det for the three numerators with ONE reciprocal.  gfx950's IEEE
// division is v_div_scale (num, den), y = v_rcp, e = fma(-den, y, 1), y1 = fma(e, y, y),
// q = num * y1, r = fma(-den, q, num), q1 = fma(r, y1, q), r1 = fma(-den, q1, num),
// v_div_fmas(r1, y1, q1), v_div_fixup(q2, den, num).  When no operand is near the exponent
// limits, v_div_scale returns its operand unchanged with VCC = 0 and v_div_fmas is a plain
// fma, so the sequence below (which keeps v_div_fixup: it gives a zero numerator the sign
// num ^ den) yields the bits of `/`; only the reciprocal refinement y1 depends on det alone,
// and it is shared.  Range: 2^-40 <= |det|
// <= 2^40 is checked here; numerators are 0 or 2^-49 <= |n| <= 2^49 by r.quot (every v0 and
// origin coordinate is 0 or in [2^-26, 2^48]).  Then |n / det| lies in [2^-89, 2^89],
// exponent differences stay below 96 and nothing is subnormal, so none of v_div_scale's
// scaling cases can arise.  Any other lane takes `/`.
__device__ __forceinline__ float quot_step(float n, float det, float y1) {
  const float q = n * y1;
  const float r = __builtin_fmaf(-det, q, n);
  const float q1 = __builtin_fmaf(r, y1, q);
  const float r1 = __builtin_fmaf(-det, q1, n);
  return __builtin_amdgcn_div_fixupf(__builtin_fmaf(r1, y1, q1), det, n);
}

__device__ __forceinline__ V3 tri_quotients(V3 n, float det, bool quot) {
#ifndef RT_EXP_IEEEDIV
  const float ad = __builtin_fabsf(det);
  if (quot && ad >= 0x1p-40f && ad <= 0x1p40f) {
    const float y = __builtin_amdgcn_rcpf(det);
    const float e = __builtin_fmaf(-det, y, 1.0f);
    const float y1 = __builtin_fmaf(e, y, y);
    return v3(quot_step(n.x, det, y1), quot_step(n.y, det, y1), quot_step(n.z, det, y1));
  }
#endif
  return n / det;
}

__device__ __forceinline__ bool tri_test(V3 v0, V3 a1, V3 a2, float cx, const LaneRay& r,
                                         float& t) {
#ifndef RT_EXP_CX
#define det3_cx(c1, c2, c3, cx) det3(c1, c2, c3)
#endif
  const float det = det3_cx(a1, a2, r.d, cx);
#ifndef RT_EXP_BRANCHY  // (RT_EXP_BRANCHY: the early-exit form, for A/B)
  // Branch-free: every value is computed and the reference's early exits (Triangle.cpp:46-62)
  // become one predicate with the same comparisons (a NaN fails them as there).  No
  // exec-mask save/restore per exit; with det == 0 the quotients are inf/NaN and unused.
  const V3 b = tri_quotients(v0 - r.o, det, r.quot);
  const float beta = det3(b, a2, r.d);
  const float gamma = det3(a1, b, r.d);
  const float tt = det3_cx(a1, a2, b, cx);
  t = tt;
  return (det != 0.0f) & !((beta < 0.0f) | (beta > 1.0f)) &
         !((gamma < 0.0f) | (beta + gamma > 1.0f)) & (tt > 0.0f);
#else
  if (det == 0.0f) return false;
  const V3 b = tri_quotients(v0 - r.o, det, r.quot);
  const float beta = det3(b, a2, r.d);
  if (beta < 0.0f || beta > 1.0f) return false;
  const float gamma = det3(a1, b, r.d);
  if (gamma < 0.0f || beta + gamma > 1.0f) return false;
  const float tt = det3_cx(a1, a2, b, cx);
  if (tt > 0.0f) {
    t = tt;
    return true;
  }
  return false;
#endif
}

// HW2/Sphere.h:26-52 — true for any real root, including a negative one.
__device__ __forceinline__ bool sphere_test(V3 c, float radius, const LaneRay& r, float& t) {
  const V3 co = r.o - c;
  const float a = dot(r.d, r.d);
  const float b = 2 * dot(r.d, co);
  const float cc = dot(co, co) - radius * radius;
  const float disc = b * b - 4 * a * cc;
  if (disc < -kEps) return false;
  if (disc < kEps) {
    t = -b / (2 * a);
  } else {
    const float sq = __builtin_sqrtf(disc);  // == (float)sqrt((double)disc)
    const float t1 = (-b + sq) / (2 * a);
    const float t2 = (-b - sq) / (2 * a);
    t = t2 < 0.0f ? t1 : t2;
  }
  return true;
}

// Shape::intersect of one leaf.  SPHERES == false: the scene has no spheres (host flag), so
// the sphere code is not compiled into the traversal loop.
// RT_EXP_X16: fetch a node / prim record with ONE s_load_dwordx16 (waited at once) instead of
// the 4 loads of 1-8 dwords the compiler splits it into.
typedef int v16i __attribute__((ext_vector_type(16)));
__device__ __forceinline__ v16i sload16(const void* p) {
  v16i r;
  asm volatile("s_load_dwordx16 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(p) : "memory");
  return r;
}

template <bool SPHERES>
__device__ __forceinline__ bool leaf_test(const DevPrim* __restrict__ prims, int leaf,
                                          const LaneRay& r, float& t) {
#ifdef RT_EXP_X16
  const v16i w = sload16(prims + leaf);
  DevPrim p;
  p.v0[0] = __int_as_float(w[0]);
  p.v0[1] = __int_as_float(w[1]);
  p.v0[2] = __int_as_float(w[2]);
  p.a1[0] = __int_as_float(w[3]);
  p.a1[1] = __int_as_float(w[4]);
  p.a1[2] = __int_as_float(w[5]);
  p.a2[0] = __int_as_float(w[6]);
  p.a2[1] = __int_as_float(w[7]);
  p.a2[2] = __int_as_float(w[8]);
  p.kind = w[9];
  p.material = w[10];
  p.cx = __int_as_float(w[11]);
#else
  const DevPrim& p = prims[leaf];
#endif
  const V3 v0 = ld3(p.v0);
  if (!SPHERES || p.kind == kPrimTriangle) return tri_test(v0, ld3(p.a1), ld3(p.a2), p.cx, r, t);
  return sphere_test(v0, p.a1[0], r, t);
}

// ------------------------------------------------------------------ traversal stack
// Wave-uniform (node, R lane-masks) entries — R rays per lane.  DEEP == false: entry i lives
// in VGPR lane i (select-on-lane push / v_readlane pop, no memory traffic, 64 deep).
// DEEP == true: a per-wave LDS array of kDeepStack entries for trees deeper than 64 levels
// (lane 0 writes, all lanes read the broadcast word; LDS ops of one wave complete in order).
constexpr int kDeepStack = 1024;

template <bool DEEP, int R>
struct WaveStack {
  static constexpr int kWords = 1 + 2 * R;
  int node = 0;
  unsigned mlo[R] = {}, mhi[R] = {};
  int sp = 0;  // wave-uniform
  int* lds = nullptr;

  __device__ __forceinline__ void push(int n, const uint64_t (&m)[R]) {
    if (!DEEP) {
      const bool mine = lane_id() == sp;  // v_cmp + v_cndmask: lane sp takes the entry
      node = mine ? n : node;
#pragma unroll
      for (int k = 0; k < R; k++) {
        mlo[k] = mine ? (unsigned)m[k] : mlo[k];
        mhi[k] = mine ? (unsigned)(m[k] >> 32) : mhi[k];
      }
    } else if (lane_id() == 0) {
      lds[kWords * sp] = n;
#pragma unroll
      for (int k = 0; k < R; k++) {
        lds[kWords * sp + 1 + 2 * k] = (int)(unsigned)m[k];
        lds[kWords * sp + 2 + 2 * k] = (int)(unsigned)(m[k] >> 32);
      }
    }
    sp++;
  }
  // The oldest entry (lane 0: the shallowest pending subtree) and its removal, for donation
  // (!DEEP, R == 1 only): entries 1..sp-1 move down one lane.
  __device__ __forceinline__ void bottom(int& n, uint64_t& m) const {
    n = __builtin_amdgcn_readlane(node, 0);
    m = (uint64_t)(unsigned)__builtin_amdgcn_readlane(mlo[0], 0) |
        ((uint64_t)(unsigned)__builtin_amdgcn_readlane(mhi[0], 0) << 32);
  }
  __device__ __forceinline__ void drop_bottom() {
    const int src = (lane_id() + 1) << 2;
    node = __builtin_amdgcn_ds_bpermute(src, node);
    mlo[0] = (unsigned)__builtin_amdgcn_ds_bpermute(src, (int)mlo[0]);
    mhi[0] = (unsigned)__builtin_amdgcn_ds_bpermute(src, (int)mhi[0]);
    sp--;
  }
  __device__ __forceinline__ void pop(int& n, uint64_t (&m)[R]) {
    sp--;
    if (!DEEP) {
      n = __builtin_amdgcn_readlane(node, sp);
#pragma unroll
      for (int k = 0; k < R; k++)
        m[k] = (uint64_t)(unsigned)__builtin_amdgcn_readlane(mlo[k], sp) |
               ((uint64_t)(unsigned)__builtin_amdgcn_readlane(mhi[k], sp) << 32);
    } else {
      n = uniform(lds[kWords * sp]);
#pragma unroll
      for (int k = 0; k < R; k++)
        m[k] = (uint64_t)(unsigned)uniform(lds[kWords * sp + 1 + 2 * k]) |
               ((uint64_t)(unsigned)uniform(lds[kWords * sp + 2 + 2 * k]) << 32);
    }
  }
};

// Distance culling (RT_TRAVERSAL_CULL only): skip a child whose approximate entry distance
// exceeds best_t (1 + 2^-8).  Not proven exact: a triangle whose computed t undershoots its
// true distance by more than the margin (rays within ~1e-5 rad of its plane) could be missed.
__device__ __forceinline__ float cull_limit(float t) { return t + t * 0x1p-8f; }

// Node fetch.  Default: the wave-uniform address makes this a scalar (s_load) fetch.
// RT_EXP_VNODE (experiment): four buffer_load_dwordx4 with the same address on every lane.
__device__ __forceinline__ DevNode load_node(const DevNode* __restrict__ nodes, int node) {
#ifdef RT_EXP_VNODE
  DevNode N;
  typedef float v4f __attribute__((ext_vector_type(4)));
  const v4f* src = reinterpret_cast<const v4f*>(nodes + node);
  const int zero = (int)__builtin_amdgcn_mbcnt_lo(0u, 0u);  // VGPR zero: keep it a vector load
  const v4f q0 = src[0 + zero];
  const v4f q1 = src[1 + zero];
  const v4f q2 = src[2 + zero];
  const v4f q3 = src[3 + zero];
  const float f[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
  for (int a = 0; a < 3; a++)
    for (int c = 0; c < 2; c++) {
      N.lo[a][c] = f[2 * a + c];
      N.hi[a][c] = f[6 + 2 * a + c];
    }
  N.child[0] = uniform(__float_as_int(q3.x));
  N.child[1] = uniform(__float_as_int(q3.y));
  N.axis = 0;
  N.pad = 0;
  return N;
#elif defined(RT_EXP_X16)
#ifdef RT_EXP_DUP  // scalar-cache pressure probe: a second, redundant fetch of the same node
  (void)sload16(nodes + node);
#endif
  const v16i w = sload16(nodes + node);
  DevNode N;
  for (int a = 0; a < 3; a++)
    for (int c = 0; c < 2; c++) {
      N.lo[a][c] = __int_as_float(w[2 * a + c]);
      N.hi[a][c] = __int_as_float(w[6 + 2 * a + c]);
    }
  N.child[0] = w[12];
  N.child[1] = w[13];
  N.axis = w[14];
  N.pad = w[15];
  return N;
#else
  return nodes[node];
#endif
}

// RT_EXP_PREFETCH: at the start of a visit, touch the children's records (node, or the leaf's
// 48-B prim, which may straddle two 64-B lines) so they are in the scalar cache when the next
// visit / the leaf test loads them.  The destination registers are retired after an explicit
// s_waitcnt at the end of the same visit, so no load is in flight when they are reused.
struct ChildPrefetch {
  int a = 0, b = 0, c = 0, d = 0;
  __device__ __forceinline__ void issue(const DevNode* __restrict__ nodes,
                                        const DevPrim* __restrict__ prims, int c0, int c1) {
#ifdef RT_EXP_PREFETCH
    const char* p0 = c0 >= 0 ? (const char*)(nodes + c0) : (const char*)(prims + ~c0);
    const char* p1 = c1 >= 0 ? (const char*)(nodes + c1) : (const char*)(prims + ~c1);
    asm volatile("s_load_dword %0, %1, 0x0" : "=s"(a) : "s"(p0));
    asm volatile("s_load_dword %0, %1, 0x2c" : "=s"(b) : "s"(p0));
    asm volatile("s_load_dword %0, %1, 0x0" : "=s"(c) : "s"(p1));
    asm volatile("s_load_dword %0, %1, 0x2c" : "=s"(d) : "s"(p1));
#endif
  }
  __device__ __forceinline__ void retire() {
#ifdef RT_EXP_PREFETCH
    asm volatile("s_waitcnt lgkmcnt(0)" ::"s"(a), "s"(b), "s"(c), "s"(d) : "memory");
#endif
  }
};

__device__ __forceinline__ bool child_box_exact(const DevNode& N, int c, const LaneRay& r) {
  const float b[6] = {N.lo[0][c], N.lo[1][c], N.lo[2][c], N.hi[0][c], N.hi[1][c], N.hi[2][c]};
  return box_exact(b, r);
}

// Treelet guard that the fast test could not decide: the reference's literal test on the
// guard box and on every enclosing reference box (the ancestry of BVH.cpp:31-55).
__device__ bool guard_exact(const RenderParams& P, int child, const LaneRay& r) {
  int v = child >= 0 ? child : P.anc[~child].leaf_parent;
  while (v >= 0) {
    if (!box_exact(P.anc[v].box, r)) return false;
    v = P.anc[v].parent;
  }
  return true;
}

// One packet visit of a node of either tree, per child:
//   * leaf of a reference node: every lane in the node tests it (leaves have no box; the slot
//     holds a +-1e30 box that every normalised ray accepts, so no special case is needed);
//   * inner child of a reference node: the reference's box test (fast, else box_exact);
//   * guarded child of a culling node (treelet root or lone leaf): the reference's acceptance
//     of its guard box, decided with margin — which implies every enclosing reference box
//     accepts too (accel_build.cpp) — else guard_exact over the whole ancestry;
//   * inner child of a culling node: the conservative cull test.
// h0/h1: lanes that enter (inner) or test (leaf) each child.
template <bool SKIP>
__device__ __forceinline__ void visit_node(const RenderParams& P, const DevNode& N,
                                           const LaneRay& r, bool in, bool& h0, bool& h1,
                                           float& t0, float& t1) {
  const float b0[6] = {N.lo[0][0], N.lo[1][0], N.lo[2][0], N.hi[0][0], N.hi[1][0], N.hi[2][0]};
  const float b1[6] = {N.lo[0][1], N.lo[1][1], N.lo[2][1], N.hi[0][1], N.hi[1][1], N.hi[2][1]};
  float f0, f1;
  slab_span<SKIP>(b0, r, t0, f0);
  slab_span<SKIP>(b1, r, t1, f1);
  bool in0, out0, in1, out1;
  decide_sure(t0, f0, in0, out0);
  decide_sure(t1, f1, in1, out1);
  const int pad = N.pad;  // wave-uniform
  const bool an = (pad & kAccelNode) != 0;
  const bool g0 = (pad & kAccelGuard0) != 0, g1 = (pad & kAccelGuard1) != 0;
  // (a reference node's leaf slot holds a +-1e30 box, scene_build.cpp: every lane accepts it)
  const bool cull0 = an & !g0, cull1 = an & !g1;
  h0 = in & (in0 | (cull0 & !out0));
  h1 = in & (in1 | (cull1 & !out1));
  const bool u0 = in & !cull0 & !(in0 | out0);
  const bool u1 = in & !cull1 & !(in1 | out1);
  if (ballot(u0 | u1)) {
    if (u0) h0 = g0 ? guard_exact(P, N.child[0], r) : child_box_exact(N, 0, r);
    if (u1) h1 = g1 ? guard_exact(P, N.child[1], r) : child_box_exact(N, 1, r);
    DIAG(if (u0 | u1) atomicAdd(&g_exact_fallbacks, 1ull));
  }
}

template <int R>
__device__ __forceinline__ uint64_t any_of(const uint64_t (&m)[R]) {
  uint64_t a = 0;
#pragma unroll
  for (int k = 0; k < R; k++) a |= m[k];
  return a;
}

// Pick the next node: near child first (judged by the first lane of the first ray entering
// both), the far one pushed; with neither, pop (masks restricted to `alive`).  Returns false
// when the traversal is over.
template <bool DEEP, int R>
__device__ __forceinline__ bool advance(WaveStack<DEEP, R>& st, int c0, int c1,
                                        const uint64_t (&m0)[R], const uint64_t (&m1)[R],
                                        const float (&t0)[R], const float (&t1)[R], int& node,
                                        uint64_t (&m)[R], const uint64_t (&alive)[R]) {
  const bool e0 = any_of(m0) != 0, e1 = any_of(m1) != 0;
  if (e0 && e1) {
    int kk = 0;
    uint64_t both = m0[0] & m1[0];
#pragma unroll
    for (int k = 1; k < R; k++)
      if (!both && (m0[k] & m1[k])) {
        both = m0[k] & m1[k];
        kk = k;
      }
    bool near1 = false;
    if (both) {
      const int f = __builtin_ctzll(both);
      float f0 = 0.0f, f1 = 0.0f;
#pragma unroll
      for (int k = 0; k < R; k++)
        if (k == kk) {
          f0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t0[k]), f));
          f1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t1[k]), f));
        }
      near1 = f1 < f0;
    }
    if (near1) {
      st.push(c0, m0);
      node = c1;
#pragma unroll
      for (int k = 0; k < R; k++) m[k] = m1[k];
    } else {
      st.push(c1, m1);
      node = c0;
#pragma unroll
      for (int k = 0; k < R; k++) m[k] = m0[k];
    }
    return true;
  }
  if (e0 || e1) {
    node = e0 ? c0 : c1;
#pragma unroll
    for (int k = 0; k < R; k++) m[k] = e0 ? m0[k] : m1[k];
    return true;
  }
  for (;;) {
    if (st.sp == 0) return false;
    st.pop(node, m);
#pragma unroll
    for (int k = 0; k < R; k++) m[k] &= alive[k];
    if (any_of(m)) return true;
  }
}

// ------------------------------------------------------------------ batched leaf tests
// A packet reaches a leaf with only the few lanes whose rays pass over that triangle (C3:
// ~14 of 64), so testing leaves one at a time runs the triangle test at ~20% SIMD efficiency.
// With R == 1 the traversal instead queues (lane, leaf) pairs in a per-wave LDS list and runs
// them 64 at a time, one pair per lane (the owner's ray fetched with ds_bpermute, the
// triangle with a per-lane load), once 64 are pending and when the walk ends.  Results land
// per ray by LDS atomics: closest hit = atomic min of the key (t bits << 32 | leaf), which for
// 0 < t orders exactly like the reference's (t, DFS leaf) rule; shadow = atomic or.  The
// queued tests are the ones the reference makes, so the answer is unchanged; only FAST
// culling sees best_t a little later (after each flush), which can only cull less.
// RT_EXP_NOBATCH: leaves tested where they are met (the R > 1 path always does).
#ifndef RT_BATCH_FLUSH
#define RT_BATCH_FLUSH 64
#endif
constexpr int kBatchFlush = RT_BATCH_FLUSH;  // run the queue once this many tests are pending
constexpr int kBatchCap = kBatchFlush + 256;  // < kBatchFlush pending + 2 pairs x 64 per visit
#ifndef RT_SHADOW_FLUSH  // shadow rays: a smaller queue finds occluders (and stops lanes) sooner
#define RT_SHADOW_FLUSH RT_BATCH_FLUSH
#endif
constexpr int kShadowFlush = RT_SHADOW_FLUSH;
static_assert(kShadowFlush <= kBatchFlush, "the queue is sized for kBatchFlush");
#ifndef RT_TRACE_WAVES
#define RT_TRACE_WAVES 4
#endif

struct WaveLeafLds {
  unsigned long long q[kBatchCap];  // lo 32: leaf index, hi 32: lane
  unsigned long long key[64];       // per lane: closest-hit key, or shadow flag
};


#if defined(RT_EXP_NOBATCH)
constexpr bool kBatchLeaves = false;
#else
constexpr bool kBatchLeaves = true;
#endif

constexpr unsigned long long kNoHitKey = (0x7f800000ull << 32) | 0xffffffffull;  // (+inf, -1)

// Queue leaf `leaf` for the lanes of `m` (wave-uniform); n = pending entries (wave-uniform).
__device__ __forceinline__ void batch_push(WaveLeafLds& L, int& n, int leaf, uint64_t m) {
  const int lane = lane_id();
  if ((m >> lane) & 1) {
    const int below = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
    L.q[n + below] = ((unsigned long long)lane << 32) | (unsigned)leaf;
  }
  n += __builtin_popcountll(m);
}

__device__ __forceinline__ float lane_f(int src, float v) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(v)));
}

// Runs the n queued tests; SHADOW: 0 < t < thr of the owner sets its flag, else the owner's
// key takes min(key, (t, leaf)) for 0 < t < inf.  All lanes of the wave take part.
template <bool SHADOW, bool SPHERES>
__device__ __forceinline__ void batch_flush(WaveLeafLds& L, int n, const DevPrim* __restrict__ prims,
                                            const LaneRay& r, float thr) {
  const int lane = lane_id();
  for (int base = 0; base < n; base += 64) {
    const int i = base + lane;
    const bool valid = i < n;
    const unsigned long long e = valid ? L.q[i] : 0ull;
    const int src = (int)(e >> 32), leaf = (int)(unsigned)e;
    LaneRay rr;
    rr.o = v3(lane_f(src, r.o.x), lane_f(src, r.o.y), lane_f(src, r.o.z));
    rr.d = v3(lane_f(src, r.d.x), lane_f(src, r.d.y), lane_f(src, r.d.z));
    rr.quot = __builtin_amdgcn_ds_bpermute(src << 2, (int)r.quot) != 0;
    const float othr = SHADOW ? lane_f(src, thr) : 0.0f;
    float t = 0.0f;
    const bool hit = leaf_test<SPHERES>(prims, leaf, rr, t);  // leaf 0 for idle lanes: unused
    if (SHADOW) {
      if (valid & hit & (t > 0.0f) & (t < othr)) L.key[src] = 1ull;  // any writer: same value
    } else if (valid & hit & (t > 0.0f) & (t < RT_INF)) {
      atomicMin(&L.key[src], ((unsigned long long)__float_as_uint(t) << 32) | (unsigned)leaf);
    }
  }
}

// ------------------------------------------------------------------ wide culling nodes
// Kernels with the batched leaf queue and one ray per lane walk the 4-wide culling tree
// (accel_build.cpp collapse_wide); others get the binary one.
bool wide_nodes_supported() { return kBatchLeaves && kRaysPerLane == 1; }

// The whole 128-B node in one round trip: two s_load_dwordx16 and one wait.  Left to itself
// the compiler splits the record into ~14 loads of 1-8 dwords in three dependent rounds (and,
// short of SGPRs, reloads the first slot's box after the flags test).  RT_WIDE_SLOAD=0 for A/B.
#ifndef RT_WIDE_SLOAD
#define RT_WIDE_SLOAD 1
#endif
#ifndef RT_WIDE_PK  // slab spans of a wide node's slots two at a time (packed fp32)
#define RT_WIDE_PK 0
#endif
__device__ __forceinline__ DevNode4 load_node4(const DevNode* __restrict__ nodes, int idx) {
#if RT_WIDE_SLOAD
  v16i a, b;
  const void* p = nodes + idx;
  asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx16 %1, %2, 0x40\n\ts_waitcnt lgkmcnt(0)"
               : "=s"(a), "=s"(b) : "s"(p) : "memory");
  DevNode4 N;
#pragma unroll
  for (int k = 0; k < 4; k++) {
#pragma unroll
    for (int x = 0; x < 3; x++) {
      N.lo[x][k] = __int_as_float(a[4 * x + k]);
      N.hi[x][k] = __int_as_float(k + 4 * x < 4 ? a[12 + 4 * x + k] : b[4 * x + k - 4]);
    }
    N.child[k] = b[8 + k];
  }
  N.flags = b[12];
  return N;
#else
  return *reinterpret_cast<const DevNode4*>(nodes + idx);
#endif
}

// One packet visit of a wide culling node (R == 1, batched leaves), slot by slot with the
// binary tree's rules (visit_node): a guarded slot accepts on a decided guard test (else
// guard_exact), and its leaf or leaf pair goes straight to the leaf queue; an inner slot
// culls only on a sure reject.  Of the entered inner slots one becomes `node` (SHADOW: the
// nearest by the entry distance of the first entering lane, so occluders turn up early) and
// the others are pushed.  `alive`: lanes still searching.  Up to 4 slots x 2 leaves x 64 lanes
// of leaf tests are queued per visit, so the queue is run in between when it could overflow.
// Returns false when the walk is over.
template <bool SKIP, bool SHADOW, bool DEEP, bool SPHERES>
__device__ __forceinline__ bool visit_wide(const RenderParams& P, const DevNode* __restrict__ nodes,
                                           const DevPrim* __restrict__ prims, WaveLeafLds& L,
                                           int& pending, const LaneRay& r, float thr, int& node,
                                           uint64_t& m, uint64_t alive, WaveStack<DEEP, 1>& st,
                                           Diag& dg) {
  const DevNode4 N = load_node4(nodes, node & ~kWideTag);
  const bool in = (m >> lane_id()) & 1;
  const int fl = N.flags;
  DIAG(dg.nodes++; dg.wide++; dg.node_lanes += __builtin_popcountll(m));
  int nxt = -1;
  uint64_t nm = 0;
  float nkey = 0.0f;
#if RT_WIDE_PK
  float tn4[4], tf4[4];  // all four spans up front, two slots per packed instruction
  slab_span2<SKIP>(N.lo, N.hi, 0, r, tn4, tf4);
  slab_span2<SKIP>(N.lo, N.hi, 2, r, tn4 + 2, tf4 + 2);
#endif
#pragma unroll
  for (int c = 0; c < 4; c++) {
    if (!(fl & (kWideValid << c))) continue;
#if RT_WIDE_PK
    const float tn = tn4[c], tf = tf4[c];
#else
    const float b[6] = {N.lo[0][c], N.lo[1][c], N.lo[2][c], N.hi[0][c], N.hi[1][c], N.hi[2][c]};
    float tn, tf;
    slab_span<SKIP>(b, r, tn, tf);
#endif
    bool sin, sout;
    decide_sure(tn, tf, sin, sout);
    const int ch = N.child[c];
    const bool guard = (fl & (kWideGuard << c)) != 0;
    bool h;
    if (guard) {
      h = in & sin;
      const bool u = in & !(sin | sout);
      if (ballot(u)) {
        if (u) h = guard_exact(P, ch, r);
        DIAG(if (u) atomicAdd(&g_exact_fallbacks, 1ull));
      }
    } else {
      h = in & !sout;
    }
    const uint64_t hm = ballot(h) & alive;
    if (!hm) continue;
    if (guard && ch < 0) {  // a leaf, or a leaf pair
      const bool pair = (fl & (kWidePair << c)) != 0;
      if (pending > kBatchCap - 128) {
        batch_flush<SHADOW, SPHERES>(L, pending, prims, r, thr);
        pending = 0;
      }
      batch_push(L, pending, ~ch, hm);
      if (pair) batch_push(L, pending, ~ch + 1, hm);
      DIAG(dg.leaves += 1 + pair; dg.leaf_lanes += (1 + pair) * __builtin_popcountll(hm));
      continue;
    }
    uint64_t mm[1] = {hm};
    if (SHADOW) {
      const float key = __int_as_float(
          __builtin_amdgcn_readlane(__float_as_int(tn), (int)__builtin_ctzll(hm)));
      if (nxt < 0 || key < nkey) {
        if (nxt >= 0) {
          uint64_t pm[1] = {nm};
          st.push(nxt, pm);
        }
        nxt = ch;
        nm = hm;
        nkey = key;
      } else {
        st.push(ch, mm);
      }
    } else if (nxt < 0) {
      nxt = ch;
      nm = hm;
    } else {
      st.push(ch, mm);
    }
  }
  if (nxt >= 0) {
    node = nxt;
    m = nm;
    return true;
  }
  for (;;) {
    if (st.sp == 0) return false;
    uint64_t mm[1];
    st.pop(node, mm);
    m = mm[0] & alive;
    if (m) return true;
  }
}

// ------------------------------------------------------------------ subtree sharing
// A workgroup's packets cost unequal amounts (tools/timeline.py: C3 primary packets take 60 to
// 265 us), and a workgroup keeps its slot until its last wave ends, so waves that finish early
// idle while a heavy packet runs: the C3 primary kernel held ~90 % of its wave slots in the bulk
// of the frame and spent its last 40 % draining.  With sharing, the waves of a workgroup split
// their packets' traversals between them through LDS.  A wave without work raises its bit in
// `want` and waits at its inbox; a traversing wave that sees a raised bit (checked every 4th
// visit) claims that wave (atomic and of the bit) and hands it its OLDEST stack entry — the
// shallowest pending subtree — as (owner packet, light, node, lane mask).  The helper rebuilds
// the owner packet's rays bit for bit and traverses that subtree exactly as the owner would.
// Each piece's answer merges into the owner's per-lane result in LDS — closest hit by 64-bit
// min of the (t bits, DFS leaf) key (the reference's rule, §4.1), shadow by or — and after a
// workgroup barrier every wave writes its own packet.  A claimed wave's bit stays clear until
// it is idle again, so `want` == all waves means nobody traverses and nobody can hand out work:
// every wave then leaves.  Workgroup-local and lock-free: LDS atomics only (a lock taken and
// released in a polling loop measured as a livelock on gfx950).
struct ShareEntry {
  unsigned long long mask;
  int node, owner, light, pad;
};

template <int W>
struct BlockShare {
  int want;     // bit i: wave i waits for work
  int flag[W];  // inbox i is full
  int sel[W];   // each wave's own packet (tile), -1 for none
  ShareEntry box[W];
  unsigned long long res[W][64];  // per packet and lane: primary key / shadow light bits
};

__device__ __forceinline__ int lds_load(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

struct NoDonor {
  static constexpr bool kOn = false;
  __device__ __forceinline__ bool tick() { return false; }
  __device__ __forceinline__ bool donate(int, uint64_t) { return false; }
};

// The donation policy of one traversal piece in a sharing workgroup.
template <int W>
struct Sharer {
  static constexpr bool kOn = true;
  BlockShare<W>* S;
  int owner, light, visits;  // wave-uniform
  __device__ __forceinline__ bool tick() {
#ifdef RT_EXP_NODONATE
    return false;
#else
    return (++visits & 3) == 0 && lds_load(&S->want) != 0;
#endif
  }
  __device__ __forceinline__ bool donate(int node, uint64_t mask) {
    int ok = 0;
    if (lane_id() == 0) {
      int m = lds_load(&S->want);
      while (m) {
        const int i = __builtin_ctz((unsigned)m), bit = 1 << i;
        const int old = atomicAnd(&S->want, ~bit);
        if (old & bit) {  // wave i is ours
          S->box[i].mask = mask;
          S->box[i].node = node;
          S->box[i].owner = owner;
          S->box[i].light = light;
          __hip_atomic_store(&S->flag[i], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          ok = 1;
          break;
        }
        m = old & ~bit;
      }
    }
    return uniform(ok) != 0;
  }
};

// Called by a wave whose current piece is done: raises its want bit and waits for an entry.
// False once every wave of the workgroup wants work (no one is left to hand any out).
template <int W>
__device__ __forceinline__ bool share_next(BlockShare<W>& S, int& owner, int& node, uint64_t& mask,
                                           int& light) {
  const int wv = (int)threadIdx.x >> 6;
  int got = 0, o = 0, n = 0, l = 0;
  unsigned lo = 0, hi = 0;
  if (lane_id() == 0) {
    atomicOr(&S.want, 1 << wv);
    for (;;) {
      if (__hip_atomic_load(&S.flag[wv], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) {
        const ShareEntry& e = S.box[wv];
        lo = (unsigned)e.mask;
        hi = (unsigned)(e.mask >> 32);
        n = e.node;
        o = e.owner;
        l = e.light;
        __hip_atomic_store(&S.flag[wv], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        got = 1;
        break;
      }
      if (lds_load(&S.want) == (1 << W) - 1) break;
      __builtin_amdgcn_s_sleep(2);
    }
  }
  if (!uniform(got)) return false;
  owner = uniform(o);
  node = uniform(n);
  light = uniform(l);
  mask = (uint64_t)(unsigned)uniform((int)lo) | ((uint64_t)(unsigned)uniform((int)hi) << 32);
  return true;
}

// ------------------------------------------------------------------ closest hit
// R rays per lane.  Returns the reference's (t, leaf) for every active ray: leaf < 0 = miss.
// DN: the donation policy (NoDonor, or Sharer in sharing workgroups, R == 1 and !DEEP only);
// start_node >= 0: traverse the shared subtree (start_node, start_mask) instead of the tree.
template <bool SKIP, bool FAST, bool DEEP, bool SPHERES, int R, bool CULL = false,
          class DN = NoDonor, bool WO = false>
__device__ __forceinline__ void closest_hit(const RenderParams& P,
                                            const DevNode* __restrict__ nodes,
                                            const DevPrim* __restrict__ prims, int* spill, WaveLeafLds& L,
                                            const LaneRay (&r)[R], const bool (&active)[R],
                                            float (&best_t)[R], int (&best_leaf)[R], Diag& dg,
                                            DN& dn, int start_node = -1,
                                            uint64_t start_mask = 0) {
  static_assert(!DN::kOn || (R == 1 && !DEEP), "donation needs the one-ray-per-lane lane stack");
#pragma unroll
  for (int k = 0; k < R; k++) {
    best_t[k] = RT_INF;
    best_leaf[k] = -1;
  }
  if (P.root_kind != kRootNode) {  // the root IS the primitive (BVH.h:13-14): its own rule
#pragma unroll
    for (int k = 0; k < R; k++) {
      float t;
      if (active[k] && leaf_test<SPHERES>(prims, P.root_ref, r[k], t)) {
        best_t[k] = t;
        best_leaf[k] = P.root_ref;
      }
    }
    return;
  }
  const bool accel = FAST && P.accel_root >= 0;  // culling tree over treelets (§4.4)
  const bool task = DN::kOn && start_node >= 0;
  uint64_t m[R];
  if (task) {
    m[0] = start_mask & ballot(active[0]);
  } else {
#pragma unroll
    for (int k = 0; k < R; k++) {
      float tn, tf;
      bool acc, und;
      if (accel) {
        slab_span<SKIP>(P.accel_box, r[k], tn, tf);
        m[k] = ballot(active[k] && decide_cull(tn, tf));
      } else {
        slab_fast<SKIP>(P.root_box, r[k], tn, acc, und);
        m[k] = ballot(active[k] && (acc || (und && box_exact(P.root_box, r[k]))));
      }
    }
  }
  if (!any_of(m)) return;
  const int lane = lane_id();
  WaveStack<DEEP, R> st;
  st.lds = spill;
  uint64_t everyone[R];
#pragma unroll
  for (int k = 0; k < R; k++) everyone[k] = ~0ull;
  constexpr bool batch = kBatchLeaves && R == 1;
  int pending = 0;
  if (batch) L.key[lane] = kNoHitKey;
  int node = task ? start_node : (accel ? P.accel_root : P.root_ref);
  for (;;) {
    if constexpr (batch) {  // between visits: only the ray, the stack and best_t are live
      if (pending >= kBatchFlush) {
        batch_flush<false, SPHERES>(L, pending, prims, r[0], 0.0f);
        pending = 0;
        const unsigned long long key = L.key[lane];
        best_t[0] = __uint_as_float((unsigned)(key >> 32));
        best_leaf[0] = (int)(unsigned)key;
      }
    }
    if constexpr (DN::kOn) {  // hand the oldest pending subtree to the work queue
      if (dn.tick() && st.sp > 0) {
        int n0;
        uint64_t m0;
        st.bottom(n0, m0);
        if (dn.donate(n0, m0)) st.drop_bottom();
      }
    }
    if constexpr (batch && FAST) {  // a wide culling node (WO: every node the walk meets is one)
      if (WO || (node & kWideTag)) {
        uint64_t mm = m[0];
        const bool more = visit_wide<SKIP, false, DEEP, SPHERES>(P, nodes, prims, L, pending, r[0],
                                                                0.0f, node, mm, ~0ull, st, dg);
        m[0] = mm;
        if (!more) break;
        continue;
      }
    }
    const DevNode N = load_node(nodes, node);
    ChildPrefetch pf;
    pf.issue(nodes, prims, N.child[0], N.child[1]);
    bool h0[R], h1[R];
    float t0[R], t1[R];
#pragma unroll
    for (int k = 0; k < R; k++)
      visit_node<SKIP>(P, N, r[k], (m[k] >> lane) & 1, h0[k], h1[k], t0[k], t1[k]);
    DIAG(dg.nodes++; dg.node_lanes += __builtin_popcountll(any_of(m));
         const int nl0 = N.child[0] < 0 ? 1 + ((N.pad & kAccelPair0) != 0) : 0;
         const int nl1 = N.child[1] < 0 ? 1 + ((N.pad & kAccelPair1) != 0) : 0;
         dg.leaves += nl0 + nl1;
         dg.leaf_lanes += nl0 * __builtin_popcountll(ballot(h0[0])) +
                          nl1 * __builtin_popcountll(ballot(h1[0])));
    if constexpr (batch) {  // queue the leaf children's tests; run them 64 at a time
      if (N.child[0] < 0) {
        const uint64_t b = ballot(h0[0]);
        batch_push(L, pending, ~N.child[0], b);
        if (N.pad & kAccelPair0) batch_push(L, pending, ~N.child[0] + 1, b);
      }
      if (N.child[1] < 0) {
        const uint64_t b = ballot(h1[0]);
        batch_push(L, pending, ~N.child[1], b);
        if (N.pad & kAccelPair1) batch_push(L, pending, ~N.child[1] + 1, b);
      }
    } else {
#ifndef RT_EXP_NOLEAF
#pragma unroll 1
    for (int slot = 0; slot < 4; slot++) {  // leaf children: Shape::intersect, 0 < t < best
      const int side = slot >> 1;             // (slot & 1: the second leaf of a leaf pair)
      const int c = side ? N.child[1] : N.child[0];
      if (c < 0 && (!(slot & 1) || (N.pad & (side ? kAccelPair1 : kAccelPair0)))) {
        const int leaf = ~c + (slot & 1);
#pragma unroll
        for (int k = 0; k < R; k++) {
          const bool tests = side ? h1[k] : h0[k];
          float t = 0.0f;
#ifndef RT_EXP_BRANCHY  // (RT_EXP_BRANCHY: the early-exit form, for A/B)
          if (ballot(tests)) {  // one wave-uniform branch; the update itself is a select
            const bool hit = leaf_test<SPHERES>(prims, leaf, r[k], t);
            const bool take = tests & hit & (t > 0.0f) & (t < RT_INF) &
                              ((t < best_t[k]) | ((t == best_t[k]) & (leaf < best_leaf[k])));
            best_t[k] = take ? t : best_t[k];
            best_leaf[k] = take ? leaf : best_leaf[k];
          }
#else
          if (tests && leaf_test<SPHERES>(prims, leaf, r[k], t) && t > 0.0f && t < RT_INF &&
              (t < best_t[k] || (t == best_t[k] && leaf < best_leaf[k]))) {
            best_t[k] = t;
            best_leaf[k] = leaf;
          }
#endif
        }
      }
    }
#else
#pragma unroll
    for (int k = 0; k < R; k++) best_leaf[k] -= (int)((m[k] >> lane) & 1);  // keep it observable
#endif
    }
    uint64_t m0[R], m1[R];
#pragma unroll
    for (int k = 0; k < R; k++) {  // leaves are done; only inner children are entered
      h0[k] &= N.child[0] >= 0;
      h1[k] &= N.child[1] >= 0;
      if (FAST && CULL) {
        const float lim = cull_limit(best_t[k]);
        h0[k] = h0[k] && t0[k] <= lim;
        h1[k] = h1[k] && t1[k] <= lim;
      }
      m0[k] = ballot(h0[k]);
      m1[k] = ballot(h1[k]);
    }
    pf.retire();
    if (!advance(st, N.child[0], N.child[1], m0, m1, t0, t1, node, m, everyone)) break;
  }
  if constexpr (batch) {
    if (pending) batch_flush<false, SPHERES>(L, pending, prims, r[0], 0.0f);
    const unsigned long long key = L.key[lane];
    best_t[0] = __uint_as_float((unsigned)(key >> 32));
    best_leaf[0] = (int)(unsigned)key;
  }
}

// ------------------------------------------------------------------ shadow (any hit)
// Occluded iff some leaf the ray may reach has 0 < t < thr — identical to the reference's
// closest-hit shadow test `0 < t_closest < dist - eps` (HW2/Scene.cpp:123-127), appendix A.7.
template <bool SKIP, bool FAST, bool DEEP, bool SPHERES, int R, bool CULL = false,
          class DN = NoDonor, bool WO = false>
__device__ __forceinline__ void occluded(const RenderParams& P, const DevNode* __restrict__ nodes,
                                         const DevPrim* __restrict__ prims, int* spill, WaveLeafLds& L,
                                         const LaneRay (&r)[R], const bool (&active)[R],
                                         const float (&thr)[R], bool (&occ)[R], Diag& dg,
                                         DN& dn, int start_node = -1, uint64_t start_mask = 0) {
  static_assert(!DN::kOn || (R == 1 && !DEEP), "donation needs the one-ray-per-lane lane stack");
#pragma unroll
  for (int k = 0; k < R; k++) occ[k] = false;
  if (P.root_kind != kRootNode) {
#pragma unroll
    for (int k = 0; k < R; k++) {
      float t;
      occ[k] = active[k] && leaf_test<SPHERES>(prims, P.root_ref, r[k], t) && t < thr[k] &&
               t > 0.0f;
    }
    return;
  }
  const bool accel = FAST && P.accel_root >= 0;
  const bool task = DN::kOn && start_node >= 0;
  uint64_t m[R], alive[R];
  if (task) {
    m[0] = alive[0] = start_mask & ballot(active[0] && thr[0] > 0.0f);
  } else {
#pragma unroll
    for (int k = 0; k < R; k++) {
      float tn, tf;
      bool acc, und;
      // thr <= 0 (or NaN): nothing can satisfy 0 < t < thr
      if (accel) {
        slab_span<SKIP>(P.accel_box, r[k], tn, tf);
        m[k] = ballot(active[k] && thr[k] > 0.0f && decide_cull(tn, tf));
      } else {
        slab_fast<SKIP>(P.root_box, r[k], tn, acc, und);
        m[k] = ballot(active[k] && thr[k] > 0.0f &&
                      (acc || (und && box_exact(P.root_box, r[k]))));
      }
      alive[k] = m[k];
    }
  }
  if (!any_of(m)) return;
  const int lane = lane_id();
  WaveStack<DEEP, R> st;
  st.lds = spill;
  constexpr bool batch = kBatchLeaves && R == 1;
  int pending = 0;
  if (batch) L.key[lane] = 0ull;
  int node = task ? start_node : (accel ? P.accel_root : P.root_ref);
  for (;;) {
    if constexpr (batch) {  // between visits; a lane found occluded stops entering nodes
      if (pending >= kShadowFlush) {
        batch_flush<true, SPHERES>(L, pending, prims, r[0], thr[0]);
        pending = 0;
        occ[0] = L.key[lane] != 0ull;
        alive[0] &= ~ballot(occ[0]);
        m[0] &= alive[0];
        if (!m[0] && !advance(st, 0, 0, m, m, thr, thr, node, m, alive)) break;
      }
    }
    if constexpr (DN::kOn) {  // hand the oldest pending subtree (still-unoccluded lanes) over
      if (dn.tick() && st.sp > 0) {
        int n0;
        uint64_t m0;
        st.bottom(n0, m0);
        m0 &= alive[0];
        if (!m0 || dn.donate(n0, m0)) st.drop_bottom();
      }
    }
    if constexpr (batch && FAST) {  // a wide culling node (WO: every node the walk meets is one)
      if (WO || (node & kWideTag)) {
        uint64_t mm = m[0];
        const bool more = visit_wide<SKIP, true, DEEP, SPHERES>(P, nodes, prims, L, pending, r[0],
                                                               thr[0], node, mm, alive[0], st, dg);
        m[0] = mm;
        if (!more) break;
        continue;
      }
    }
    const DevNode N = load_node(nodes, node);
    ChildPrefetch pf;
    pf.issue(nodes, prims, N.child[0], N.child[1]);
    bool h0[R], h1[R];
    float t0[R], t1[R];
#pragma unroll
    for (int k = 0; k < R; k++)
      visit_node<SKIP>(P, N, r[k], (m[k] >> lane) & 1, h0[k], h1[k], t0[k], t1[k]);
    DIAG(dg.nodes++; dg.node_lanes += __builtin_popcountll(any_of(m));
         const int nl0 = N.child[0] < 0 ? 1 + ((N.pad & kAccelPair0) != 0) : 0;
         const int nl1 = N.child[1] < 0 ? 1 + ((N.pad & kAccelPair1) != 0) : 0;
         dg.leaves += nl0 + nl1;
         dg.leaf_lanes += nl0 * __builtin_popcountll(ballot(h0[0])) +
                          nl1 * __builtin_popcountll(ballot(h1[0])));
    if constexpr (batch) {  // queue the still-unoccluded lanes' leaf tests
      if (N.child[0] < 0) {
        const uint64_t b = ballot(h0[0]) & alive[0];
        batch_push(L, pending, ~N.child[0], b);
        if (N.pad & kAccelPair0) batch_push(L, pending, ~N.child[0] + 1, b);
      }
      if (N.child[1] < 0) {
        const uint64_t b = ballot(h1[0]) & alive[0];
        batch_push(L, pending, ~N.child[1], b);
        if (N.pad & kAccelPair1) batch_push(L, pending, ~N.child[1] + 1, b);
      }
    } else {
#pragma unroll 1
    for (int slot = 0; slot < 4; slot++) {  // (slot & 1: the second leaf of a leaf pair)
      const int side = slot >> 1;
      const int c = side ? N.child[1] : N.child[0];
      if (c < 0 && (!(slot & 1) || (N.pad & (side ? kAccelPair1 : kAccelPair0)))) {
        const int leaf = ~c + (slot & 1);
#pragma unroll
        for (int k = 0; k < R; k++) {
          const bool tests = side ? h1[k] : h0[k];
          float t = 0.0f;
#ifndef RT_EXP_BRANCHY  // (RT_EXP_BRANCHY: the early-exit form, for A/B)
          const bool want = tests & !occ[k];
          if (ballot(want)) {
            const bool hit = leaf_test<SPHERES>(prims, leaf, r[k], t);
            occ[k] = occ[k] | (want & hit & (t > 0.0f) & (t < thr[k]));
          }
#else
          if (tests && !occ[k] && leaf_test<SPHERES>(prims, leaf, r[k], t) && t > 0.0f &&
              t < thr[k])
            occ[k] = true;
#endif
        }
      }
    }
    }
    uint64_t m0[R], m1[R];
#pragma unroll
    for (int k = 0; k < R; k++) {
      alive[k] &= ~ballot(occ[k]);
      h0[k] &= N.child[0] >= 0;
      h1[k] &= N.child[1] >= 0;
      if (FAST && CULL) {
        const float lim = cull_limit(thr[k]);
        h0[k] = h0[k] && t0[k] <= lim;
        h1[k] = h1[k] && t1[k] <= lim;
      }
      m0[k] = ballot(h0[k]) & alive[k];
      m1[k] = ballot(h1[k]) & alive[k];
    }
    pf.retire();
    if (!any_of(alive)) break;
    if (!advance(st, N.child[0], N.child[1], m0, m1, t0, t1, node, m, alive)) break;
  }
  if constexpr (batch) {
    if (pending) batch_flush<true, SPHERES>(L, pending, prims, r[0], thr[0]);
    occ[0] = L.key[lane] != 0ull;
  }
}

// The kernel's RenderParams (its FIRST argument, so at offset 0 of the kernarg segment) read
// through a pointer the compiler cannot see through: loads from it are not hoisted above this
// point, so the persistent packet loop does not pull every field it uses into SGPRs for the
// whole kernel (they were spilled to VGPR lanes across the traversal and reloaded per visit).
typedef __attribute__((address_space(4))) const RenderParams KernargParams;
__device__ __forceinline__ const RenderParams& fresh_params(const RenderParams& P) {
#ifdef RT_EXP_NOLAUNDER
  return P;
#else
  KernargParams* p = (KernargParams*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return *(const RenderParams*)p;
#endif
}

// ------------------------------------------------------------------ render kernels
// Two launches per frame (wavefront style): `trace_primary` finds each pixel's closest hit and
// writes an 8-byte {t, leaf} record; `shade` rebuilds the shading inputs from it and runs the
// point-light loop with its shadow rays.  Splitting keeps each kernel's live state small
// (occupancy is what hides the dependent node loads), at 16 B of HBM traffic per pixel.
struct PacketPixel {
  int lane, px, py;
  bool valid;
};

__device__ __forceinline__ PacketPixel packet_pixel(const RenderParams& P, int sel) {
  PacketPixel q;
  q.lane = lane_id();
  const int tile = P.tile_begin + sel * P.tile_step;
  const int tx = tile % P.tiles_x, ty = tile / P.tiles_x;
  q.px = tx * kTile + (q.lane & 7);
  const int lr = ty * kTile + (q.lane >> 3);  // logical row
  q.valid = q.px < P.width && lr < P.rows;
  q.py = P.row0 + lr * P.row_stride;
  return q;
}

// ------------------------------------------------------------------ MSAA sample positions
// HW2/Scene.cpp:35-44: a std::default_random_engine (libstdc++ minstd_rand0, x <- 16807 x mod
// 2^31-1) per pixel, seeded here with splitmix64(seed, pixel) instead of the wall clock, and
// uniform_real_distribution<float>(0, 1) = generate_canonical<float, 24>: one draw u,
// float(u - 1) / 2^31, clamped below 1.  Sample s = x*n + y uses draws 2s+1 and 2s+2.
__device__ __forceinline__ unsigned long long msaa_pixel_seed(unsigned long long base,
                                                              unsigned long long pixel) {
  unsigned long long z = base + 0x9E3779B97F4A7C15ull * (pixel + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ unsigned minstd_state0(unsigned long long seed) {
  const unsigned x = (unsigned)(seed % kMinstdM);
  return x == 0 ? 1u : x;
}

__device__ __forceinline__ unsigned minstd_mulmod(unsigned a, unsigned b) {
  unsigned long long p = (unsigned long long)a * b;  // < 2^62; 2^31 = 1 (mod 2^31-1)
  p = (p & kMinstdM) + (p >> 31);
  p = (p & kMinstdM) + (p >> 31);
  return (unsigned)(p >= kMinstdM ? p - kMinstdM : p);
}

__device__ __forceinline__ float minstd_uniform01(unsigned u) {
  float r = (float)(u - 1u) / 2147483648.0f;  // exact: power-of-two divisor
  return r >= 1.0f ? __uint_as_float(0x3f7fffffu) : r;
}

// sample_x, sample_y of HW2/Scene.cpp:43-44 for sample index s of pixel (px, py)
__device__ __forceinline__ void msaa_offsets(const RenderParams& P, int px, int py, float& sx,
                                             float& sy) {
  const unsigned u0 = minstd_state0(
      msaa_pixel_seed(P.msaa_seed, (unsigned long long)py * (unsigned)P.width + (unsigned)px));
  const float n = (float)P.msaa_n;
  sx = ((float)(P.msaa_s / P.msaa_n) + minstd_uniform01(minstd_mulmod(u0, P.msaa_mul[0]))) / n;
  sy = ((float)(P.msaa_s % P.msaa_n) + minstd_uniform01(minstd_mulmod(u0, P.msaa_mul[1]))) / n;
}

// Camera::calculate_ray_at (HW2/Camera.h:30-35); x + 0.5 is exact in fp32 for x < 2^23.
// MSAA passes x = i + sample_x - 0.5 (a double narrowed to the float parameter) and the
// camera widens it again for x + 0.5 before the float multiply.
__device__ __forceinline__ V3 primary_dir(const RenderParams& P, int px, int py) {
  float fx = (float)px + 0.5f, fy = (float)py + 0.5f;
  if (P.msaa_n) {
    float sx, sy;
    msaa_offsets(P, px, py, sx, sy);
    fx = (float)((double)(float)((double)((float)px + sx) - 0.5) + 0.5);
    fy = (float)((double)(float)((double)((float)py + sy) - 0.5) + 0.5);
  }
  const V3 s = (ld3(P.cam_tl) + ld3(P.cam_su) * fx) - ld3(P.cam_sv) * fy;
  return normalize(s - ld3(P.cam_e));
}

__device__ __forceinline__ unsigned long long* counter_row(const RenderParams& P, int sel) {
  return P.counters + kCounterWidth * (sel % kCounterSlots);
}

__device__ __forceinline__ unsigned long long hit_key(int2_t rec) {
  return ((unsigned long long)(unsigned)rec.y << 32) | (unsigned)rec.x;
}
__device__ __forceinline__ float hit_t(int2_t rec) { return __int_as_float(rec.y); }
__device__ __forceinline__ int hit_leaf(int2_t rec) { return rec.x; }

// R selected tiles per wave (tile sel0 + k is ray k of every lane): one packet traversal
// serves 64*R rays, so the per-visit overhead (node fetch, masks, stack) is shared.
template <bool FAST, bool DEEP, bool SPHERES, int R, bool CULL, bool WO = false>
__device__ __forceinline__ void primary_packet(const RenderParams& P,
                                               const DevNode* __restrict__ nodes,
                                               const DevPrim* __restrict__ prims, int sel0,
                                               int* spill, WaveLeafLds& L) {
  PacketPixel q[R];
  LaneRay ray[R];
  bool valid[R];
  bool any_skip = false;
#pragma unroll
  for (int k = 0; k < R; k++) {
    q[k] = packet_pixel(P, sel0 + k);
    valid[k] = q[k].valid && sel0 + k < P.num_sel_tiles;
    ray[k] = make_ray(ld3(P.cam_e), primary_dir(P, q[k].px, q[k].py), P.quot_ok);
#ifndef RT_EXP_UNIFORM_ORIGIN
    // The camera origin is wave-uniform; left to itself the compiler keeps it in 3 SGPRs and
    // copies it to VGPRs at every node visit (a VALU op takes one SGPR operand, the box
    // coordinate already is one).  Pin it to VGPRs once.
    asm volatile("" : "+v"(ray[k].o.x), "+v"(ray[k].o.y), "+v"(ray[k].o.z));
#endif
    any_skip |= valid[k] && (ray[k].skip0 || ray[k].skip1 || ray[k].skip2);
  }
  Diag dg;
  float t[R];
  int leaf[R];
  NoDonor nd;
  if (ballot(any_skip))
    closest_hit<true, FAST, DEEP, SPHERES, R, CULL, NoDonor, WO>(P, nodes, prims, spill, L, ray, valid, t, leaf,
                                                    dg, nd);
  else
    closest_hit<false, FAST, DEEP, SPHERES, R, CULL, NoDonor, WO>(P, nodes, prims, spill, L, ray, valid, t, leaf,
                                                     dg, nd);
  const RenderParams& Pw = fresh_params(P);  // post-traversal fields: not live across it
  unsigned long long nvalid = 0, nhit = 0;
#pragma unroll
  for (int k = 0; k < R; k++) {
    if (sel0 + k < Pw.num_sel_tiles) {
      int2_t rec;  // key layout: leaf low, t bits high (rt_internal.h)
      rec.x = valid[k] ? leaf[k] : -2;  // -1 miss, -2 outside the image
      rec.y = __float_as_int(t[k]);
      Pw.hits[(size_t)(sel0 + k) * (kTile * kTile) + q[k].lane] = rec;
    }
    nvalid += __builtin_popcountll(ballot(valid[k]));
    nhit += __builtin_popcountll(ballot(valid[k] && leaf[k] >= 0));
  }
  if (Pw.counters && q[0].lane == 0) {  // spread over kCounterSlots rows: no hot address
    unsigned long long* c = counter_row(Pw, sel0);
    atomicAdd(&c[kCntPrimary], nvalid);
    atomicAdd(&c[kCntHits], nhit);
#ifdef RT_DIAG
    atomicAdd(&c[kCntPrimNodes], dg.nodes);
    atomicAdd(&c[kCntPrimNodeLanes], dg.node_lanes);
    atomicAdd(&c[kCntPrimLeaves], dg.leaves);
    atomicAdd(&c[kCntPrimLeafLanes], dg.leaf_lanes);
    atomicAdd(&c[kCntPrimWide], dg.wide);
#endif
  }
}

// One piece of a packet in a sharing workgroup: the closest hit of tile sel's rays over the
// whole tree (node < 0) or over the shared subtree (node, mask); returns this lane's key.
template <bool FAST, bool SPHERES, bool CULL, int W>
__device__ __forceinline__ unsigned long long primary_piece(const RenderParams& P,
                                                            const DevNode* __restrict__ nodes,
                                                            const DevPrim* __restrict__ prims,
                                                            int sel, WaveLeafLds& L, Sharer<W>& sh,
                                                            int node, uint64_t mask, Diag& dg) {
  const PacketPixel q = packet_pixel(P, sel);
  const bool valid[1] = {q.valid};
  LaneRay ray[1] = {make_ray(ld3(P.cam_e), primary_dir(P, q.px, q.py), P.quot_ok)};
  asm volatile("" : "+v"(ray[0].o.x), "+v"(ray[0].o.y), "+v"(ray[0].o.z));  // (primary_packet)
  const bool any_skip = valid[0] && (ray[0].skip0 || ray[0].skip1 || ray[0].skip2);
  float t[1];
  int leaf[1];
  if (ballot(any_skip))
    closest_hit<true, FAST, false, SPHERES, 1, CULL>(P, nodes, prims, nullptr, L, ray, valid, t,
                                                     leaf, dg, sh, node, mask);
  else
    closest_hit<false, FAST, false, SPHERES, 1, CULL>(P, nodes, prims, nullptr, L, ray, valid, t,
                                                      leaf, dg, sh, node, mask);
  int2_t rec;
  rec.x = leaf[0];
  rec.y = __float_as_int(t[0]);
  return leaf[0] >= 0 ? hit_key(rec) : kNoHitKey;
}

// Hit point and normal of a primary hit, rebuilt from its {t, leaf} record exactly as
// trace_ray computes them (HW2/Scene.cpp:101-105; Sphere.h:42,50 for sphere normals).
__device__ __forceinline__ V3 hit_point(const RenderParams& P, const PacketPixel& q, float t) {
  return ld3(P.cam_e) + primary_dir(P, q.px, q.py) * t;  // Ray::point_at = o + t*d
}

// Shadow rays of HW2/Scene.cpp:113-127: one bit per point light, set when the light is
// occluded for this pixel's primary hit.  R tiles per wave as in primary_packet.
template <bool FAST, bool DEEP, bool SPHERES, int R, bool CULL, bool WO = false>
__device__ __forceinline__ void shadow_packet(const RenderParams& P0,
                                              const DevNode* __restrict__ nodes,
                                              const DevPrim* __restrict__ prims,
                                              const DevLight* __restrict__ lights, int sel0,
                                              int* spill, WaveLeafLds& L) {
  Diag dg;
  for (int w = 0; w < P0.occ_words; w++) {
    unsigned bits[R];
#pragma unroll
    for (int k = 0; k < R; k++) bits[k] = 0;
    const int lend = min(P0.num_lights, 32 * (w + 1));
    for (int li = 32 * w; li < lend; li++) {
      // per light: the pixel's hit record is re-read and its hit point rebuilt, so nothing but
      // the occlusion bits is live across the traversal (register pressure, not traffic: the
      // 8-B record is an L2 hit)
      const RenderParams& P = fresh_params(P0);
      const DevLight& lt = lights[li];
      LaneRay sr[R];
      float thr[R];
      bool hit[R];
      bool any_skip = false;
#pragma unroll
      for (int k = 0; k < R; k++) {
        const PacketPixel q = packet_pixel(P, sel0 + k);
        int2_t rec;
        rec.x = -2;
        rec.y = 0;
        if (sel0 + k < P.num_sel_tiles) rec = P.hits[(size_t)(sel0 + k) * (kTile * kTile) + q.lane];
        hit[k] = hit_leaf(rec) >= 0;
        const V3 pk = hit[k] ? hit_point(P, q, hit_t(rec)) : v3(0, 0, 0);
        const V3 ld = ld3(lt.position) - pk;
        const V3 wi = normalize(ld);
        const float dist = length(ld);
        sr[k] = make_ray(pk + wi * P.eps, wi, P.quot_ok);  // p + eps * w_i
        thr[k] = dist - P.eps;
        any_skip |= hit[k] && (sr[k].skip0 || sr[k].skip1 || sr[k].skip2);
      }
      bool occ[R];
      NoDonor nd;
      if (ballot(any_skip))
        occluded<true, FAST, DEEP, SPHERES, R, CULL, NoDonor, WO>(P, nodes, prims, spill, L, sr, hit, thr, occ, dg, nd);
      else
        occluded<false, FAST, DEEP, SPHERES, R, CULL, NoDonor, WO>(P, nodes, prims, spill, L, sr, hit, thr, occ, dg, nd);
#pragma unroll
      for (int k = 0; k < R; k++) bits[k] |= (occ[k] ? 1u : 0u) << (li - 32 * w);
    }
    const RenderParams& Pw = fresh_params(P0);
#pragma unroll
    for (int k = 0; k < R; k++)
      if (sel0 + k < Pw.num_sel_tiles)
        Pw.occ[((size_t)(sel0 + k) * (kTile * kTile) + lane_id()) * Pw.occ_words + w] = bits[k];
  }
  const RenderParams& Pc = fresh_params(P0);
  unsigned long long nhit = 0;
#pragma unroll
  for (int k = 0; k < R; k++) {
    const bool inside = sel0 + k < Pc.num_sel_tiles;
    nhit += __builtin_popcountll(
        ballot(inside && hit_leaf(Pc.hits[(size_t)(sel0 + k) * (kTile * kTile) + lane_id()]) >= 0));
  }
  if (Pc.counters && lane_id() == 0) {
    unsigned long long* c = counter_row(Pc, sel0);
    atomicAdd(&c[kCntShadow], nhit * (unsigned long long)Pc.num_lights);
#ifdef RT_DIAG
    atomicAdd(&c[kCntShadNodes], dg.nodes);
    atomicAdd(&c[kCntShadNodeLanes], dg.node_lanes);
    atomicAdd(&c[kCntShadLeaves], dg.leaves);
    atomicAdd(&c[kCntShadLeafLanes], dg.leaf_lanes);
    atomicAdd(&c[kCntShadWide], dg.wide);
#endif
  }
}

// One piece of a packet's shadow rays in a sharing workgroup: point light li for tile sel0
// (HW2/Scene.cpp:113-127 as in shadow_packet), over the whole tree (start_node < 0) or over a
// shared subtree.  Returns this lane's occlusion.
template <bool FAST, bool SPHERES, bool CULL, class DN>
__device__ __forceinline__ bool shadow_piece(const RenderParams& P0,
                                            const DevNode* __restrict__ nodes,
                                            const DevPrim* __restrict__ prims,
                                            const DevLight* __restrict__ lights, int sel0, int li,
                                            int* spill, WaveLeafLds& L, DN& dn, int start_node,
                                            uint64_t start_mask, Diag& dg) {
  const RenderParams& P = P0;
  const DevLight& lt = lights[li];
  const PacketPixel q = packet_pixel(P, sel0);
  const int2_t rec = P.hits[(size_t)sel0 * (kTile * kTile) + q.lane];
  bool hit[1] = {hit_leaf(rec) >= 0};
  const V3 pk = hit[0] ? hit_point(P, q, hit_t(rec)) : v3(0, 0, 0);
  const V3 ld = ld3(lt.position) - pk;
  const V3 wi = normalize(ld);
  const float dist = length(ld);
  LaneRay sr[1] = {make_ray(pk + wi * P.eps, wi, P.quot_ok)};  // p + eps * w_i
  float thr[1] = {dist - P.eps};
  const bool any_skip = hit[0] && (sr[0].skip0 || sr[0].skip1 || sr[0].skip2);
  bool occ[1];
  if (ballot(any_skip))
    occluded<true, FAST, false, SPHERES, 1, CULL>(P, nodes, prims, spill, L, sr, hit, thr, occ, dg,
                                                  dn, start_node, start_mask);
  else
    occluded<false, FAST, false, SPHERES, 1, CULL>(P, nodes, prims, spill, L, sr, hit, thr, occ,
                                                   dg, dn, start_node, start_mask);
  return occ[0];
}

// Local shading of HW2/Scene.cpp:101-138 given the occlusion bits, in the reference's
// accumulation order: ambient, then per light diffuse then specular.  No traversal here, so
// the fp64 pow (HW2 calls ::pow(double, double)) costs no occupancy in the traversal kernels.
__device__ __forceinline__ void shade_pixel(const RenderParams& P,
                                            const DevPrim* __restrict__ prims,
                                            const float* __restrict__ normals,
                                            const DevMaterial* __restrict__ mats,
                                            const DevLight* __restrict__ lights, int sel) {
  const PacketPixel q = packet_pixel(P, sel);
  const size_t pix = (size_t)sel * (kTile * kTile) + q.lane;
  const int2_t rec = P.hits[pix];
  const bool valid = hit_leaf(rec) != -2;
  const bool hit = hit_leaf(rec) >= 0;
  V3 color = v3(0.0f, 0.0f, 0.0f);
  if (hit) {
    const int leaf = hit_leaf(rec);
    const V3 e = ld3(P.cam_e);
    const V3 p = hit_point(P, q, hit_t(rec));
    const DevPrim& pr = prims[leaf];
    const V3 n = pr.kind == kPrimTriangle ? ld3(normals + 4 * leaf) : normalize(p - ld3(pr.v0));
    const DevMaterial& m = mats[pr.material];
    const V3 w0 = normalize(e - p);  // (ray.o - intersection_point).normalize()
    color = color + ld3(m.ambient) * ld3(P.ambient);
    for (int li = 0; li < P.num_lights; li++) {
      if ((P.occ[pix * P.occ_words + (li >> 5)] >> (li & 31)) & 1u) continue;
      const DevLight& L = lights[li];
      const V3 ld = ld3(L.position) - p;
      const V3 wi = normalize(ld);
      const float dist = length(ld);
      const V3 I = ld3(L.intensity);
      const float d2 = dist * dist;
      const float cos_d = dot(n, wi);
      color = color + ((ld3(m.diffuse) * I) * cos_d) / d2;
      const float cos_s = __builtin_fmaxf(dot(n, normalize(w0 + wi)), 0.0f);
      const float pw = (float)pow((double)cos_s, (double)m.phong_exponent);
      color = color + ((ld3(m.specular) * I) * pw) / d2;
    }
  } else if (valid) {
    color = ld3(P.background);  // primary miss: max_recursion_depth == depth
  }
  if (valid) {
    float* o;
    if (P.tile_major)
      o = P.out + 3 * pix;
    else
      o = P.out + 3 * ((size_t)q.py * P.width + q.px);
    o[0] = 0.0f + color.x;  // Pixel::add_color(color, 1) onto a zeroed pixel
    o[1] = 0.0f + color.y;
    o[2] = 0.0f + color.z;
  } else if (P.tile_major) {
    float* o = P.out + 3 * pix;
    o[0] = o[1] = o[2] = 0.0f;
  }
}

// ------------------------------------------------------------------ recursion (f1)
// HW2/Scene.cpp:88-196 with MaxRecursionDepth > 0: mirror rays (:141-146) and dielectrics
// (:149-194, refract_ray :72-86).  Each lane walks its ray tree in the reference's post order
// with an explicit stack of frames in HBM (layout [level][field][lane]); traversal calls stay
// wave-uniform packet calls over the lanes' current rays.  The parent's colour is combined
// with each child result in the source's order: color += km (x) child; and for a dielectric
// color += k (x) (r*refl + (1-r)*trans), with r*refl held in the frame until trans returns.
enum : int {
  kFrColor = 0, kFrStage = 3, kFrP = 4, kFrN = 7, kFrW0 = 10, kFrD = 13, kFrT = 16,
  kFrMat = 17, kFrDepth = 18, kFrMedium = 19, kFrK = 20, kFrR = 23, kFrA = 24, kFrFields = 28
};
enum : int {
  kStStart = 0, kStMirrorWait = 1, kStRefr = 2, kStTirWait = 3, kStReflWait = 4,
  kStTransWait = 5, kStDone = 6
};

struct FrameRef {
  float* base;
  size_t stride;  // floats between fields (= lanes in the launch)
  __device__ __forceinline__ float& f(int field) const { return base[(size_t)field * stride]; }
  __device__ __forceinline__ V3 v(int field) const { return v3(f(field), f(field + 1), f(field + 2)); }
  __device__ __forceinline__ void put(int field, V3 a) const {
    f(field) = a.x;
    f(field + 1) = a.y;
    f(field + 2) = a.z;
  }
  __device__ __forceinline__ int i(int field) const { return __float_as_int(f(field)); }
  __device__ __forceinline__ void put_i(int field, int x) const { f(field) = __int_as_float(x); }
};

// HW2/Scene.cpp:72-86
__device__ __forceinline__ bool refract_ray(V3 dir, V3 n, float idx, V3& out) {
  const float n_ratio = 1 / idx;
  const float cos_t = dot(v3(-dir.x, -dir.y, -dir.z), n);
  const float delta = 1 - (n_ratio) * (n_ratio) * (1 - (cos_t * cos_t));
  if (delta < 0.0f) return false;
  out = normalize((dir + n * cos_t) * n_ratio - n * __builtin_sqrtf(delta));
  return true;
}

// Local shading of one hit (ambient + point lights with shadow rays), Scene.cpp:107-139.
// Wave-uniform: every lane calls it; `shade` selects the lanes that shade (hit, !in_medium).
template <bool FAST, bool DEEP, bool SPHERES>
__device__ __forceinline__ V3 local_color(const RenderParams& P, const DevNode* __restrict__ nodes,
                                          const DevPrim* __restrict__ prims,
                                          const DevMaterial* __restrict__ mats,
                                          const DevLight* __restrict__ lights, int* spill, WaveLeafLds& L,
                                          bool shade, V3 o, V3 p, V3 n, int mat, Diag& dg,
                                          unsigned long long& shadow_rays) {
  V3 color = v3(0.0f, 0.0f, 0.0f);
  const DevMaterial& m = mats[shade ? mat : 0];
  if (shade) color = color + ld3(m.ambient) * ld3(P.ambient);
  const V3 w0 = shade ? normalize(o - p) : v3(0, 0, 0);
  for (int li = 0; li < P.num_lights; li++) {
    const DevLight& lt = lights[li];
    const V3 ld = ld3(lt.position) - p;
    const V3 wi = normalize(ld);
    const float dist = length(ld);
    const LaneRay sr[1] = {make_ray(p + wi * P.eps, wi, P.quot_ok)};
    const float thr[1] = {dist - P.eps};
    const bool act[1] = {shade};
    const bool sskip = ballot(shade && (sr[0].skip0 || sr[0].skip1 || sr[0].skip2)) != 0;
    bool occ[1];
    NoDonor nd;
    if (sskip)
      occluded<true, FAST, DEEP, SPHERES, 1>(P, nodes, prims, spill, L, sr, act, thr, occ, dg, nd);
    else
      occluded<false, FAST, DEEP, SPHERES, 1>(P, nodes, prims, spill, L, sr, act, thr, occ, dg, nd);
    shadow_rays += __builtin_popcountll(ballot(shade));
    if (shade && !occ[0]) {
      const V3 I = ld3(lt.intensity);
      const float d2 = dist * dist;
      color = color + ((ld3(m.diffuse) * I) * dot(n, wi)) / d2;
      const float cos_s = __builtin_fmaxf(dot(n, normalize(w0 + wi)), 0.0f);
      const float pw = (float)pow((double)cos_s, (double)m.phong_exponent);
      color = color + ((ld3(m.specular) * I) * pw) / d2;
    }
  }
  return color;
}

template <bool FAST, bool DEEP, bool SPHERES>
__device__ __forceinline__ void recursive_packet(const RenderParams& P,
                                                 const DevNode* __restrict__ nodes,
                                                 const DevPrim* __restrict__ prims,
                                                 const float* __restrict__ normals,
                                                 const DevMaterial* __restrict__ mats,
                                                 const DevLight* __restrict__ lights, int sel,
                                                 int* spill, WaveLeafLds& L) {
  const PacketPixel q = packet_pixel(P, sel);
  const size_t lanes_total = (size_t)P.num_sel_tiles * (kTile * kTile);
  const size_t g = (size_t)sel * (kTile * kTile) + q.lane;
  auto frame = [&](int level) {
    return FrameRef{P.frames + (size_t)level * kFrFields * lanes_total + g, lanes_total};
  };
  // current ray of this lane
  V3 ro = ld3(P.cam_e), rd = primary_dir(P, q.px, q.py);
  bool medium = false;
  int depth = P.max_depth;
  bool active = q.valid;  // has a ray to trace
  int sp = 0;             // frames on this lane's stack
  V3 res = v3(0, 0, 0), out = v3(0, 0, 0);
  Diag dg;
  unsigned long long n_primary = __builtin_popcountll(ballot(q.valid)), n_hits = 0;
  unsigned long long n_shadow = 0, n_secondary = 0;
  bool first = true;
  while (ballot(active)) {
    const LaneRay rays[1] = {make_ray(ro, rd, P.quot_ok)};
    const LaneRay& ray = rays[0];
    const bool act[1] = {active};
    const bool skip = ballot(active && (ray.skip0 || ray.skip1 || ray.skip2)) != 0;
    float ts[1];
    int leaves[1];
    NoDonor nd;
    if (skip)
      closest_hit<true, FAST, DEEP, SPHERES, 1>(P, nodes, prims, spill, L, rays, act, ts, leaves, dg, nd);
    else
      closest_hit<false, FAST, DEEP, SPHERES, 1>(P, nodes, prims, spill, L, rays, act, ts, leaves, dg, nd);
    const float t = ts[0];
    const int leaf = leaves[0];
    const bool hit = active && leaf >= 0;
    if (first) n_hits = __builtin_popcountll(ballot(hit));
    first = false;
    V3 p = v3(0, 0, 0), n = v3(0, 0, 0);
    int mat = 0;
    if (hit) {
      p = ray.o + ray.d * t;
      const DevPrim& pr = prims[leaf];
      n = pr.kind == kPrimTriangle ? ld3(normals + 4 * leaf) : normalize(p - ld3(pr.v0));
      mat = pr.material;
    }
    const V3 local = local_color<FAST, DEEP, SPHERES>(P, nodes, prims, mats, lights, spill, L,
                                                      hit && !medium, ray.o, p, n, mat, dg,
                                                      n_shadow);
    if (active) {
      bool spawned = false;
      if (hit) {  // open a frame for this hit
        const FrameRef F = frame(sp++);
        F.put(kFrColor, local);
        F.put_i(kFrStage, kStStart);
        F.put(kFrP, p);
        F.put(kFrN, n);
        F.put(kFrW0, normalize(ray.o - p));
        F.put(kFrD, ray.d);
        F.f(kFrT) = t;
        F.put_i(kFrMat, mat);
        F.put_i(kFrDepth, depth);
        F.put_i(kFrMedium, medium ? 1 : 0);
      } else {  // a miss returns background only at the primary depth (Scene.cpp:96-99)
        res = depth == P.max_depth ? ld3(P.background) : v3(0.0f, 0.0f, 0.0f);
      }
      // run the post-order state machine until a new ray is spawned or the tree is done
      while (sp > 0 && !spawned) {
        const FrameRef F = frame(sp - 1);
        const int stage = F.i(kFrStage);
        const DevMaterial& m = mats[F.i(kFrMat)];
        const int fdepth = F.i(kFrDepth);
        V3 color = F.v(kFrColor);
        const V3 fn = F.v(kFrN), fp = F.v(kFrP), fw0 = F.v(kFrW0);
        const V3 wr = normalize(fn * (2 * dot(fn, fw0)) - fw0);  // (2 n.w0) n - w0
        int next = stage;
        if (stage == kStStart) {
          const bool mirror = m.mirror[0] != 0.0f || m.mirror[1] != 0.0f || m.mirror[2] != 0.0f;
          if (mirror && fdepth > 0) {
            ro = fp + wr * P.eps;
            rd = wr;
            medium = false;
            spawned = true;
            next = kStMirrorWait;
          } else {
            next = kStRefr;
          }
        } else if (stage == kStMirrorWait) {
          color = color + ld3(m.mirror) * res;
          next = kStRefr;
        } else if (stage == kStRefr) {
          const bool glass = m.transparency[0] != 0.0f || m.transparency[1] != 0.0f ||
                             m.transparency[2] != 0.0f;
          if (glass && fdepth > 0) {
            V3 td = v3(0.0f, 0.0f, 0.0f), k = v3(0.0f, 0.0f, 0.0f);
            float cos_t = 0.0f;
            const V3 dn = normalize(F.v(kFrD));
            const float idx = m.refraction_index;
            bool tir = false, entering;
            if (dot(dn, fn) < 0.0f) {
              refract_ray(dn, fn, idx, td);
              cos_t = dot(v3(-dn.x, -dn.y, -dn.z), fn);
              k = v3(1.0f, 1.0f, 1.0f);
              entering = true;
            } else {
              const double tt = (double)F.f(kFrT);
              k.x = (float)exp(-log((double)m.transparency[0]) * tt);
              k.y = (float)exp(-log((double)m.transparency[1]) * tt);
              k.z = (float)exp(-log((double)m.transparency[2]) * tt);
              entering = false;
              if (refract_ray(dn, v3(-fn.x, -fn.y, -fn.z), 1.0f / idx, td))
                cos_t = dot(td, fn);
              else
                tir = true;
            }
            F.put(kFrK, k);
            ro = fp + wr * P.eps;
            rd = wr;
            spawned = true;
            if (tir) {
              medium = true;
              next = kStTirWait;
            } else {
              const float r0 = (idx - 1) * (idx - 1) / ((idx + 1) * (idx + 1));
              const float r =
                  (float)((double)r0 + (double)(1 - r0) * pow((double)(1 - cos_t), 5.0));
              F.f(kFrR) = r;
              F.put(kFrA, td);  // transmission direction until the reflection returns
              medium = !entering;
              F.put_i(kFrMedium, entering ? 1 : 0);  // medium flag of the transmission ray
              next = kStReflWait;
            }
          } else {
            next = kStDone;
          }
        } else if (stage == kStTirWait) {
          color = color + F.v(kFrK) * res;
          next = kStDone;
        } else if (stage == kStReflWait) {
          const V3 td = F.v(kFrA);
          F.put(kFrA, res * F.f(kFrR));  // r * trace(reflection)
          ro = fp + td * P.eps;
          rd = td;
          medium = F.i(kFrMedium) != 0;
          spawned = true;
          next = kStTransWait;
        } else if (stage == kStTransWait) {
          color = color + F.v(kFrK) * (F.v(kFrA) + res * (1 - F.f(kFrR)));
          next = kStDone;
        }
        if (next == kStDone) {
          res = color;
          sp--;
          continue;
        }
        F.put(kFrColor, color);
        F.put_i(kFrStage, next);
        if (spawned) {
          depth = fdepth - 1;
          n_secondary++;
        }
      }
      if (!spawned) {  // the whole tree of this pixel is done
        out = res;
        active = false;
      }
    }
  }
  if (q.valid) {
    float* o;
    if (P.tile_major)
      o = P.out + 3 * g;
    else
      o = P.out + 3 * ((size_t)q.py * P.width + q.px);
    o[0] = 0.0f + out.x;  // Pixel::add_color(color, 1) onto a zeroed pixel
    o[1] = 0.0f + out.y;
    o[2] = 0.0f + out.z;
  } else if (P.tile_major) {
    float* o = P.out + 3 * g;
    o[0] = o[1] = o[2] = 0.0f;
  }
  if (P.counters) {
    // n_secondary is per lane: reduce over the wave with atomics from every lane that spawned
    unsigned long long* c = counter_row(P, sel);
    if (n_secondary) atomicAdd(&c[kCntSecondary], n_secondary);
    if (q.lane == 0) {
      atomicAdd(&c[kCntPrimary], n_primary);
      atomicAdd(&c[kCntHits], n_hits);
      atomicAdd(&c[kCntShadow], n_shadow);
    }
  }
}

// Traversal kernels hide their dependent node loads with occupancy: hold them to 8 waves/SIMD
// (<= 64 VGPRs, <= 100 SGPRs); the compiler otherwise settles at 7 on SGPR count.
#ifndef RT_TRACE_MIN_WAVES  // (A/B: fewer waves per SIMD, more registers per wave)
#define RT_TRACE_MIN_WAVES 8
#endif
#ifndef RT_PRIMARY_MIN_WAVES  // primary kernel only (A/B: RT_PRIMARY_MIN_WAVES=8)
#define RT_PRIMARY_MIN_WAVES 7  // 32 more SGPRs for the wide node: frame 0.703 -> 0.691 ms
#endif
#define RT_PRIMARY_OCCUPANCY __attribute__((amdgpu_waves_per_eu(RT_PRIMARY_MIN_WAVES, 8)))
#ifndef RT_TRAVERSAL_OCCUPANCY
#define RT_TRAVERSAL_OCCUPANCY __attribute__((amdgpu_waves_per_eu(RT_TRACE_MIN_WAVES, 8)))
#endif

// XCD-aware block order: blocks b and b+8 share an XCD (round-robin dispatch), so hand each
// XCD a contiguous run of blocks — neighbouring packets share BVH nodes through its L2.
template <int W>
__device__ __forceinline__ int packet_index() {
  const int nb = (int)gridDim.x, b = (int)blockIdx.x;
  const int q = nb / 8, rem = nb % 8, x = b % 8;
  const int logical = (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + b / 8;
  return uniform(logical * W + ((int)threadIdx.x >> 6));
}

// Traversal workgroups: kTraceWaves packets, which the hardware keeps on ONE CU, so they share
// its scalar cache.  With P.tile_block the workgroup's packets form a kBlockW x kBlockH block
// of tiles (blocks row-major over the frame) instead of a run along a tile row: neighbouring
// rays walk the same nodes, and the cache serves them once.  Deep trees keep 4-wave groups
// (their LDS stack is 12 KB per wave).
#ifndef RT_TRACE_BLOCK_W
#define RT_TRACE_BLOCK_W 2
#endif
constexpr int kTraceWaves = RT_TRACE_WAVES;
template <bool DEEP>
constexpr int trace_waves() { return DEEP ? 4 : kTraceWaves; }

template <int W>
__host__ __device__ constexpr int block_w() { return W >= RT_TRACE_BLOCK_W ? RT_TRACE_BLOCK_W : W; }

// Tile (= sel, tile_step 1) of logical packet p; -1 for a padding packet of an edge block.
template <int W>
__device__ __forceinline__ int packet_sel(const RenderParams& P, int p) {
  if (!P.tile_block) return p;
  constexpr int BW = block_w<W>(), BH = W / BW;
  const int w = p % W, b = p / W;
  const int nbx = (P.tiles_x + BW - 1) / BW;
  const int tx = (b % nbx) * BW + w % BW, ty = (b / nbx) * BH + w / BW;
  const int tiles_y = P.tiles_total / P.tiles_x;
  return (tx < P.tiles_x && ty < tiles_y) ? ty * P.tiles_x + tx : -1;
}

// Logical packets of a traversal launch (R tiles each; with tile_block, padded to whole blocks).
template <int W, int R>
__host__ __device__ __forceinline__ int trace_packets(const RenderParams& P) {
  if (!P.tile_block) return (P.num_sel_tiles + R - 1) / R;
  constexpr int BW = block_w<W>(), BH = W / BW;
  const int tiles_y = P.tiles_total / P.tiles_x;
  return ((P.tiles_x + BW - 1) / BW) * ((tiles_y + BH - 1) / BH) * W;
}

// RT_TIMELINE (experiment builds only): every traversal wave records its start and end on the
// 100 MHz clock and its own tile, so tools/timeline.py can draw the occupancy curve of a launch.
#ifdef RT_TIMELINE
constexpr int kTimelineWaves = 1 << 18;
__device__ unsigned long long g_timeline[2][kTimelineWaves][3];
#define TL_BEGIN                                                   \
  int tl_sel = -1;                                                  \
  const unsigned long long tl0 = __builtin_amdgcn_s_memrealtime()
#define TL_SEL(x) tl_sel = (x)
#define TL_END(k)                                                                         \
  do {                                                                                    \
    const unsigned long long tl1 = __builtin_amdgcn_s_memrealtime();                      \
    const int wid = (int)blockIdx.x * (int)(blockDim.x >> 6) + ((int)threadIdx.x >> 6);   \
    if (lane_id() == 0 && wid < kTimelineWaves) {                                         \
      g_timeline[k][wid][0] = tl0;                                                        \
      g_timeline[k][wid][1] = tl1;                                                        \
      g_timeline[k][wid][2] = (unsigned long long)(long long)tl_sel;                       \
    }                                                                                     \
  } while (0)
#else
#define TL_BEGIN
#define TL_SEL(x)
#define TL_END(k)
#endif

// Sharing workgroups (RT_EXP_SHARE, R == 1, lane stack; see "subtree sharing"): each wave
// starts with its own packet, and every piece of work, own or shared, goes through the one call
// site in the loop.  Bit-identical, but slower on C3, so off by default: every
// wave traverses its own packet alone.
#ifdef RT_EXP_SHARE
constexpr bool kShare = true;
#else
constexpr bool kShare = false;
#endif

template <bool FAST, bool SPHERES, bool CULL, int W>
__device__ __forceinline__ void share_primary(const RenderParams& P, const DevNode* __restrict__ nodes,
                                              const DevPrim* __restrict__ prims, int sel,
                                              WaveLeafLds& L, BlockShare<W>& SH) {
  const int wv = (int)threadIdx.x >> 6, lane = lane_id();
  if (threadIdx.x == 0) SH.want = 0;
  if (lane == 0) {
    SH.sel[wv] = sel;
    SH.flag[wv] = 0;
  }
  SH.res[wv][lane] = kNoHitKey;
  __syncthreads();
  Sharer<W> sh;
  sh.S = &SH;
  sh.light = 0;
  Diag dg;
  int owner = wv, node = -1, light = 0;
  uint64_t mask = 0;
  bool have = sel >= 0;
  unsigned long long shared = 0;
  for (;;) {
    if (!have && !share_next(SH, owner, node, mask, light)) break;
    const int tsel = uniform(SH.sel[owner]);
    sh.owner = owner;
    sh.visits = 0;
    const unsigned long long key =
        primary_piece<FAST, SPHERES, CULL, W>(fresh_params(P), nodes, prims, tsel, L, sh,
                                               have ? -1 : node, mask, dg);
    if (key != kNoHitKey) atomicMin(&SH.res[owner][lane], key);
    shared += have ? 0 : 1;
    have = false;
  }
  __syncthreads();  // every piece of every packet of the workgroup has merged
  const RenderParams& Pw = fresh_params(P);
  if (sel >= 0) {
    const PacketPixel q = packet_pixel(Pw, sel);
    const unsigned long long key = SH.res[wv][lane];
    int2_t rec;  // key layout: leaf low, t bits high (rt_internal.h)
    rec.x = q.valid ? (int)(unsigned)key : -2;  // -1 miss, -2 outside the image
    rec.y = (int)(unsigned)(key >> 32);
    Pw.hits[(size_t)sel * (kTile * kTile) + q.lane] = rec;
    const unsigned long long nvalid = __builtin_popcountll(ballot(q.valid));
    const unsigned long long nhit = __builtin_popcountll(ballot(q.valid && rec.x >= 0));
    if (Pw.counters && lane == 0) {
      unsigned long long* c = counter_row(Pw, sel);
      atomicAdd(&c[kCntPrimary], nvalid);
      atomicAdd(&c[kCntHits], nhit);
    }
  }
  if (Pw.counters && lane == 0) {
    unsigned long long* c = counter_row(Pw, (int)blockIdx.x);
    if (shared) atomicAdd(&c[kCntShared], shared);
#ifdef RT_DIAG
    atomicAdd(&c[kCntPrimNodes], dg.nodes);
    atomicAdd(&c[kCntPrimNodeLanes], dg.node_lanes);
    atomicAdd(&c[kCntPrimLeaves], dg.leaves);
    atomicAdd(&c[kCntPrimLeafLanes], dg.leaf_lanes);
    atomicAdd(&c[kCntPrimWide], dg.wide);
#endif
  }
}

// Shadow rays in a sharing workgroup, 32 lights (one occlusion word) at a time: the waves split
// the word's (packet, light) traversals, merge the occlusion bits per packet in LDS, and write
// the word after a workgroup barrier.
template <bool FAST, bool SPHERES, bool CULL, int W>
__device__ __forceinline__ void share_shadow(const RenderParams& P, const DevNode* __restrict__ nodes,
                                             const DevPrim* __restrict__ prims,
                                             const DevLight* __restrict__ lights, int sel,
                                             WaveLeafLds& L, BlockShare<W>& SH) {
  const int wv = (int)threadIdx.x >> 6, lane = lane_id();
  const int nl = P.num_lights, words = P.occ_words;
  if (lane == 0) SH.sel[wv] = sel;
  Sharer<W> sh;
  sh.S = &SH;
  Diag dg;
  unsigned long long shared = 0;
  for (int w = 0; w < words; w++) {
    if (threadIdx.x == 0) SH.want = 0;
    if (lane == 0) SH.flag[wv] = 0;
    SH.res[wv][lane] = 0ull;
    __syncthreads();
    const int lend = min(nl, 32 * (w + 1));
    int li = 32 * w, owner = wv, node = -1, light = 0;
    uint64_t mask = 0;
    for (;;) {
      const bool have = sel >= 0 && li < lend;
      if (have) {
        owner = wv;
        light = li++;
      } else if (!share_next(SH, owner, node, mask, light)) {
        break;
      }
      sh.owner = owner;
      sh.light = light;
      sh.visits = 0;
      const bool occ = shadow_piece<FAST, SPHERES, CULL>(fresh_params(P), nodes, prims, lights,
                                                         uniform(SH.sel[owner]), light, nullptr, L,
                                                         sh, have ? -1 : node, mask, dg);
      if (occ) atomicOr(&SH.res[owner][lane], 1ull << (light & 31));
      shared += have ? 0 : 1;
    }
    __syncthreads();  // every piece of this word has merged
    if (sel >= 0) {
      const RenderParams& Pw = fresh_params(P);
      Pw.occ[((size_t)sel * (kTile * kTile) + lane) * words + w] = (unsigned)SH.res[wv][lane];
    }
  }
  const RenderParams& Pc = fresh_params(P);
  if (sel >= 0) {
    const bool hit = hit_leaf(Pc.hits[(size_t)sel * (kTile * kTile) + lane]) >= 0;
    const unsigned long long nhit = __builtin_popcountll(ballot(hit));
    if (Pc.counters && lane == 0)
      atomicAdd(&counter_row(Pc, sel)[kCntShadow], nhit * (unsigned long long)nl);
  }
  if (Pc.counters && lane == 0) {
    unsigned long long* c = counter_row(Pc, (int)blockIdx.x);
    if (shared) atomicAdd(&c[kCntShared], shared);
#ifdef RT_DIAG
    atomicAdd(&c[kCntShadNodes], dg.nodes);
    atomicAdd(&c[kCntShadNodeLanes], dg.node_lanes);
    atomicAdd(&c[kCntShadLeaves], dg.leaves);
    atomicAdd(&c[kCntShadLeafLanes], dg.leaf_lanes);
    atomicAdd(&c[kCntShadWide], dg.wide);
#endif
  }
}

// Traversal kernels: one packet per wave, XCD-remapped blocks of 2-D tile blocks.
template <bool FAST, bool DEEP, bool SPHERES, int R, bool CULL, bool WO = false>
__global__ __launch_bounds__(trace_waves<DEEP>() * 64) RT_PRIMARY_OCCUPANCY void trace_primary_kernel(
    RenderParams P, const DevNode* __restrict__ nodes, const DevPrim* __restrict__ prims) {
  extern __shared__ __attribute__((aligned(16))) int deep_stack[];
  constexpr int W = trace_waves<DEEP>();
  __shared__ WaveLeafLds leaf_lds[W];  // 2 KiB per wave
  int* spill = DEEP ? deep_stack + ((int)threadIdx.x >> 6) * (1 + 2 * R) * kDeepStack : nullptr;
  WaveLeafLds& L = leaf_lds[threadIdx.x >> 6];
  TL_BEGIN;
  const RenderParams& Q = fresh_params(P);
  const int p = packet_index<W>();
  int sel = p < trace_packets<W, R>(Q) ? (R == 1 ? packet_sel<W>(Q, p) : p * R) : -1;
  if (sel >= Q.num_sel_tiles) sel = -1;
  TL_SEL(sel);
  if constexpr (kShare && R == 1 && !DEEP) {
    __shared__ BlockShare<W> SH;
    share_primary<FAST, SPHERES, CULL, W>(P, nodes, prims, sel, L, SH);
  } else if (sel >= 0) {
    const unsigned long long c0 = __builtin_amdgcn_s_memrealtime();
    primary_packet<FAST, DEEP, SPHERES, R, CULL, WO>(Q, nodes, prims, sel, spill, L);
    const RenderParams& Pw = fresh_params(P);
    if (R == 1 && Pw.tile_cost && lane_id() == 0)  // the shadow kernel's dispatch order
      Pw.tile_cost[sel] = (unsigned)min(__builtin_amdgcn_s_memrealtime() - c0, 0xffffffffull);
  }
  TL_END(0);
}

template <bool FAST, bool DEEP, bool SPHERES, int R, bool CULL, bool WO = false>
__global__ __launch_bounds__(trace_waves<DEEP>() * 64) RT_TRAVERSAL_OCCUPANCY void trace_shadow_kernel(
    RenderParams P, const DevNode* __restrict__ nodes, const DevPrim* __restrict__ prims,
    const DevLight* __restrict__ lights) {
  extern __shared__ __attribute__((aligned(16))) int deep_stack[];
  constexpr int W = trace_waves<DEEP>();
  __shared__ WaveLeafLds leaf_lds[W];  // 2 KiB per wave
  int* spill = DEEP ? deep_stack + ((int)threadIdx.x >> 6) * (1 + 2 * R) * kDeepStack : nullptr;
  WaveLeafLds& L = leaf_lds[threadIdx.x >> 6];
  TL_BEGIN;
  const RenderParams& Q = fresh_params(P);
  int sel;
  if (R == 1 && Q.tile_order) {  // slowest primary tiles first, in plain block order
    const int p = uniform((int)blockIdx.x * W + ((int)threadIdx.x >> 6));
    sel = p < Q.num_sel_tiles ? uniform(Q.tile_order[p]) : -1;
  } else {
    const int p = packet_index<W>();
    sel = p < trace_packets<W, R>(Q) ? (R == 1 ? packet_sel<W>(Q, p) : p * R) : -1;
  }
  if (sel >= Q.num_sel_tiles) sel = -1;
  TL_SEL(sel);
  if constexpr (kShare && R == 1 && !DEEP) {
    __shared__ BlockShare<W> SH;
    share_shadow<FAST, SPHERES, CULL, W>(P, nodes, prims, lights, sel, L, SH);
  } else if (sel >= 0) {
    shadow_packet<FAST, DEEP, SPHERES, R, CULL, WO>(Q, nodes, prims, lights, sel, spill, L);
  }
  TL_END(1);
}

template <bool FAST, bool DEEP, bool SPHERES>
__global__ __launch_bounds__(kWavesPerBlock * 64) void recursive_kernel(
    RenderParams P, const DevNode* __restrict__ nodes, const DevPrim* __restrict__ prims,
    const float* __restrict__ normals, const DevMaterial* __restrict__ mats,
    const DevLight* __restrict__ lights) {
  extern __shared__ __attribute__((aligned(16))) int deep_stack[];
  __shared__ WaveLeafLds leaf_lds[kWavesPerBlock];
  const int sel = packet_index<kWavesPerBlock>();
  if (sel >= P.num_sel_tiles) return;
  int* spill = DEEP ? deep_stack + ((int)threadIdx.x >> 6) * 3 * kDeepStack : nullptr;
  recursive_packet<FAST, DEEP, SPHERES>(P, nodes, prims, normals, mats, lights, sel, spill, leaf_lds[threadIdx.x >> 6]);
}

__global__ __launch_bounds__(kWavesPerBlock * 64) void shade_kernel(
    RenderParams P, const DevPrim* __restrict__ prims, const float* __restrict__ normals,
    const DevMaterial* __restrict__ mats, const DevLight* __restrict__ lights) {
  const int sel = uniform((int)blockIdx.x * kWavesPerBlock + ((int)threadIdx.x >> 6));
  if (sel >= P.num_sel_tiles) return;
  shade_pixel(P, prims, normals, mats, lights, sel);
}

// Heavy-first dispatch order for the shadow kernel: the tiles sorted by their primary traversal
// time, slowest first (a bucket sort on 8 steps per octave; order inside a bucket is free).
// The slow primary tiles are where the slow shadow tiles are (tools/timeline.py tile maps), and
// a kernel's tail is set by the slow tiles that start last.  One workgroup.
constexpr int kOrderBuckets = 256;
__device__ __forceinline__ int cost_bucket(unsigned c) {
  c = c ? c : 1u;
  const int msb = 31 - __builtin_clz(c);
  const int frac = msb >= 3 ? (int)((c >> (msb - 3)) & 7u) : (int)((c << (3 - msb)) & 7u);
  return min(kOrderBuckets - 1, msb * 8 + frac);
}

__global__ __launch_bounds__(1024) void order_kernel(const unsigned* __restrict__ cost,
                                                     int* __restrict__ order, int n) {
  __shared__ int hist[kOrderBuckets];
  const int tid = (int)threadIdx.x;
  for (int i = tid; i < kOrderBuckets; i += 1024) hist[i] = 0;
  __syncthreads();
  for (int i = tid; i < n; i += 1024) atomicAdd(&hist[cost_bucket(cost[i])], 1);
  __syncthreads();
  if (tid == 0) {  // exclusive offsets, heaviest bucket first
    int run = 0;
    for (int b = kOrderBuckets - 1; b >= 0; b--) {
      const int c = hist[b];
      hist[b] = run;
      run += c;
    }
  }
  __syncthreads();
  for (int i = tid; i < n; i += 1024) order[atomicAdd(&hist[cost_bucket(cost[i])], 1)] = i;
}

// marks (nullable): 4 events recorded before the primary kernel, after it, after the shadow
// kernel and after the shade kernel (rt_set_kernel_timing).  A recursive scene's single kernel
// is timed between marks 2 and 3.
static inline void mark(const hipEvent_t* marks, int k, hipStream_t stream) {
  if (marks) (void)hipEventRecord(marks[k], stream);
}

template <bool FAST, bool DEEP, bool SPHERES, bool CULL, bool WO = false>
static void launch_variant(const RenderParams& P, const DevNode* nodes, const DevPrim* prims,
                           const float* normals, const DevMaterial* mats,
                           const DevLight* lights, int blocks, const hipEvent_t* marks,
                           hipStream_t stream) {
  const size_t lds = DEEP ? sizeof(int) * 3 * kDeepStack * kWavesPerBlock : 0;
  if (P.frames) {  // recursive scenes: one kernel walks each pixel's ray tree
    mark(marks, 0, stream);
    mark(marks, 1, stream);
    mark(marks, 2, stream);
    hipLaunchKernelGGL((recursive_kernel<FAST, DEEP, SPHERES>), dim3(blocks),
                       dim3(kWavesPerBlock * 64), lds, stream, P, nodes, prims, normals, mats,
                       lights);
    mark(marks, 3, stream);
    return;
  }
  constexpr int R = kRaysPerLane;
  constexpr int W = trace_waves<DEEP>();
  RenderParams T = P;
  T.tile_block = R == 1 && P.tile_begin == 0 && P.tile_step == 1;
  int tblocks = (trace_packets<W, R>(T) + W - 1) / W;
  const size_t tlds = DEEP ? sizeof(int) * (1 + 2 * R) * kDeepStack * W : 0;
  RenderParams S = T;
  S.tile_cost = nullptr;  // (read by the shadow kernel through tile_order only)
  const bool ordered = R == 1 && P.num_lights > 0 && T.tile_order != nullptr;
  if (!ordered) T.tile_cost = S.tile_cost = nullptr, T.tile_order = S.tile_order = nullptr;
  mark(marks, 0, stream);
  hipLaunchKernelGGL((trace_primary_kernel<FAST, DEEP, SPHERES, R, CULL, WO>), dim3(tblocks),
                     dim3(W * 64), tlds, stream, T, nodes, prims);
  mark(marks, 1, stream);
  if (ordered)
    hipLaunchKernelGGL(order_kernel, dim3(1), dim3(1024), 0, stream, T.tile_cost, T.tile_order,
                       T.num_sel_tiles);
  const int sblocks = ordered ? (T.num_sel_tiles + W - 1) / W : tblocks;
  if (P.num_lights > 0)
    hipLaunchKernelGGL((trace_shadow_kernel<FAST, DEEP, SPHERES, R, CULL, WO>), dim3(sblocks),
                       dim3(W * 64), tlds, stream, S, nodes, prims, lights);
  mark(marks, 2, stream);
  hipLaunchKernelGGL(shade_kernel, dim3(blocks), dim3(kWavesPerBlock * 64), 0, stream, P,
                     prims, normals, mats, lights);
  mark(marks, 3, stream);
}

// Gaussian splat of HW2/Scene.cpp:46-62 turned inside out: one thread per destination pixel
// gathers every contribution the reference adds to it, in the order a single-threaded
// render_image adds them (source rows, source columns, samples x-major), so the fp32 sums of
// Pixel::add_color are reproduced exactly; then Pixel::get_color's color / weight.
__device__ __forceinline__ float gaussian_filter(float x, float y, float sigma) {
  // HW2/Scene.cpp:12-14: double exp of a float argument, double division, narrowed
  return (float)(exp((double)(-(x * x + y * y) / (2 * sigma * sigma))) /
                 (2 * M_PI * (double)sigma));
}

__global__ __launch_bounds__(256) void msaa_resolve_kernel(MsaaResolveParams M) {
  const int ai = (int)(blockIdx.x * 16 + (threadIdx.x & 15));
  const int aj = (int)(blockIdx.y * 16 + (threadIdx.x >> 4));
  if (ai >= M.width || aj >= M.height) return;
  const int n = M.n, S = n * n;
  const size_t frame = (size_t)M.width * M.height * 3;
  float cr = 0.0f, cg = 0.0f, cb = 0.0f, wsum = 0.0f;
  for (int j = aj - 1; j < aj + 2; j++) {
    if (j < 0 || j >= M.height) continue;
    for (int i = ai - 1; i < ai + 2; i++) {
      if (i < 0 || i >= M.width) continue;
      unsigned u = minstd_state0(
          msaa_pixel_seed(M.seed, (unsigned long long)j * (unsigned)M.width + (unsigned)i));
      const float* src = M.samples + 3 * ((size_t)j * M.width + i);
      for (int k = 0; k < S; k++) {
        u = minstd_mulmod(u, kMinstdA);
        const float ex = minstd_uniform01(u);
        u = minstd_mulmod(u, kMinstdA);
        const float ey = minstd_uniform01(u);
        const float sample_x = ((float)(k / n) + ex) / (float)n;
        const float sample_y = ((float)(k % n) + ey) / (float)n;
        const float s_x = ((float)i + sample_x) - ((float)ai + 0.5f);
        const float s_y = ((float)j + sample_y) - ((float)aj + 0.5f);
        const float w = gaussian_filter(s_x, s_y, 1.0f / 3.0f);
        const float* c = src + (size_t)k * frame;
        cr = cr + c[0] * w;
        cg = cg + c[1] * w;
        cb = cb + c[2] * w;
        wsum = wsum + w;
      }
    }
  }
  float* o = M.out + 3 * ((size_t)aj * M.width + ai);
  o[0] = cr / wsum;
  o[1] = cg / wsum;
  o[2] = cb / wsum;
}

hipError_t launch_msaa_resolve(const MsaaResolveParams& M, hipStream_t stream) {
  const dim3 grid((M.width + 15) / 16, (M.height + 15) / 16);
  hipLaunchKernelGGL(msaa_resolve_kernel, grid, dim3(256), 0, stream, M);
  return hipGetLastError();
}

int max_supported_depth() { return kDeepStack; }

// Self-check of tri_quotients against `/` on random operands spanning the whole fast range:
// |det| in [2^-40, 2^40] (a quarter with all-ones mantissas, where a reciprocal is hardest),
// numerators 0 or in [2^-49, 2^49], a quarter of them chosen so the quotient sits next to a
// rounding midpoint.  counts[0] += mismatches, counts[1] += cases.
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void quot_check_kernel(unsigned long long seed, long long count,
                                                         unsigned long long* counts) {
  unsigned long long bad = 0, n = 0;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < count; i += (long long)gridDim.x * 256) {
    const unsigned long long a = mix64(seed + 0x9E3779B97F4A7C15ull * (unsigned long long)(i + 1));
    const unsigned long long b = mix64(a ^ 0xD1B54A32D192ED03ull);
    const int ed = (int)(a % 81) - 40, en = (int)((a >> 8) % 99) - 49;
    unsigned md = (unsigned)(a >> 16) & 0x7fffffu;
    if (((a >> 40) & 3) == 0) md = 0x7fffffu - (unsigned)((a >> 42) & 3);
    float det = __uint_as_float(((unsigned)(ed + 127) << 23) | md);
    if ((a >> 44) & 1) det = -det;
    float num = __uint_as_float(((unsigned)(en + 127) << 23) | ((unsigned)b & 0x7fffffu));
    if ((b >> 23) & 1) num = -num;
    if (((b >> 24) & 3) == 0) {  // num = det * (a quotient just off a midpoint)
      const double q = ldexp(1.0 + (((b >> 26) & 0x7fffff) + 0.5) / 8388608.0, en - ed);
      const float m = (float)(q * (double)det);
      if (quot_coord(m) && __builtin_fabsf(m) >= 0x1p-49f && __builtin_fabsf(m) <= 0x1p49f) num = m;
    }
    if (((b >> 50) & 15) == 0) num = 0.0f;
    const V3 got = tri_quotients(v3(num, -num, num), det, true);
    const float want = num / det, wneg = (-num) / det;
    bad += (unsigned)(__float_as_uint(got.x) != __float_as_uint(want)) |
           (unsigned)(__float_as_uint(got.y) != __float_as_uint(wneg));
    n++;
  }
  atomicAdd(&counts[0], bad);
  atomicAdd(&counts[1], n);
}

hipError_t launch_quot_check(unsigned long long seed, long long count, unsigned long long* counts,
                             hipStream_t stream) {
  hipLaunchKernelGGL(quot_check_kernel, dim3(2048), dim3(256), 0, stream, seed, count, counts);
  return hipGetLastError();
}

hipError_t launch_render(const RenderParams& P, const DevNode* nodes, const DevPrim* prims,
                         const float* normals, const DevMaterial* mats, const DevLight* lights,
                         bool fast, bool deep, bool spheres, bool cull, bool wide_only,
                         const hipEvent_t* marks, hipStream_t stream) {
  if (P.num_sel_tiles <= 0) return hipSuccess;
  const int blocks = (P.num_sel_tiles + kWavesPerBlock - 1) / kWavesPerBlock;
  // wide_only (the culling tree is 4-wide and reaches no binary node): kernels without the
  // binary visit path, which costs the wide walk registers when compiled in
  const bool wo = wide_only && fast && !deep && !cull && kRaysPerLane == 1 && kBatchLeaves;
  const int v = (wo ? 16 : 0) | (fast && cull ? 8 : 0) | (fast ? 4 : 0) | (deep ? 2 : 0) |
                (spheres ? 1 : 0);
  switch (v) {
#define RT_CASE(F, D, S, C, W)                                                                    \
  case (W ? 16 : 0) | (C ? 8 : 0) | (F ? 4 : 0) | (D ? 2 : 0) | (S ? 1 : 0):                      \
    launch_variant<F, D, S, C, W>(P, nodes, prims, normals, mats, lights, blocks, marks, stream); \
    break;
    RT_CASE(true, false, false, false, true)
    RT_CASE(true, false, true, false, true)
    RT_CASE(true, false, false, false, false)
    RT_CASE(true, false, true, false, false)
    RT_CASE(true, true, false, false, false)
    RT_CASE(true, true, true, false, false)
    RT_CASE(false, false, false, false, false)
    RT_CASE(false, false, true, false, false)
    RT_CASE(false, true, false, false, false)
    RT_CASE(false, true, true, false, false)
    RT_CASE(true, false, false, true, false)
    RT_CASE(true, false, true, true, false)
    RT_CASE(true, true, false, true, false)
    RT_CASE(true, true, true, true, false)
#undef RT_CASE
  }
  return hipGetLastError();
}

unsigned long long read_reset_exact_fallbacks() {
#ifdef RT_DIAG
  unsigned long long v = 0, z = 0;
  (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_exact_fallbacks), sizeof v);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_exact_fallbacks), &z, sizeof z);
  return v;
#else
  return 0;
#endif
}

// Copies (and clears) the RT_TIMELINE wave records: out[2][kTimelineWaves][3] start/end
// ticks of the 100 MHz clock and tile (sel, -1 for none).  Returns the number of values written, 0 in other builds.
long long read_reset_timeline(unsigned long long* out, long long max_values) {
#ifdef RT_TIMELINE
  const long long n = 2ll * kTimelineWaves * 3;
  if (max_values < n) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_timeline), n * sizeof *out) != hipSuccess) return -1;
  std::vector<unsigned long long> z((size_t)n, 0ull);
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_timeline), z.data(), n * sizeof *out) != hipSuccess) return -1;
  return n;
#else
  (void)out;
  (void)max_values;
  return 0;
#endif
}

bool diag_build() {
#ifdef RT_DIAG
  return true;
#else
  return false;
#endif
}

}  // namespace rt
