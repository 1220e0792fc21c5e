// MI355X (gfx950) render kernels: HW2's Scene::render_image -> trace_ray -> BVH::intersect ->
// Triangle/Sphere::intersect -> Point_light shading + shadow rays.
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
//     any visiting order gives the reference's answer;
//   * leaf tests are queued per wave in LDS and run 64 at a time, one (ray, leaf) pair per lane.
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

#ifdef RT_DIAG
#define DIAG(stmt) stmt
#else
#define DIAG(stmt)
#endif
struct Diag {  // per-wave traversal work (RT_DIAG builds)
  unsigned long long nodes = 0, node_lanes = 0, leaves = 0, leaf_lanes = 0, wide = 0, guard = 0;
  // per-phase attribution (rt_debug_phases): events of the visit loop, and shader-clock cycles
  // (s_memrealtime, 100 MHz) of this wave spent in its phases
  unsigned long long ev[kPhaseEvents] = {};
  unsigned long long cyc_visit = 0, cyc_load = 0, cyc_flush = 0;
};
#ifdef RT_DIAG
// [0, kPhaseEvents): primary events, [kPhaseEvents, 2 kPhaseEvents): shadow events, then the
// cycle counters (kPhCyc*)
__device__ unsigned long long g_phase[kPhaseSlots];
__device__ __forceinline__ unsigned long long clock_now() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  return t;
}
#endif

// Packets (8x8 tiles, one wave each) per traversal workgroup.  Two: a workgroup's LDS (leaf
// queues, ~5.6 KiB per wave, which like the VGPRs caps a CU at 28 waves) stays allocated until
// its slowest wave ends, so the finished waves of a 4-wave workgroup hold slots a new workgroup
// cannot use; with two, half as much sits idle behind a heavy packet (C3: frame 0.335 -> 0.327
// ms with six in flight, a 1/8 band 0.047 -> 0.045 ms; profiles/r06/ab_trace_waves.json).
// (A/B builds: 1, 2 or 4.)
#ifndef RT_TRACE_WAVES
#define RT_TRACE_WAVES 2
#endif
constexpr int kTraceWaves = RT_TRACE_WAVES;
static_assert(kTraceWaves == 1 || kTraceWaves == 2 || kTraceWaves == 4, "1, 2 or 4 waves");
// A split tile's quadrants take kSplitEntries workgroups of kTraceWaves waves.
constexpr int kQuadrants = 4, kSplitEntries = kQuadrants / kTraceWaves;

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
  V3 m;       // 2^-18 |o| / d per axis: the ray's share of the culling margin (visit_wide)
  bool skip0, skip1, skip2;  // |d_i| < 1e-6: axis ignored (HW2/bounding_box.cpp:21)
  bool quot;  // origin and scene in the shared-reciprocal range (tri_quotients)
  int sh0, sh1, sh2;  // 16 where 1/d_i < 0 (the slot's hi plane is the entry plane), else 0
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
  r.m = v3(0x1p-18f * __builtin_fabsf(o.x) * r.r.x, 0x1p-18f * __builtin_fabsf(o.y) * r.r.y,
           0x1p-18f * __builtin_fabsf(o.z) * r.r.z);
  r.skip0 = __builtin_fabsf(d.x) < kEps;
  r.skip1 = __builtin_fabsf(d.y) < kEps;
  r.skip2 = __builtin_fabsf(d.z) < kEps;
  r.quot = scene_quot_ok && quot_coord(o.x) && quot_coord(o.y) && quot_coord(o.z);
  r.sh0 = (int)((__float_as_uint(r.r.x) >> 27) & 16u);
  r.sh1 = (int)((__float_as_uint(r.r.y) >> 27) & 16u);
  r.sh2 = (int)((__float_as_uint(r.r.z) >> 27) & 16u);
  return r;
}

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
// This lane's bit of a wave-uniform mask, as the exec mask itself (s_and_saveexec) — written as
// (m >> lane) & 1 the compiler keeps a 64-bit 1 << lane per lane (two VGPRs, spilled in the
// traversal kernels) and tests it with v_and + v_cmp_u64 at every queue push.
__device__ __forceinline__ bool lane_in(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); }
// Lane masks of one fp32 compare, straight from the v_cmp (ballot of a combined boolean makes
// the compiler round-trip it through a VGPR: v_cndmask + v_cmp per mask).  LLVM FCmp
// predicates; ordered, so NaN gives false as the C++ operators do.
enum : int { kFcmpOGT = 2, kFcmpOGE = 3, kFcmpOLT = 4, kFcmpULT = 12 };
__device__ __forceinline__ uint64_t lanes_gt(float a, float b) { return __builtin_amdgcn_fcmpf(a, b, kFcmpOGT); }
__device__ __forceinline__ uint64_t lanes_ge(float a, float b) { return __builtin_amdgcn_fcmpf(a, b, kFcmpOGE); }
__device__ __forceinline__ uint64_t lanes_lt(float a, float b) { return __builtin_amdgcn_fcmpf(a, b, kFcmpOLT); }
// !(a >= b): true for a NaN operand too
__device__ __forceinline__ uint64_t lanes_nge(float a, float b) { return __builtin_amdgcn_fcmpf(a, b, kFcmpULT); }
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
// flagged for box_exact.  tnear (approximate entry distance) only orders.
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

template <bool SKIP>
__device__ __forceinline__ void slab_fast(const float* b, const LaneRay& r, float& tn,
                                          bool& accept, bool& undecided) {
  float tf;
  slab_span<SKIP>(b, r, tn, tf);
  bool out;
  decide_sure(tn, tf, accept, out);
  undecided = !(accept | out);
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

// Correctly rounded n / det for the three numerators with ONE reciprocal.  gfx950's IEEE
// division is v_div_scale (num, den), y = v_rcp, e = fma(-den, y, 1), y1 = fma(e, y, y),
// q = num * y1, r = fma(-den, q, num), q1 = fma(r, y1, q), r1 = fma(-den, q1, num),
// v_div_fmas(r1, y1, q1), v_div_fixup(q2, den, num).  When no operand is near the exponent
// limits, v_div_scale returns its operand unchanged with VCC = 0 and v_div_fmas is a plain
// fma, so the sequence below (which keeps v_div_fixup: it gives a zero numerator the sign
// num ^ den) yields the bits of `/`; only the reciprocal refinement y1 depends on det alone,
// and it is shared.  Range: 2^-40 <= |det| <= 2^40 is checked here; numerators are 0 or
// 2^-49 <= |n| <= 2^49 by r.quot (every v0 and origin coordinate is 0 or in [2^-26, 2^48]).
// Then |n / det| lies in [2^-89, 2^89], exponent differences stay below 96 and nothing is
// subnormal, so none of v_div_scale's scaling cases can arise.  Any other lane takes `/`.
__device__ __forceinline__ float quot_step(float n, float det, float y1) {
  const float q = n * y1;
  const float r = __builtin_fmaf(-det, q, n);
  const float q1 = __builtin_fmaf(r, y1, q);
  const float r1 = __builtin_fmaf(-det, q1, n);
  return __builtin_amdgcn_div_fixupf(__builtin_fmaf(r1, y1, q1), det, n);
}

__device__ __forceinline__ V3 tri_quotients(V3 n, float det, bool quot) {
  const float ad = __builtin_fabsf(det);
  if (quot && ad >= 0x1p-40f && ad <= 0x1p40f) {
    const float y = __builtin_amdgcn_rcpf(det);
    const float e = __builtin_fmaf(-det, y, 1.0f);
    const float y1 = __builtin_fmaf(e, y, y);
    return v3(quot_step(n.x, det, y1), quot_step(n.y, det, y1), quot_step(n.z, det, y1));
  }
  return n / det;
}

// Branch-free: every value is computed and the reference's early exits (Triangle.cpp:46-62)
// become one predicate with the same comparisons (a NaN fails them as there).  With det == 0
// the quotients are inf/NaN and unused.
__device__ __forceinline__ bool tri_test(V3 v0, V3 a1, V3 a2, const LaneRay& r, float& t) {
  const float det = det3(a1, a2, r.d);
  const V3 b = tri_quotients(v0 - r.o, det, r.quot);
  const float beta = det3(b, a2, r.d);
  const float gamma = det3(a1, b, r.d);
  const float tt = det3(a1, a2, b);
  t = tt;
  return (det != 0.0f) & !((beta < 0.0f) | (beta > 1.0f)) &
         !((gamma < 0.0f) | (beta + gamma > 1.0f)) & (tt > 0.0f);
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
template <bool SPHERES>
__device__ __forceinline__ bool leaf_test(const DevPrim* __restrict__ prims, int leaf,
                                          const LaneRay& r, float& t) {
  const DevPrim& p = prims[leaf];
  const V3 v0 = ld3(p.v0);
  if (!SPHERES || p.kind == kPrimTriangle) return tri_test(v0, ld3(p.a1), ld3(p.a2), r, t);
  return sphere_test(v0, p.a1[0], r, t);
}

// ------------------------------------------------------------------ traversal stack
// Wave-uniform (node, lane-mask) entries.  DEEP == false: entry i lives in VGPR lane i
// (select-on-lane push / v_readlane pop, no memory traffic, 64 deep).  DEEP == true: a
// per-wave LDS array of kDeepStack entries for trees deeper than 64 levels (lane 0 writes,
// all lanes read the broadcast word; LDS ops of one wave complete in order).
constexpr int kDeepStack = 1024;
constexpr int kDeepWords = 3;  // node, mask lo, mask hi

template <bool DEEP>
struct WaveStack {
  int node = 0;
  unsigned mlo = 0, mhi = 0;
  int sp = 0;  // wave-uniform
  int* lds = nullptr;
  DIAG(unsigned long long pushes = 0; unsigned long long pops = 0;)

  __device__ __forceinline__ void push(int n, uint64_t m) {
    if (!DEEP) {
      const bool mine = lane_id() == sp;  // v_cmp + v_cndmask: lane sp takes the entry
      node = mine ? n : node;
      mlo = mine ? (unsigned)m : mlo;
      mhi = mine ? (unsigned)(m >> 32) : mhi;
    } else if (lane_id() == 0) {
      lds[kDeepWords * sp] = n;
      lds[kDeepWords * sp + 1] = (int)(unsigned)m;
      lds[kDeepWords * sp + 2] = (int)(unsigned)(m >> 32);
    }
    sp++;
    DIAG(pushes++);
  }
  __device__ __forceinline__ void pop(int& n, uint64_t& m) {
    sp--;
    DIAG(pops++);
    if (!DEEP) {
      n = __builtin_amdgcn_readlane(node, sp);
      m = (uint64_t)(unsigned)__builtin_amdgcn_readlane(mlo, sp) |
          ((uint64_t)(unsigned)__builtin_amdgcn_readlane(mhi, sp) << 32);
    } else {
      n = uniform(lds[kDeepWords * sp]);
      m = (uint64_t)(unsigned)uniform(lds[kDeepWords * sp + 1]) |
          ((uint64_t)(unsigned)uniform(lds[kDeepWords * sp + 2]) << 32);
    }
  }
  // Pop entries until one still has a lane of `alive`; false when the stack runs empty.
  __device__ __forceinline__ bool pop_live(int& n, uint64_t& m, uint64_t alive) {
    for (;;) {
      if (sp == 0) return false;
      pop(n, m);
      m &= alive;
      if (m) return true;
    }
  }
};

__device__ __forceinline__ bool child_box_exact(const DevNode& N, int c, const LaneRay& r) {
  const float b[6] = {N.lo[0][c], N.lo[1][c], N.lo[2][c], N.hi[0][c], N.hi[1][c], N.hi[2][c]};
  return box_exact(b, r);
}

// A leaf's guard that the fast test could not decide: the reference's literal test on the
// holder's box and on every enclosing reference box (the ancestry of BVH.cpp:31-55).
// child: a reference node index, or ~leaf (its holder's box first).
__device__ bool guard_exact(const RenderParams& P, int child, const LaneRay& r) {
  int v = child >= 0 ? child : P.anc[~child].leaf_parent;
  while (v >= 0) {
    if (!box_exact(P.anc[v].box, r)) return false;
    v = P.anc[v].parent;
  }
  return true;
}

// One packet visit of a reference node (RT_TRAVERSAL_REFERENCE, or a scene without culling
// tree), per child: a leaf child is tested by every lane in the node (leaves have no box; the
// slot holds a +-1e30 box that every normalised ray accepts); an inner child's box takes the
// reference's test (fast, else box_exact).  h0/h1: lanes that enter (inner) or test (leaf).
template <bool SKIP>
__device__ __forceinline__ void visit_node(const DevNode& N, const LaneRay& r, bool in, bool& h0,
                                           bool& h1, float& t0, float& t1) {
  const float b0[6] = {N.lo[0][0], N.lo[1][0], N.lo[2][0], N.hi[0][0], N.hi[1][0], N.hi[2][0]};
  const float b1[6] = {N.lo[0][1], N.lo[1][1], N.lo[2][1], N.hi[0][1], N.hi[1][1], N.hi[2][1]};
  float f0, f1;
  slab_span<SKIP>(b0, r, t0, f0);
  slab_span<SKIP>(b1, r, t1, f1);
  bool in0, out0, in1, out1;
  decide_sure(t0, f0, in0, out0);
  decide_sure(t1, f1, in1, out1);
  h0 = in & in0;
  h1 = in & in1;
  const bool u0 = in & !(in0 | out0);
  const bool u1 = in & !(in1 | out1);
  if (ballot(u0 | u1)) {
    if (u0) h0 = child_box_exact(N, 0, r);
    if (u1) h1 = child_box_exact(N, 1, r);
    DIAG(if (u0 | u1) atomicAdd(&g_exact_fallbacks, 1ull));
  }
}

// Pick the next node after a binary visit: near child first (judged by the first lane that
// enters both), the far one pushed; with neither, pop (masks restricted to `alive`).  Returns
// false when the traversal is over.
template <bool DEEP>
__device__ __forceinline__ bool advance(WaveStack<DEEP>& st, int c0, int c1, uint64_t m0,
                                        uint64_t m1, float t0, float t1, int& node, uint64_t& m,
                                        uint64_t alive) {
  if (m0 && m1) {
    const uint64_t both = m0 & m1;
    bool near1 = false;
    if (both) {
      const int f = __builtin_ctzll(both);
      const float f0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t0), f));
      const float f1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t1), f));
      near1 = f1 < f0;
    }
    if (near1) {
      st.push(c0, m0);
      node = c1;
      m = m1;
    } else {
      st.push(c1, m1);
      node = c0;
      m = m0;
    }
    return true;
  }
  if (m0 || m1) {
    node = m0 ? c0 : c1;
    m = m0 ? m0 : m1;
    return true;
  }
  return st.pop_live(node, m, alive);
}

// ------------------------------------------------------------------ batched leaf tests
// A packet reaches a leaf with only the few lanes whose rays pass over that triangle (C3:
// ~14 of 64), so testing leaves one at a time runs the triangle test at ~20% SIMD efficiency.
// The traversal instead queues (lane, leaf) pairs in a per-wave LDS list and runs them 64 at a
// time, one pair per lane (the owner's ray fetched with ds_bpermute, the leaf with a per-lane
// load), once kBatchFlush are pending and when the walk ends.  Results land per ray by LDS
// atomics: closest hit = atomic min of the key (t bits << 32 | DFS leaf), which for 0 < t
// orders exactly like the reference's (t, DFS leaf) rule; shadow = a flag.
// CULL (the culling tree): an entry is a DevLeaf, and its lane first takes the reference's
// decision on the leaf's GUARD box — the fast slab test with the 2^-20 band, which on accept
// implies every enclosing reference box accepts, else guard_exact over the
// ancestry — so exactly the leaves the reference reaches are tested.  Without CULL (reference
// walk) an entry is a DFS leaf whose boxes the walk has already decided.
// The queue is flushed only between visits, once kBatchFlush tests are pending, and holds a whole
// wide visit's pushes (8 slots x 2 leaves x 64 lanes) above that: no flush inside the slot loop.
// (Round 5: the in-loop check inlined the batch test into every slot and held 69 SGPRs in VGPR
// lanes; without it 7 spill and the C3 frame kernel runs 0.406 -> 0.395 ms, four in flight
// 0.385 -> 0.374, profiles/r05/ab_visit_flush.json.  LDS: 22.6 KB per 4-wave workgroup, seven
// workgroups per CU.)
#ifndef RT_BATCH_FLUSH  // (A/B builds)
#define RT_BATCH_FLUSH 128
#endif
constexpr int kBatchFlush = RT_BATCH_FLUSH;
constexpr int kBatchCap = kBatchFlush + kWideSlots * 2 * 64;
constexpr int kShadowFlush = kBatchFlush;

// The primary traversal's queue pushes write every lane: lanes outside the push mask write a
// junk entry past the queue (q[kBatchCap + ...], never read) instead of taking an exec-mask
// branch (the shadow traversal keeps the branch: junk writes cost it VGPR spills).
constexpr int kPushJunk = 128;

// A queue entry is one 32-bit word: the owner lane above kQueueLeafBits, the leaf (DevLeaf or
// DFS index, < 2^26: rt_api.hip refuses larger scenes) below.
constexpr int kQueueLeafBits = 26;
constexpr unsigned kQueueLeafMask = (1u << kQueueLeafBits) - 1u;
struct WaveLeafLds {
  unsigned q[kBatchCap + kPushJunk];  // lane << kQueueLeafBits | leaf
  unsigned long long key[64];       // per lane: closest-hit key, or shadow flag
  int sub;  // the wave's quadrant of a split tile, -1: whole packet (trace_frame_kernel)
};

constexpr unsigned long long kNoHitKey = (0x7f800000ull << 32) | 0xffffffffull;  // (+inf, -1)

// This lane's index computed afresh (asm-opaque), so that it is not kept live (and spilled)
// across a traversal: the shadow phase's light loop.
__device__ __forceinline__ int fresh_lane() {
  int lane;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  return lane;
}

// Queue leaf `leaf` for the lanes of `m` (wave-uniform); n = pending entries (wave-uniform).
// (Round 5: 32-bit entries, and lane_id() left to the compiler instead of an asm-opaque
// recomputation per push: C3 frame 0.3905 -> 0.3802 ms four in flight, profiles/r05/ab_queue32.json.)

template <bool ALL = false>
__device__ __forceinline__ void batch_push(WaveLeafLds& L, int& n, int leaf, uint64_t m) {
  const int lane = lane_id();
  const int below = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
  const unsigned e = ((unsigned)lane << kQueueLeafBits) | (unsigned)leaf;
  if (ALL) {
    L.q[lane_in(m) ? n + below : kBatchCap + lane] = e;
  } else if (lane_in(m)) {
    L.q[n + below] = e;
  }
  n += __builtin_popcountll(m);
}

// Queue leaves `leaf` and `leaf + 1` (a pair) for the lanes of `m`: each lane's two entries are
// adjacent (one ds_write2_b32), the queue order does not matter.
template <bool ALL = false>
__device__ __forceinline__ void batch_push_pair(WaveLeafLds& L, int& n, int leaf, uint64_t m) {
  const int lane = lane_id();
  const int below = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
  const unsigned e = ((unsigned)lane << kQueueLeafBits) | (unsigned)leaf;
  if (ALL) {  // (n may be odd: two 4-B writes, ds_write2_b32)
    const int at = lane_in(m) ? n + 2 * below : kBatchCap + 2 * lane;
    L.q[at] = e;
    L.q[at + 1] = e + 1u;
  } else if (lane_in(m)) {
    L.q[n + 2 * below] = e;
    L.q[n + 2 * below + 1] = e + 1u;
  }
  n += 2 * __builtin_popcountll(m);
}

__device__ __forceinline__ float lane_f(int src, float v) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(v)));
}

typedef float f4 __attribute__((ext_vector_type(4)));

// Runs the n queued tests; SHADOW: 0 < t < thr of the owner sets its flag, else the owner's
// key takes min(key, (t, leaf)) for 0 < t < inf.  All lanes of the wave take part.  SKIP:
// some lane of the wave skips an axis (else the guard test needs no skip flags).
template <bool SHADOW, bool SPHERES, bool CULL, bool SKIP = true>
__device__ __forceinline__ void batch_flush(const RenderParams& P, WaveLeafLds& L, int n,
                                            const LaneRay& r, float thr, Diag& dg) {
  const int lane = lane_id();
  for (int base = 0; base < n; base += 64) {
    const int i = base + lane;
    const bool valid = i < n;
    const unsigned e = valid ? L.q[i] : 0u;
    const int src = (int)(e >> kQueueLeafBits), idx = (int)(e & kQueueLeafMask);
    LaneRay rr;
    rr.o = v3(lane_f(src, r.o.x), lane_f(src, r.o.y), lane_f(src, r.o.z));
    rr.d = v3(lane_f(src, r.d.x), lane_f(src, r.d.y), lane_f(src, r.d.z));
    rr.quot = __builtin_amdgcn_ds_bpermute(src << 2, (int)r.quot) != 0;
    const float othr = SHADOW ? lane_f(src, thr) : 0.0f;
    float t = 0.0f;
    bool hit;
    int leaf;
    if constexpr (CULL) {
      const f4* q = reinterpret_cast<const f4*>(P.leaves + idx);  // idle lanes: record 0, unused
      const f4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
      const int tag = __float_as_int(q0.w);
      leaf = tag & ~kLeafSphere;
      // the guard: the holder box {q1.w, q2.w, q3.x, q3.y, q3.z, q3.w}
      rr.r = v3(__builtin_amdgcn_rcpf(rr.d.x), __builtin_amdgcn_rcpf(rr.d.y),
                __builtin_amdgcn_rcpf(rr.d.z));
      rr.skip0 = SKIP && __builtin_fabsf(rr.d.x) < kEps;
      rr.skip1 = SKIP && __builtin_fabsf(rr.d.y) < kEps;
      rr.skip2 = SKIP && __builtin_fabsf(rr.d.z) < kEps;
      const float g[6] = {q1.w, q2.w, q3.x, q3.y, q3.z, q3.w};
      float tn, tf;
      slab_span<SKIP>(g, rr, tn, tf);
      bool in, out;
      decide_sure(tn, tf, in, out);
      bool ok = valid & in;
      const bool und = valid & !(in | out);
      if (ballot(und)) {
        if (und) ok = guard_exact(P, ~leaf, rr);
        DIAG(if (und) atomicAdd(&g_exact_fallbacks, 1ull));
      }
      DIAG(dg.guard += __builtin_popcountll(ballot(valid)));
      const V3 v0 = v3(q0.x, q0.y, q0.z);
      if (!SPHERES || !(tag & kLeafSphere))
        hit = tri_test(v0, v3(q1.x, q1.y, q1.z), v3(q2.x, q2.y, q2.z), rr, t);
      else
        hit = sphere_test(v0, q1.x, rr, t);
      hit &= ok;
    } else {
      hit = leaf_test<SPHERES>(P.prims, idx, rr, t);  // leaf 0 for idle lanes: unused
      leaf = idx;
    }
    if (SHADOW) {
      if (valid & hit & (t > 0.0f) & (t < othr)) L.key[src] = 1ull;  // any writer: same value
    } else if (valid & hit & (t > 0.0f) & (t < RT_INF)) {
      atomicMin(&L.key[src], ((unsigned long long)__float_as_uint(t) << 32) | (unsigned)leaf);
    }
  }
}

// Queues the leaf tests of a visited reference node's leaf children for the lanes of h0 / h1.
__device__ __forceinline__ void queue_binary_leaves(WaveLeafLds& L, int& pending, const DevNode& N,
                                                    bool h0, bool h1, uint64_t alive, Diag& dg) {
  if (N.child[0] < 0) {
    const uint64_t b = ballot(h0) & alive;
    batch_push(L, pending, ~N.child[0], b);
    DIAG(dg.leaves++; dg.leaf_lanes += __builtin_popcountll(b));
  }
  if (N.child[1] < 0) {
    const uint64_t b = ballot(h1) & alive;
    batch_push(L, pending, ~N.child[1], b);
    DIAG(dg.leaves++; dg.leaf_lanes += __builtin_popcountll(b));
  }
}

// ------------------------------------------------------------------ 8-wide culling nodes
// The whole 128-B node (DevNode8) in one round trip: two s_load_dwordx16 and one wait.
typedef int v16i __attribute__((ext_vector_type(16)));
// `ref` is the tagged node reference: (ref << 6) as 32 bits is the byte offset of its first slot
// (the tag bit falls off the top; the host keeps the node array below 2^26 slots), used as the
// loads' SGPR offset — one shift and one add per visit instead of a 64-bit address.
__device__ __forceinline__ void load_node8(const DevNode* __restrict__ nodes, int ref, v16i& a,
                                           v16i& b) {
  const unsigned off = (unsigned)ref << 6, off2 = off + 64u;
  asm volatile("s_load_dwordx16 %0, %2, %3\n\ts_load_dwordx16 %1, %2, %4\n\ts_waitcnt lgkmcnt(0)"
               : "=&s"(a), "=&s"(b) : "s"(nodes), "s"(off), "s"(off2) : "memory");
}

// fp16 halves of a slot word: the compiler feeds them to v_fma_mix_f32 straight from the SGPR
__device__ __forceinline__ float half_lo(int w) {
  return (float)__builtin_bit_cast(_Float16, (unsigned short)((unsigned)w & 0xffffu));
}
__device__ __forceinline__ float half_hi(int w) {
  return (float)__builtin_bit_cast(_Float16, (unsigned short)((unsigned)w >> 16));
}

#define RT_NODE_WORD(k) ((k) < 16 ? a[(k)] : b[(k) - 16])

// One packet visit of an 8-wide culling node.  Every slot takes a plain slab test on its
// conservative box (plane t = fma(h, 2^k / d, (origin - o) / d), the entry plane moved earlier
// and the exit plane later by the ray's own margin 2^-18 |o| / |d| — DESIGN.md §4.2: with the
// host's margin the test never culls a treelet the reference would enter, so no decision band
// is needed); the valid slots come first and the visit stops at the first invalid one (whose
// NaN planes would fail the test anyway).  A leafy slot's leaves go to the leaf queue (the exact
// guard decision is taken there); of the entered inner slots the first becomes `node` and the
// others are pushed.  `alive`: lanes still searching.  Returns false when the walk is over.
// (Round 5: shadow rays used to enter the nearest slot by the first entering lane's entry
// distance, so occluders would turn up early; the readlane and compare per entered slot cost
// more than it saved — C3 frame kernel 0.397 -> 0.392 ms, four in flight 0.374 -> 0.369 ms,
// profiles/r05/ab_shadow_first.json.  Any-hit: the visiting order does not change the answer.)
// Plane order per lane: a slot word holds the lo plane in its low half and the hi plane in its
// high half; one v_alignbit by the ray's sh (16 where 1/d < 0) puts the lane's ENTRY plane low,
// so a slot costs 3 alignbit + 6 fma_mix + max3 + min3 + 2 compares instead of a min and a max
// per axis on top (same values: the entry plane moved down, the exit plane up by |m|).  A
// skipped axis (SKIP) gets S = 0 and planes -inf / +inf, once per visit.
template <bool SKIP, bool SHADOW, bool DEEP, bool SPHERES>
__device__ __forceinline__ bool visit_wide(const RenderParams& P, const DevNode* __restrict__ nodes,
                                           WaveLeafLds& L, int& pending, const LaneRay& r, int& node,
                                           uint64_t& m, uint64_t alive, WaveStack<DEEP>& st,
                                           Diag& dg) {
  v16i a, b;
  DIAG(const unsigned long long tl0 = clock_now());
  load_node8(nodes, node, a, b);
  DIAG(dg.cyc_load += clock_now() - tl0);
  const unsigned scale = (unsigned)a[3];
  const int inner_base = a[4], leaf_base = a[5], kinds = a[6];
  const unsigned offs = (unsigned)a[7];
  const unsigned inner = (unsigned)kinds & ~((unsigned)kinds >> 8) & 0xffu;
  DIAG(dg.nodes++; dg.wide++; dg.node_lanes += __builtin_popcountll(m));
  const float o[3] = {r.o.x, r.o.y, r.o.z}, rc[3] = {r.r.x, r.r.y, r.r.z}, mg[3] = {r.m.x, r.m.y, r.m.z};
  const int sh[3] = {r.sh0, r.sh1, r.sh2};
  float S[3], Alo[3], Ahi[3];
#pragma unroll
  for (int x = 0; x < 3; x++) {
    S[x] = __builtin_amdgcn_ldexpf(rc[x], (int)(signed char)(scale >> (8 * x)));
    const float A = (__int_as_float(a[x]) - o[x]) * rc[x];
    Alo[x] = A - __builtin_fabsf(mg[x]);  // entry plane earlier
    Ahi[x] = A + __builtin_fabsf(mg[x]);  // exit plane later
    if (SKIP) {  // a skipped axis: every plane at -inf / +inf (fma(h, 0, -+inf), h finite)
      const bool sk = x == 0 ? r.skip0 : (x == 1 ? r.skip1 : r.skip2);
      S[x] = sk ? 0.0f : S[x];
      Alo[x] = sk ? -RT_INF : Alo[x];
      Ahi[x] = sk ? RT_INF : Ahi[x];
    }
  }
  int nxt = -1;
  uint64_t nm = 0;
#pragma unroll
  for (int c = 0; c < kWideSlots; c++) {
    // the valid slots come first (check_accel): stop at the first invalid one (its NaN planes
    // would fail the test anyway)
    if (!(kinds & (kSlotValid << c))) break;
    DIAG(dg.ev[kPhSlotsTested]++);
    float n3[3], f3[3];
#pragma unroll
    for (int x = 0; x < 3; x++) {
      // this lane's entry plane into the low half
      const int w = (int)__builtin_amdgcn_alignbit((unsigned)RT_NODE_WORD(8 + 3 * c + x),
                                                   (unsigned)RT_NODE_WORD(8 + 3 * c + x),
                                                   (unsigned)sh[x]);
      n3[x] = __builtin_fmaf(half_lo(w), S[x], Alo[x]);
      f3[x] = __builtin_fmaf(half_hi(w), S[x], Ahi[x]);
    }
    const float tn = __builtin_fmaxf(__builtin_fmaxf(n3[0], n3[1]), n3[2]);
    const float tf = __builtin_fminf(__builtin_fminf(f3[0], f3[1]), f3[2]);
    // out: !(tf >= max(tn, 0)) — one compare (tn and tf are never NaN on a valid slot: finite
    // fp16 planes, finite scales, skipped axes at -inf / +inf)
    const uint64_t hm = m & alive & ~lanes_nge(tf, __builtin_fmaxf(tn, 0.0f));
    if (!hm) continue;
    DIAG(dg.ev[kPhSlotHits]++);
    if (kinds & (kSlotLeafy << c)) {
      DIAG(dg.ev[kPhLeafyHits]++);
      const int leaf = leaf_base + (int)((offs >> (4 * c)) & 15u);
      const bool pair = (kinds & (kSlotPair << c)) != 0;
      DIAG(dg.ev[kPhPairHits] += pair);
      // (the shadow kernel keeps the exec-mask pushes: junk writes cost it VGPR spills)
#ifdef RT_PRIO_PUSH  // (A/B builds: the leaf pushes at another priority; +0.3 %, in the noise)
      __builtin_amdgcn_s_setprio(RT_PRIO_PUSH);
#endif
      if (pair)
        batch_push_pair<!SHADOW>(L, pending, leaf, hm);
      else
        batch_push<!SHADOW>(L, pending, leaf, hm);
#ifdef RT_PRIO_PUSH
      __builtin_amdgcn_s_setprio(3);  // (RT_PRIO_V)
#endif
      DIAG(dg.leaves += 1 + pair; dg.leaf_lanes += (1 + pair) * __builtin_popcountll(hm));
      continue;
    }
    const int ch = (inner_base + 2 * __builtin_popcount(inner & ((1u << c) - 1u))) | kWideTag;
    DIAG(dg.ev[kPhInnerHits]++);
    if (nxt < 0) {
      nxt = ch;
      nm = hm;
    } else {
      st.push(ch, hm);
    }
  }
  if (nxt >= 0) {
    node = nxt;
    m = nm;
    return true;
  }
  return st.pop_live(node, m, alive);
}
#undef RT_NODE_WORD

// Wave priority (s_setprio) by phase (round 6).  A node visit is the traversal's dependent chain
// — scalar node load -> slot tests -> lane masks -> next node — of short VALU -> SALU -> branch
// steps, each waiting on the one before; the leaf-batch flushes are long runs of independent
// VALU work on loaded records.  With the visits at the highest priority the arbiter issues a
// ready visit instruction first and the flushes (lowest) fill the slots the chains leave idle;
// setup and shading sit between.  Same box, three interleaved rounds
// (profiles/r06/ab_priority*.json): C3 frame kernel 0.390 -> 0.362 ms one frame at a time,
// six in flight 0.352 -> 0.333 ms per frame; the flushes above the visits, or at the visits'
// level, measured slower.  (A/B builds: -DRT_PRIO_V=.. -DRT_PRIO_F=.. -DRT_PRIO_REST=..)
#ifndef RT_PRIO_V
#define RT_PRIO_V 3
#endif
#ifndef RT_PRIO_F
#define RT_PRIO_F 0
#endif
#ifndef RT_PRIO_REST
#define RT_PRIO_REST 1
#endif
#define RT_PRIO_VISIT_BEGIN __builtin_amdgcn_s_setprio(RT_PRIO_V)
#define RT_PRIO_VISIT_END __builtin_amdgcn_s_setprio(RT_PRIO_REST)
#define RT_PRIO_FLUSH_BEGIN __builtin_amdgcn_s_setprio(RT_PRIO_F)
#define RT_PRIO_FLUSH_END __builtin_amdgcn_s_setprio(RT_PRIO_REST)
// ------------------------------------------------------------------ closest hit
// The reference's (t, leaf) for every active ray: leaf < 0 = miss.  FAST: the 8-wide culling
// tree over reference treelets (the launch takes it only when the scene has one); otherwise
// the reference tree itself.
template <bool SKIP, bool FAST, bool DEEP, bool SPHERES>
__device__ __forceinline__ void closest_hit(const RenderParams& P, const DevNode* __restrict__ nodes,
                                            int* spill, WaveLeafLds& L, const LaneRay& r,
                                            bool active, float& best_t, int& best_leaf, Diag& dg) {
  best_t = RT_INF;
  best_leaf = -1;
  if (P.root_kind != kRootNode) {  // the root IS the primitive (BVH.h:13-14): its own rule
    float t;
    if (active && leaf_test<SPHERES>(P.prims, P.root_ref, r, t)) {
      best_t = t;
      best_leaf = P.root_ref;
    }
    return;
  }
  uint64_t m;
  {
    float tn, tf;
    bool acc, und;
    if (FAST) {  // the culling tree's root box (conservative, tested with the band)
      slab_span<SKIP>(P.accel_box, r, tn, tf);
      m = ballot(active && decide_cull(tn, tf));
    } else {
      slab_fast<SKIP>(P.root_box, r, tn, acc, und);
      m = ballot(active && (acc || (und && box_exact(P.root_box, r))));
    }
  }
  if (!m) return;
  const int lane = lane_id();
  WaveStack<DEEP> st;
  st.lds = spill;
  int pending = 0;
  L.key[lane] = kNoHitKey;
  int node = FAST ? P.accel_root : P.root_ref;
  for (;;) {
    if (pending >= kBatchFlush) {  // between visits: only the ray and the stack are live
      DIAG(const unsigned long long tf0 = clock_now());
      RT_PRIO_FLUSH_BEGIN;
      batch_flush<false, SPHERES, FAST, SKIP>(P, L, pending, r, 0.0f, dg);
      RT_PRIO_FLUSH_END;
      DIAG(dg.cyc_flush += clock_now() - tf0; dg.ev[kPhFlushes]++;
           dg.ev[kPhFlushIters] += (pending + 63) / 64);
      pending = 0;
    }
    if constexpr (FAST) {
      DIAG(const unsigned long long tv0 = clock_now(); dg.ev[kPhVisits]++);
      RT_PRIO_VISIT_BEGIN;
      const bool more =
          visit_wide<SKIP, false, DEEP, SPHERES>(P, nodes, L, pending, r, node, m, ~0ull, st, dg);
      RT_PRIO_VISIT_END;
      DIAG(dg.cyc_visit += clock_now() - tv0);
      if (!more) break;
    } else {
      const DevNode N = nodes[node];
      bool h0, h1;
      float t0, t1;
      visit_node<SKIP>(N, r, lane_in(m), h0, h1, t0, t1);
      DIAG(dg.nodes++; dg.node_lanes += __builtin_popcountll(m));
      queue_binary_leaves(L, pending, N, h0, h1, ~0ull, dg);
      // leaves are queued; only inner children are entered
      const uint64_t m0 = N.child[0] >= 0 ? ballot(h0) : 0ull;
      const uint64_t m1 = N.child[1] >= 0 ? ballot(h1) : 0ull;
      if (!advance(st, N.child[0], N.child[1], m0, m1, t0, t1, node, m, ~0ull)) break;
    }
  }
  if (pending) {
    DIAG(const unsigned long long tf0 = clock_now());
    RT_PRIO_FLUSH_BEGIN;
    batch_flush<false, SPHERES, FAST, SKIP>(P, L, pending, r, 0.0f, dg);
    RT_PRIO_FLUSH_END;
    DIAG(dg.cyc_flush += clock_now() - tf0; dg.ev[kPhFlushes]++;
         dg.ev[kPhFlushIters] += (pending + 63) / 64);
  }
  DIAG(dg.ev[kPhPushes] += st.pushes; dg.ev[kPhPops] += st.pops);
  const unsigned long long key = L.key[lane];
  best_t = __uint_as_float((unsigned)(key >> 32));
  best_leaf = (int)(unsigned)key;
}

// ------------------------------------------------------------------ shadow (any hit)
// Occluded iff some leaf the ray may reach has 0 < t < thr — identical to the reference's
// closest-hit shadow test `0 < t_closest < dist - eps` (HW2/Scene.cpp:123-127), appendix A.7.
template <bool SKIP, bool FAST, bool DEEP, bool SPHERES>
__device__ __forceinline__ bool occluded(const RenderParams& P, const DevNode* __restrict__ nodes,
                                         int* spill, WaveLeafLds& L, const LaneRay& r, bool active,
                                         float thr, Diag& dg) {
  if (P.root_kind != kRootNode) {
    float t;
    return active && leaf_test<SPHERES>(P.prims, P.root_ref, r, t) && t < thr && t > 0.0f;
  }
  uint64_t m;
  {
    float tn, tf;
    bool acc, und;
    // thr <= 0 (or NaN): nothing can satisfy 0 < t < thr
    if (FAST) {
      slab_span<SKIP>(P.accel_box, r, tn, tf);
      m = ballot(active && thr > 0.0f && decide_cull(tn, tf));
    } else {
      slab_fast<SKIP>(P.root_box, r, tn, acc, und);
      m = ballot(active && thr > 0.0f && (acc || (und && box_exact(P.root_box, r))));
    }
  }
  if (!m) return false;
  uint64_t alive = m;
  const int lane = lane_id();
  WaveStack<DEEP> st;
  st.lds = spill;
  int pending = 0;
  unsigned long long clear = 0ull;
  asm volatile("" : "+v"(clear));  // a fresh zero here, not one kept (and spilled) across the walk
  L.key[lane] = clear;
  int node = FAST ? P.accel_root : P.root_ref;
  for (;;) {
    if (pending >= kShadowFlush) {  // between visits; a lane found occluded stops entering nodes
      DIAG(const unsigned long long tf0 = clock_now());
      RT_PRIO_FLUSH_BEGIN;
      batch_flush<true, SPHERES, FAST, SKIP>(P, L, pending, r, thr, dg);
      RT_PRIO_FLUSH_END;
      DIAG(dg.cyc_flush += clock_now() - tf0; dg.ev[kPhFlushes]++;
           dg.ev[kPhFlushIters] += (pending + 63) / 64);
      pending = 0;
      alive &= ~ballot(L.key[lane] != 0ull);
      m &= alive;
      if (!m && !st.pop_live(node, m, alive)) break;
    }
    if constexpr (FAST) {
      DIAG(const unsigned long long tv0 = clock_now(); dg.ev[kPhVisits]++);
      RT_PRIO_VISIT_BEGIN;
      const bool more =
          visit_wide<SKIP, true, DEEP, SPHERES>(P, nodes, L, pending, r, node, m, alive, st, dg);
      RT_PRIO_VISIT_END;
      DIAG(dg.cyc_visit += clock_now() - tv0);
      if (!more) break;
    } else {
      const DevNode N = nodes[node];
      bool h0, h1;
      float t0, t1;
      visit_node<SKIP>(N, r, lane_in(m), h0, h1, t0, t1);
      DIAG(dg.nodes++; dg.node_lanes += __builtin_popcountll(m));
      queue_binary_leaves(L, pending, N, h0, h1, alive, dg);  // the still-unoccluded lanes
      const uint64_t m0 = N.child[0] >= 0 ? ballot(h0) & alive : 0ull;
      const uint64_t m1 = N.child[1] >= 0 ? ballot(h1) & alive : 0ull;
      if (!advance(st, N.child[0], N.child[1], m0, m1, t0, t1, node, m, alive)) break;
    }
  }
  if (pending) {
    DIAG(const unsigned long long tf0 = clock_now());
    RT_PRIO_FLUSH_BEGIN;
    batch_flush<true, SPHERES, FAST, SKIP>(P, L, pending, r, thr, dg);
    RT_PRIO_FLUSH_END;
    DIAG(dg.cyc_flush += clock_now() - tf0; dg.ev[kPhFlushes]++;
         dg.ev[kPhFlushIters] += (pending + 63) / 64);
  }
  DIAG(dg.ev[kPhPushes] += st.pushes; dg.ev[kPhPops] += st.pops);
  return L.key[lane] != 0ull;
}

// The kernel's RenderParams (its FIRST argument, so at offset 0 of the kernarg segment) read
// through a pointer the compiler cannot see through: loads from it are not hoisted above this
// point, so the packet code does not pull every field it uses into SGPRs for the whole kernel
// (they were spilled to VGPR lanes across the traversal and reloaded per visit).
typedef __attribute__((address_space(4))) const RenderParams KernargParams;
__device__ __forceinline__ const RenderParams& fresh_params(const RenderParams& P) {
  (void)P;
  KernargParams* p = (KernargParams*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return *(const RenderParams*)p;
}

// ------------------------------------------------------------------ render kernels
// Three phases per packet (trace_frame_kernel): the primary phase finds each pixel's closest
// hit and writes an 8-byte {t, leaf} record; the shadow phase rebuilds the hit point from it
// and traces the point-light shadow rays into occlusion bits; the shading phase runs the
// point-light loop.  Going through the records keeps each phase's live state small
// (occupancy is what hides the dependent node loads).
//
// A packet is normally one wave's 64 lanes = the tile's 8x8 pixels.  A heavy tile can instead
// be split over four waves (sub = 0..3: wave `sub` takes quadrant `sub` of the tile, 4x4 pixels
// in lanes 0..15): fewer rays per wave walk a smaller union of BVH paths, and the
// four quadrants run side by side (kSplitEntries workgroups of kTraceWaves waves).
struct PacketPixel {
  int lane;  // pixel lane: the pixel's index within the tile's 8x8 (its record's slot)
  int px, py;
  bool own;    // this wave lane holds a pixel of the packet (all lanes unless split)
  bool valid;  // ... inside the image
};

// Pixel lane of wave lane `lane` (-1: none, the lanes 16..63 of a quadrant wave).
__device__ __forceinline__ int pixel_lane(int lane, int sub) {
  if (sub < 0) return lane;
  return lane < 16 ? ((sub >> 1) * 4 + (lane >> 2)) * kTile + (sub & 1) * 4 + (lane & 3) : -1;
}

__device__ __forceinline__ PacketPixel packet_pixel(const RenderParams& P, int sel, int sub = -1,
                                                   int lane = lane_id()) {
  PacketPixel q;
  const int pl = pixel_lane(lane, sub);
  q.own = pl >= 0;
  q.lane = q.own ? pl : 0;
  int tx, ty;
  if (P.block_deal) {  // selected block sel / 4, its tile sel % 4
    deal_block_tile(P.tiles_x, P.tile_begin + (sel >> 2) * P.tile_step, sel & 3, tx, ty);
  } else {
    const int tile = P.tile_begin + sel * P.tile_step;
    tx = tile % P.tiles_x;
    ty = tile / P.tiles_x;
  }
  q.px = tx * kTile + (q.lane & 7);
  const int lr = ty * kTile + (q.lane >> 3);  // logical row
  q.valid = q.own && q.px < P.width && lr < P.rows;
  q.py = P.row0 + lr * P.row_stride;
  return q;
}

// This wave's quadrant (-1: the whole packet), kept in the wave's LDS block instead of a
// register across the traversals.
__device__ __forceinline__ int wave_sub(const WaveLeafLds& L) { return uniform(L.sub); }

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

__device__ __forceinline__ float hit_t(int2_t rec) { return __int_as_float(rec.y); }
__device__ __forceinline__ int hit_leaf(int2_t rec) { return rec.x; }

// One wave = the 8x8 packet of selected tile `sel` (< num_sel_tiles): closest hit per pixel
// into its 8-B record.
template <bool FAST, bool DEEP, bool SPHERES>
__device__ __forceinline__ void primary_packet(const RenderParams& P,
                                               const DevNode* __restrict__ nodes, int sel,
                                               int* spill, WaveLeafLds& L) {
  const PacketPixel q = packet_pixel(P, sel, wave_sub(L));
  LaneRay ray = make_ray(ld3(P.cam_e), primary_dir(P, q.px, q.py), P.quot_ok);
  // The camera origin is wave-uniform; left to itself the compiler keeps it in 3 SGPRs and
  // copies it to VGPRs at every node visit (a VALU op takes one SGPR operand, the box
  // coordinate already is one).  Pin it to VGPRs once.
  asm volatile("" : "+v"(ray.o.x), "+v"(ray.o.y), "+v"(ray.o.z));
  const bool any_skip = q.valid && (ray.skip0 || ray.skip1 || ray.skip2);
  Diag dg;
  float t;
  int leaf;
  if (ballot(any_skip))
    closest_hit<true, FAST, DEEP, SPHERES>(P, nodes, spill, L, ray, q.valid, t, leaf, dg);
  else
    closest_hit<false, FAST, DEEP, SPHERES>(P, nodes, spill, L, ray, q.valid, t, leaf, dg);
  const RenderParams& Pw = fresh_params(P);  // post-traversal fields: not live across it
  const PacketPixel qw = packet_pixel(Pw, sel, wave_sub(L));  // (recomputed, not kept)
  int2_t rec;  // key layout: leaf low, t bits high (rt_internal.h)
  rec.x = qw.valid ? leaf : -2;  // -1 miss, -2 outside the image
  rec.y = __float_as_int(t);
  if (qw.own) Pw.hits[(size_t)sel * (kTile * kTile) + qw.lane] = rec;
  const unsigned long long nvalid = __builtin_popcountll(ballot(qw.valid));  // (all lanes)
  const unsigned long long nhit = __builtin_popcountll(ballot(qw.valid && leaf >= 0));
  if (Pw.counters && lane_id() == 0) {  // spread over kCounterSlots rows: no hot address
    unsigned long long* c = counter_row(Pw, sel);
    atomicAdd(&c[kCntPrimary], nvalid);
    atomicAdd(&c[kCntHits], nhit);
#ifdef RT_DIAG
    atomicAdd(&c[kCntPrimNodes], dg.nodes);
    atomicAdd(&c[kCntPrimNodeLanes], dg.node_lanes);
    atomicAdd(&c[kCntPrimLeaves], dg.leaves);
    atomicAdd(&c[kCntPrimLeafLanes], dg.leaf_lanes);
    atomicAdd(&c[kCntPrimWide], dg.wide);
    atomicAdd(&c[kCntGuardTests], dg.guard);
    for (int k = 0; k < kPhaseEvents; k++) atomicAdd(&g_phase[k], dg.ev[k]);
    atomicAdd(&g_phase[kPhCycPrimVisit], dg.cyc_visit);
    atomicAdd(&g_phase[kPhCycPrimLoad], dg.cyc_load);
    atomicAdd(&g_phase[kPhCycPrimFlush], dg.cyc_flush);
#endif
  }
}

// Hit point and normal of a primary hit, rebuilt from its {t, leaf} record exactly as
// trace_ray computes them (HW2/Scene.cpp:101-105; Sphere.h:42,50 for sphere normals).
__device__ __forceinline__ V3 hit_point(const RenderParams& P, const PacketPixel& q, float t) {
  return ld3(P.cam_e) + primary_dir(P, q.px, q.py) * t;  // Ray::point_at = o + t*d
}

// Shadow rays of HW2/Scene.cpp:113-127: one bit per point light, set when the light is
// occluded for this pixel's primary hit.
template <bool FAST, bool DEEP, bool SPHERES>
__device__ __forceinline__ void shadow_packet(const RenderParams& P0,
                                              const DevNode* __restrict__ nodes,
                                              const DevLight* __restrict__ lights, int sel,
                                              int* spill, WaveLeafLds& L) {
  Diag dg;
  for (int w = 0; w < P0.occ_words; w++) {
    unsigned bits = 0;
    const int lend = min(P0.num_lights, 32 * (w + 1));
    for (int li = 32 * w; li < lend; li++) {
      // per light: the pixel's hit record is re-read and its hit point rebuilt, so nothing but
      // the occlusion bits is live across the traversal (register pressure, not traffic: the
      // 8-B record is an L2 hit)
      const RenderParams& P = fresh_params(P0);
      const DevLight& lt = lights[li];
      // the packet's pixel indices recomputed here, not hoisted out of the light loop (where
      // they would be live across the traversal and spilled to scratch)
      int sel_l = sel;
      asm volatile("" : "+s"(sel_l));
      const int lane_l = fresh_lane();
      const PacketPixel q = packet_pixel(P, sel_l, wave_sub(L), lane_l);
      const int2_t rec = P.hits[(size_t)sel_l * (kTile * kTile) + q.lane];
      const bool hit = q.own && hit_leaf(rec) >= 0;
      const V3 pk = hit ? hit_point(P, q, hit_t(rec)) : v3(0, 0, 0);
      const V3 ld = ld3(lt.position) - pk;
      const V3 wi = normalize(ld);
      const float dist = length(ld);
      const LaneRay sr = make_ray(pk + wi * P.eps, wi, P.quot_ok);  // p + eps * w_i
      const float thr = dist - P.eps;
      const bool any_skip = hit && (sr.skip0 || sr.skip1 || sr.skip2);
      const bool occ = ballot(any_skip)
                           ? occluded<true, FAST, DEEP, SPHERES>(P, nodes, spill, L, sr, hit, thr, dg)
                           : occluded<false, FAST, DEEP, SPHERES>(P, nodes, spill, L, sr, hit, thr, dg);
      bits |= (occ ? 1u : 0u) << (li - 32 * w);
    }
    const RenderParams& Pw = fresh_params(P0);
    int sel_w = sel;
    asm volatile("" : "+s"(sel_w));
    const int pl = pixel_lane(fresh_lane(), wave_sub(L));
    if (pl >= 0) Pw.occ[((size_t)sel_w * (kTile * kTile) + pl) * Pw.occ_words + w] = bits;
  }
  const RenderParams& Pc = fresh_params(P0);
  if (Pc.counters) {
    const int pl = pixel_lane(lane_id(), wave_sub(L));
    const bool hit = pl >= 0 && hit_leaf(Pc.hits[(size_t)sel * (kTile * kTile) + pl]) >= 0;
    const unsigned long long nhit = __builtin_popcountll(ballot(hit));
    if (lane_id() == 0) {
      unsigned long long* c = counter_row(Pc, sel);
      atomicAdd(&c[kCntShadow], nhit * (unsigned long long)Pc.num_lights);
#ifdef RT_DIAG
      atomicAdd(&c[kCntShadNodes], dg.nodes);
      atomicAdd(&c[kCntShadNodeLanes], dg.node_lanes);
      atomicAdd(&c[kCntShadLeaves], dg.leaves);
      atomicAdd(&c[kCntShadLeafLanes], dg.leaf_lanes);
      atomicAdd(&c[kCntShadWide], dg.wide);
      atomicAdd(&c[kCntGuardTests], dg.guard);
      for (int k = 0; k < kPhaseEvents; k++) atomicAdd(&g_phase[kPhaseEvents + k], dg.ev[k]);
      atomicAdd(&g_phase[kPhCycShadVisit], dg.cyc_visit);
      atomicAdd(&g_phase[kPhCycShadLoad], dg.cyc_load);
      atomicAdd(&g_phase[kPhCycShadFlush], dg.cyc_flush);
#endif
    }
  }
}

// Local shading of HW2/Scene.cpp:101-138 given the occlusion bits, in the reference's
// accumulation order: ambient, then per light diffuse then specular.  No traversal here, so
// the fp64 pow (HW2 calls ::pow(double, double)) costs no occupancy in the traversal kernels.
// The leaf's normal and material come in one 16-B load (normals[4 * leaf + 3] holds the
// material index); the DevPrim record is read only in scenes with spheres (its kind).
// (float)pow((double)c, (double)p) of HW2/Scene.cpp:133-137.  p == 1 returns c itself: the exact
// result is the double c, and both glibc's pow (< 0.52 ulp) and ocml's (< 1 ulp) return an exact
// result when one exists, so the reference gets c too.  Any other exponent takes the fp64 pow.
// Out of line: inlined, ocml's fp64 pow needs ~60 VGPRs and set the register budget of every
// kernel that shades (the fused frame kernel spilled to scratch around it).
__device__ __attribute__((noinline)) float phong_pow_f64(float c, float p) {
  return (float)pow((double)c, (double)p);
}
__device__ __forceinline__ float phong_pow(float c, float p) {
  if (p == 1.0f) return c;
  return phong_pow_f64(c, p);
}

// The colour of a primary hit (leaf, t) of pixel (px, py): ambient, then per unoccluded light
// diffuse and specular, in the reference's order.  occluded(li): light li's shadow bit.
template <bool SPHERES, typename Occ>
__device__ __forceinline__ V3 shade_hit(const RenderParams& P, const DevPrim* __restrict__ prims,
                                        const float* __restrict__ normals,
                                        const DevMaterial* __restrict__ mats,
                                        const DevLight* __restrict__ lights, int leaf, V3 p,
                                        Occ occluded) {
  V3 color = v3(0.0f, 0.0f, 0.0f);
  const V3 e = ld3(P.cam_e);
  const float4 nm = *reinterpret_cast<const float4*>(normals + 4 * leaf);
  const bool tri = !SPHERES || prims[leaf].kind == kPrimTriangle;
  const V3 n = tri ? v3(nm.x, nm.y, nm.z) : normalize(p - ld3(prims[leaf].v0));
  const DevMaterial& m = mats[__float_as_int(nm.w)];
  const V3 w0 = normalize(e - p);  // (ray.o - intersection_point).normalize()
  color = color + ld3(m.ambient) * ld3(P.ambient);
  for (int li = 0; li < P.num_lights; li++) {
    if (occluded(li)) continue;
    const DevLight& Lt = lights[li];
    const V3 ld = ld3(Lt.position) - p;
    const V3 wi = normalize(ld);
    const float dist = length(ld);
    const V3 I = ld3(Lt.intensity);
    const float d2 = dist * dist;
    const float cos_d = dot(n, wi);
    color = color + ((ld3(m.diffuse) * I) * cos_d) / d2;
    const float cos_s = __builtin_fmaxf(dot(n, normalize(w0 + wi)), 0.0f);
    const float pw = phong_pow(cos_s, m.phong_exponent);
    color = color + ((ld3(m.specular) * I) * pw) / d2;
  }
  return color;
}

template <bool SPHERES>
__device__ __forceinline__ void shade_pixel(const RenderParams& P,
                                            const DevPrim* __restrict__ prims,
                                            const float* __restrict__ normals,
                                            const DevMaterial* __restrict__ mats,
                                            const DevLight* __restrict__ lights, int sel,
                                            int sub, float* stage = nullptr) {
  const PacketPixel q = packet_pixel(P, sel, sub);
  const size_t pix = (size_t)sel * (kTile * kTile) + q.lane;
  const int2_t rec = P.hits[pix];
  const bool valid = q.own && hit_leaf(rec) != -2;
  const bool hit = q.own && hit_leaf(rec) >= 0;
  if (P.records) {  // RT_TILE_RECORDS: the pixel record instead of its colour (rt_resolve_*)
    if (!q.own || (!P.tile_major && !valid)) return;
    unsigned r = kRecOutside;
    if (hit)
      r = (unsigned)hit_leaf(rec) | ((P.occ[pix * P.occ_words] & kRecLightMask) << kRecLightShift);
    else if (valid)
      r = kRecMiss;
    unsigned* o = reinterpret_cast<unsigned*>(P.out);
    o[P.tile_major ? pix : (size_t)q.py * P.width + q.px] = r;  // tile-major, or row-major
    return;
  }
  V3 color = v3(0.0f, 0.0f, 0.0f);
  if (hit) {
    const unsigned* occ = P.occ + pix * P.occ_words;
    color = shade_hit<SPHERES>(P, prims, normals, mats, lights, hit_leaf(rec),
                               hit_point(P, q, hit_t(rec)),
                               [&](int li) { return ((occ[li >> 5] >> (li & 31)) & 1u) != 0; });
  } else if (valid) {
    color = ld3(P.background);  // primary miss: max_recursion_depth == depth
  }
  if (valid && stage) {  // pair_rows: the colour waits in LDS for the workgroup's row writes
    stage[3 * q.lane] = 0.0f + color.x;
    stage[3 * q.lane + 1] = 0.0f + color.y;
    stage[3 * q.lane + 2] = 0.0f + color.z;
  } else if (valid) {
    float* o;
    if (P.tile_major)
      o = P.out + 3 * pix;
    else
      o = P.out + 3 * ((size_t)q.py * P.width + q.px);
    o[0] = 0.0f + color.x;  // Pixel::add_color(color, 1) onto a zeroed pixel
    o[1] = 0.0f + color.y;
    o[2] = 0.0f + color.z;
  } else if (P.tile_major && q.own) {
    float* o = P.out + 3 * pix;
    o[0] = o[1] = o[2] = 0.0f;
  }
}

// pair_rows (rt_render into pinned host memory): the frame kernel's stores cross PCIe, where a
// wave's 8 rows of 96 B each end in a half-filled 64-B line.  The workgroup's two tiles (a 2x1
// unit, tx even) instead leave their colours in their waves' LDS; the second wave to arrive
// writes both tiles as 8 rows of 192 B — whole 64-B lines, 16-B stores.  (Same values, same
// pixels: only who stores them changes.)
__device__ __forceinline__ void pair_write(const RenderParams& P, WaveLeafLds* lds, int sel,
                                           int* arrived) {
  __threadfence_block();  // this wave's staged colours before its arrival
  int first = 0;
  if (lane_id() == 0) first = atomicAdd(arrived, 1) == 0;
  if (__builtin_amdgcn_readfirstlane(first)) return;  // the partner writes both tiles
  __threadfence_block();
  const int w = (int)threadIdx.x >> 6;
  const int tile = P.tile_begin + sel - w;  // the unit's left tile
  const int tx0 = tile % P.tiles_x, ty = tile / P.tiles_x;
  for (int f = lane_id(); f < 96; f += 64) {  // 8 rows x 12 float4
    const int r = f / 12, k = f % 12;
    const int lr = ty * kTile + r;
    if (lr >= P.rows) continue;
    const float* src = reinterpret_cast<const float*>(lds[k / 6].q) + r * 24 + (k % 6) * 4;
    const size_t y = (size_t)(P.row0 + lr * P.row_stride);
    float4* dst = reinterpret_cast<float4*>(P.out + 3 * (y * P.width + (size_t)tx0 * kTile) + 4 * k);
    *dst = make_float4(src[0], src[1], src[2], src[3]);
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
    const LaneRay sr = make_ray(p + wi * P.eps, wi, P.quot_ok);
    const float thr = dist - P.eps;
    const bool sskip = ballot(shade && (sr.skip0 || sr.skip1 || sr.skip2)) != 0;
    const bool occ = sskip ? occluded<true, FAST, DEEP, SPHERES>(P, nodes, spill, L, sr, shade, thr, dg)
                           : occluded<false, FAST, DEEP, SPHERES>(P, nodes, spill, L, sr, shade, thr, dg);
    shadow_rays += __builtin_popcountll(ballot(shade));
    if (shade && !occ) {
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
    const LaneRay ray = make_ray(ro, rd, P.quot_ok);
    const bool skip = ballot(active && (ray.skip0 || ray.skip1 || ray.skip2)) != 0;
    float t;
    int leaf;
    if (skip)
      closest_hit<true, FAST, DEEP, SPHERES>(P, nodes, spill, L, ray, active, t, leaf, dg);
    else
      closest_hit<false, FAST, DEEP, SPHERES>(P, nodes, spill, L, ray, active, t, leaf, dg);
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

// The frame kernel hides its dependent node loads with occupancy: 7 waves/SIMD (<= 72 VGPRs),
// where the wide node's 32 SGPRs and the fp32 traversal state fit without scratch (at 8 the
// traversal spills).  (Macro: A/B builds, `make exp EXTRA=-D...`.)
#ifndef RT_FRAME_MIN_WAVES
#define RT_FRAME_MIN_WAVES 7
#endif
#define RT_FRAME_OCCUPANCY __attribute__((amdgpu_waves_per_eu(RT_FRAME_MIN_WAVES, 8)))

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
// rays walk the same nodes, and the cache serves them once.
constexpr int kBlockW = kTraceWaves >= 2 ? 2 : 1, kBlockH = kTraceWaves / kBlockW;

// Tile (= sel, tile_step 1) of logical packet p; -1 for a padding packet of an edge block.
__device__ __forceinline__ int packet_sel(const RenderParams& P, int p) {
  if (!P.tile_block) return p;
  const int w = p % kTraceWaves, b = p / kTraceWaves;
  const int nbx = (P.tiles_x + kBlockW - 1) / kBlockW;
  const int tx = (b % nbx) * kBlockW + w % kBlockW, ty = (b / nbx) * kBlockH + w / kBlockW;
  const int tiles_y = P.num_sel_tiles / P.tiles_x;  // the selection's tile rows
  return (tx < P.tiles_x && ty < tiles_y) ? ty * P.tiles_x + tx : -1;
}

// Logical packets of a traversal launch (with tile_block, padded to whole blocks).
__host__ __device__ __forceinline__ int trace_packets(const RenderParams& P) {
  if (!P.tile_block) return P.num_sel_tiles;
  const int tiles_y = P.num_sel_tiles / P.tiles_x;
  return ((P.tiles_x + kBlockW - 1) / kBlockW) * ((tiles_y + kBlockH - 1) / kBlockH) * kTraceWaves;
}

// ------------------------------------------------------------------ dispatch order
// Traversal kernels are LPT-scheduled: a packet's cost varies ~5x over a C3 frame (rays that
// graze the height field walk far more nodes), and a kernel's tail is set by the heavy packets
// that start last.  The hardware dispatcher hands out workgroups in block order as slots free
// up, so launching the units (one workgroup's kTraceWaves packets) heaviest first is a
// longest-processing-time schedule.  Orders never change results: every tile is written by
// exactly one wave.
//
// Unit u = the kTraceWaves packets of logical packets u*kTraceWaves .. (a 2x2 tile block in
// tile_block mode).  Wave w's selected tile, or -1.
__device__ __forceinline__ int unit_sel(const RenderParams& P, int unit, int w) {
  const int p = unit * kTraceWaves + w;
  if (p >= trace_packets(P)) return -1;
  const int sel = packet_sel(P, p);
  return sel < P.num_sel_tiles ? sel : -1;
}

// Selected tile of this wave in a traversal launch, and its quadrant (sub, -1: the whole
// packet): ordered (block b of the grid takes entry b / regions of region b mod regions' list,
// heaviest first: a unit, -1 = none, or -2 - (p kSplitEntries + j) = quadrants j kTraceWaves ..
// of logical packet p's tile, wave k taking quadrant j kTraceWaves + k), else the XCD-remapped
// block order.
__device__ __forceinline__ int order_entry(const RenderParams& Q) {
  const int b = (int)blockIdx.x;
  return uniform(Q.unit_order[(b % Q.order_regions) * Q.order_stride + b / Q.order_regions]);
}

__device__ __forceinline__ int dispatch_sel(const RenderParams& Q) {
  const int w = (int)threadIdx.x >> 6;
  if (Q.use_order) {
    const int e = order_entry(Q);
    if (e >= 0) return uniform(unit_sel(Q, e, w));
    if (e == -1) return -1;
    const int p = (-2 - e) / kSplitEntries;  // the split tile's logical packet
    return uniform(unit_sel(Q, p / kTraceWaves, p % kTraceWaves));
  }
  const int p = packet_index<kTraceWaves>();
  const int sel = p < trace_packets(Q) ? packet_sel(Q, p) : -1;
  return sel < Q.num_sel_tiles ? sel : -1;
}

// Units of region x: chunks c = x, x + regions, ... of order_chunk consecutive units.
__device__ __forceinline__ int region_units(const RenderParams& P, int x) {
  const int full = P.order_units / P.order_chunk, rem = P.order_units % P.order_chunk;
  int n = x < full ? ((full - 1 - x) / P.order_regions + 1) * P.order_chunk : 0;
  if (rem && full % P.order_regions == x) n += rem;
  return n;
}
__device__ __forceinline__ int region_unit(const RenderParams& P, int x, int i) {
  return (x + (i / P.order_chunk) * P.order_regions) * P.order_chunk + i % P.order_chunk;
}

constexpr int kOrderBuckets = 256;
__device__ __forceinline__ int cost_bucket(unsigned c) {  // 8 steps per octave
  c = c ? c : 1u;
  const int msb = 31 - __builtin_clz(c);
  const int frac = msb >= 3 ? (int)((c >> (msb - 3)) & 7u) : (int)((c << (3 - msb)) & 7u);
  return min(kOrderBuckets - 1, msb * 8 + frac);
}

// A unit holds its workgroup slot until its slowest packet ends, so it is ranked by its
// most expensive tile (ranking by the sum measured 14 % worse in a replay of measured
// per-tile times).
__device__ __forceinline__ unsigned unit_cost(const RenderParams& P, int u) {
  unsigned c = 0;
  for (int w = 0; w < kTraceWaves; w++) {
    const int sel = unit_sel(P, u, w);
    if (sel >= 0) c = max(c, P.tile_cost[sel]);
  }
  return c;
}

// One workgroup per region: a bucket sort of the region's units by cost, heaviest first (order
// inside a bucket is free), into unit_order[x * stride ..]; -1 pads the list to `stride`.
// 256 threads: with frames in flight the GPU is full of traversal waves, and a bigger workgroup
// waits for a CU with that many free wave slots (rocprof: 1024-thread order launches averaged
// 79 us, up to 373, beside other frames' traversal; the sort itself takes 8 us).
//
// Split: the heaviest units — at most order_split per region, each costing at
// least kSplitBuckets buckets (2^(kSplitBuckets/8)) above the region's median — are listed as
// kSplitEntries entries per tile, so each of their tiles gets kSplitEntries workgroups whose
// waves take one quadrant each.  Those tiles' costs are zeroed here: the next frame's quadrant waves
// add their times into them (the tile's cost = the sum of its quadrants).
constexpr int kOrderThreads = 256;
// Split tuning (A/B builds): threshold in buckets above the median (8 per octave: 11 = 2.6 x),
// tiles split per region at most (1 / RT_SPLIT_DIV of the region's tiles, at most kMaxSplit), and
// only in launches whose regions hold at most RT_SPLIT_MAX_TILES tiles (the shares of a frame
// split over GPUs: a whole frame's tail is already hidden by the frames in flight, and splitting
// adds work).  Counted in tiles, so the split covers the same share whatever the workgroup size.
#ifndef RT_SPLIT_BUCKETS
#define RT_SPLIT_BUCKETS 11
#endif
#ifndef RT_SPLIT_DIV
#define RT_SPLIT_DIV 16
#endif
#ifndef RT_SPLIT_MAX_TILES
#define RT_SPLIT_MAX_TILES 768
#endif
constexpr int kSplitBuckets = RT_SPLIT_BUCKETS;
constexpr int kMaxSplit = 128;  // tiles split per region at most
__global__ __launch_bounds__(kOrderThreads) void order_kernel(RenderParams P) {
  __shared__ int hist[kOrderBuckets];
  __shared__ int split_info[2];  // [0] = split threshold bucket, [1] = units split
  const int tid = (int)threadIdx.x, x = (int)blockIdx.x;
  const int n = region_units(P, x);
  int* out = P.unit_order + (size_t)x * P.order_stride;
  for (int i = tid; i < kOrderBuckets; i += kOrderThreads) hist[i] = 0;
  __syncthreads();
  for (int i = tid; i < n; i += kOrderThreads)
    atomicAdd(&hist[cost_bucket(unit_cost(P, region_unit(P, x, i)))], 1);
  __syncthreads();
  if (tid < 64) {  // exclusive offsets, heaviest bucket first: one wave scans the 256 buckets
    const int lane = tid;
    int v[kOrderBuckets / 64], run = 0;
#pragma unroll
    for (int k = 0; k < kOrderBuckets / 64; k++) {
      v[k] = hist[kOrderBuckets - 1 - (lane * (kOrderBuckets / 64) + k)];
      run += v[k];
    }
    int x2 = run;  // inclusive scan of the lane totals
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x2, o, 64);
      if (lane >= o) x2 += y;
    }
    int base = x2 - run;
    // the median unit's bucket (heaviest first: where the running count passes n / 2), and
    // how many units lie kSplitBuckets or more above it
    int med = -1;
#pragma unroll
    for (int k = 0; k < kOrderBuckets / 64; k++) {
      const int bucket = kOrderBuckets - 1 - (lane * (kOrderBuckets / 64) + k);
      if (base <= n / 2 && n / 2 < base + v[k]) med = bucket;
      hist[bucket] = base;
      base += v[k];
    }
    const uint64_t has = ballot(med >= 0);
    if (has) {
      const int mb = __builtin_amdgcn_readlane(med, (int)__builtin_ctzll(has));
      const int thr = mb + kSplitBuckets;
      if (lane == 0) {
        // hist[] now holds each bucket's first rank: units in buckets >= thr have ranks
        // below hist[thr - 1]'s ... i.e. the first rank of the next lighter bucket
        const int heavy = thr > kOrderBuckets - 1 ? 0 : hist[thr - 1];
        split_info[0] = thr;
        split_info[1] = min(P.order_split, heavy);
      }
    } else if (lane == 0) {
      split_info[0] = kOrderBuckets;
      split_info[1] = 0;
    }
  }
  __syncthreads();
  const int nsplit = split_info[1];
  unsigned* snap = P.tile_cost + sched_snap_offset((unsigned long long)P.num_sel_tiles);
  for (int i = tid; i < n; i += kOrderThreads) {
    const int u = region_unit(P, x, i);
    for (int w = 0; w < kTraceWaves; w++) {  // this frame's costs, kept for rt_tile_costs
      const int sel = unit_sel(P, u, w);
      if (sel >= 0) snap[sel] = P.tile_cost[sel];
    }
    const int r = atomicAdd(&hist[cost_bucket(unit_cost(P, u))], 1);
    if (r < nsplit) {  // kSplitEntries entries per tile, -1 for a padding tile of an edge block
      for (int w = 0; w < kTraceWaves; w++) {
        const int sel = unit_sel(P, u, w);
        for (int j = 0; j < kSplitEntries; j++)
          out[kQuadrants * r + kSplitEntries * w + j] =
              sel >= 0 ? -2 - ((kTraceWaves * u + w) * kSplitEntries + j) : -1;
        if (sel >= 0) P.tile_cost[sel] = 0u;
      }
    } else {
      out[r + (kQuadrants - 1) * nsplit] = u;
    }
  }
  for (int i = n + (kQuadrants - 1) * nsplit + tid; i < P.order_stride; i += kOrderThreads)
    out[i] = -1;
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
      g_timeline[k][wid][2] = (unsigned)tl_sel;                                           \
    }                                                                                     \
  } while (0)
#else
#define TL_BEGIN
#define TL_SEL(x)
#define TL_END(k)
#endif

// One launch per frame: each wave runs its packet's primary traversal, its shadow rays and its
// shading back to back, so a frame is one kernel with one tail (round 4 chained primary ->
// order -> shadow -> shade kernels, each with its own tail: a 1/8 share of a C3 frame then took
// 0.16 ms one at a time).  The hit record and occlusion bits still go through the
// stream's scratch (the same lane writes, then reads them: program order), which keeps the
// register state of the three phases apart.  tile_cost: the whole packet's time.
template <bool FAST, bool DEEP, bool SPHERES>
__global__ __launch_bounds__(kTraceWaves * 64) RT_FRAME_OCCUPANCY void trace_frame_kernel(
    RenderParams P, const DevNode* __restrict__ nodes, const DevLight* __restrict__ lights) {
  extern __shared__ __attribute__((aligned(16))) int deep_stack[];
  __shared__ WaveLeafLds leaf_lds[kTraceWaves];
  int* spill = DEEP ? deep_stack + ((int)threadIdx.x >> 6) * kDeepWords * kDeepStack : nullptr;
  WaveLeafLds& L = leaf_lds[threadIdx.x >> 6];
  __shared__ int pair_arrived;
  if (P.pair_rows) {
    if (threadIdx.x == 0) pair_arrived = 0;
    __syncthreads();
  }
  TL_BEGIN;
  const RenderParams& Q = fresh_params(P);
  const int sel = dispatch_sel(Q);
  TL_SEL(sel);
  if (sel >= 0) {
    const int e = Q.use_order ? order_entry(Q) : -1;
    L.sub = e <= -2 ? ((-2 - e) % kSplitEntries) * kTraceWaves + ((int)threadIdx.x >> 6) : -1;
    // the packet's start time waits in LDS (kept in SGPRs across the traversals it spilled)
    __shared__ unsigned long long start[kTraceWaves];
    start[threadIdx.x >> 6] = __builtin_amdgcn_s_memrealtime();
    DIAG(const unsigned long long c0 = clock_now());
    primary_packet<FAST, DEEP, SPHERES>(Q, nodes, sel, spill, L);
    DIAG(const unsigned long long c1 = clock_now());
    if (fresh_params(P).num_lights > 0)
      shadow_packet<FAST, DEEP, SPHERES>(fresh_params(P), nodes, lights, sel, spill, L);
    DIAG(const unsigned long long c2 = clock_now());
    const RenderParams& Ps = fresh_params(P);
    if (Ps.pair_rows) {
      shade_pixel<SPHERES>(Ps, Ps.prims, Ps.normals, Ps.materials, lights, sel, -1,
                           reinterpret_cast<float*>(L.q));
      pair_write(fresh_params(P), leaf_lds, sel, &pair_arrived);
    } else {
      shade_pixel<SPHERES>(Ps, Ps.prims, Ps.normals, Ps.materials, lights, sel, wave_sub(L));
    }
#ifdef RT_DIAG
    const unsigned long long c3 = clock_now();
    if (lane_id() == 0) {
      atomicAdd(&g_phase[kPhCycPrimTotal], c1 - c0);
      atomicAdd(&g_phase[kPhCycShadTotal], c2 - c1);
      atomicAdd(&g_phase[kPhCycShade], c3 - c2);
      atomicAdd(&g_phase[kPhCycFrame], c3 - c0);
      atomicAdd(&g_phase[kPhWaves], 1ull);
    }
#endif
    const RenderParams& Pw = fresh_params(P);
    if (Pw.tile_cost && lane_id() == 0) {  // the next frame's dispatch order
      const unsigned c = (unsigned)min(__builtin_amdgcn_s_memrealtime() - start[threadIdx.x >> 6],
                                       0xffffffffull);
      if (wave_sub(L) < 0)
        Pw.tile_cost[sel] = c;
      else  // a quadrant: the tile's cost is the sum of its quadrants' (zeroed by order_kernel)
        atomicAdd(&Pw.tile_cost[sel], c);
    }
  }
  TL_END(0);
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
  int* spill = DEEP ? deep_stack + ((int)threadIdx.x >> 6) * kDeepWords * kDeepStack : nullptr;
  recursive_packet<FAST, DEEP, SPHERES>(P, nodes, prims, normals, mats, lights, sel, spill,
                                        leaf_lds[threadIdx.x >> 6]);
}

// marks (nullable): 4 events recorded before the frame kernel (or the recursive kernel), after
// it, after the order kernel and at the end (rt_set_kernel_timing).
static inline void mark(const hipEvent_t* marks, int k, hipStream_t stream) {
  if (marks) (void)hipEventRecord(marks[k], stream);
}

// Dispatch-order geometry of a traversal launch: units of one traversal
// workgroup, `regions` regions of `chunk`-unit chunks (tile_block: half a row of 2x1 blocks), LPT
// within each region.  Sets T's tile_block and order_* fields, the launch's unit count (tblocks)
// and the units per region; false: the launch runs in block order (no order kernel).
#ifndef RT_ORDER_MIN_TILES  // launches selecting fewer tiles run in block order (no order kernel)
#define RT_ORDER_MIN_TILES 0
#endif
#ifndef RT_ORDER_SPLIT  // (A/B builds: 0 = no heavy-tile split)
#define RT_ORDER_SPLIT 1
#endif
static bool order_geometry(RenderParams& T, int& tblocks, int& per_region) {
  // 2-D blocks of tiles for a selection of whole tile rows: the whole frame, or a row band
  // (dist_tiles.BandPlan: tiles tile_begin .. tile_begin + num_sel_tiles - 1)
  T.tile_block = T.tile_step == 1 && !T.block_deal && T.tile_begin % T.tiles_x == 0 &&
                 T.num_sel_tiles % T.tiles_x == 0;
  tblocks = (trace_packets(T) + kTraceWaves - 1) / kTraceWaves;
  per_region = 0;
  T.use_order = 0;
  if (!(T.tile_cost != nullptr && T.unit_order != nullptr && T.order_regions > 0 &&
        T.num_sel_tiles >= RT_ORDER_MIN_TILES))
    return false;
  T.order_units = tblocks;
  const int nbx = (T.tiles_x + kBlockW - 1) / kBlockW;
  if (T.order_chunk > 0)  // host-set: that many chunks per region
    T.order_chunk = max(1, (tblocks + T.order_regions * T.order_chunk - 1) / (T.order_regions * T.order_chunk));
  else
    T.order_chunk = T.tile_block ? max(1, (nbx + 1) / 2) : 64;
  const int chunks = (T.order_units + T.order_chunk - 1) / T.order_chunk;
  per_region = ((chunks + T.order_regions - 1) / T.order_regions) * T.order_chunk;
  // room for order_split units per region listed quadrant group by quadrant group
  const int region_tiles = per_region * kTraceWaves;
  T.order_split = RT_ORDER_SPLIT && region_tiles <= RT_SPLIT_MAX_TILES
                      ? max(1, min(kMaxSplit, region_tiles / RT_SPLIT_DIV) / kTraceWaves) : 0;
  T.order_stride = per_region + (kQuadrants - 1) * T.order_split;
  return (unsigned long long)T.num_sel_tiles + (unsigned long long)T.order_regions * T.order_stride <=
         sched_snap_offset((unsigned long long)T.num_sel_tiles);
}

// The cold order of a camera's whole frame (rt_api.hip seed_cold_orders): P's tile_cost holds
// the estimated tile costs; the order kernel lists the units heaviest first into P's
// unit_order, without split entries.  Returns 1 if the launch is ordered (a list was made).
int launch_cold_order(RenderParams P, hipStream_t stream) {
  int tblocks = 0, per_region = 0;
  if (P.num_sel_tiles <= 0 || !order_geometry(P, tblocks, per_region)) return 0;
  P.order_split = 0;
  P.order_stride = per_region;
  hipLaunchKernelGGL(order_kernel, dim3(P.order_regions), dim3(kOrderThreads), 0, stream, P);
  return hipGetLastError() == hipSuccess ? 1 : 0;
}

template <bool FAST, bool DEEP, bool SPHERES>
static void launch_variant(const RenderParams& P, const DevNode* nodes, const DevPrim* prims,
                           const float* normals, const DevMaterial* mats,
                           const DevLight* lights, int blocks, const hipEvent_t* marks,
                           hipStream_t stream) {
  if (P.frames) {  // recursive scenes: one kernel walks each pixel's ray tree
    const size_t lds = DEEP ? sizeof(int) * kDeepWords * kDeepStack * kWavesPerBlock : 0;
    mark(marks, 0, stream);
    hipLaunchKernelGGL((recursive_kernel<FAST, DEEP, SPHERES>), dim3(blocks),
                       dim3(kWavesPerBlock * 64), lds, stream, P, nodes, prims, normals, mats,
                       lights);
    mark(marks, 1, stream);
    mark(marks, 2, stream);
    mark(marks, 3, stream);
    return;
  }
  RenderParams T = P;
  int tblocks = 0, per_region = 0;
  bool ordered = order_geometry(T, tblocks, per_region);
  const size_t tlds = DEEP ? sizeof(int) * kDeepWords * kDeepStack * kTraceWaves : 0;
  int oblocks = ordered ? T.order_regions * T.order_stride : tblocks;
  const RenderParams S = T;
  // one kernel per frame, dispatched by the previous frame's heavy-first order when there is one
  // (warm order: same selection, same stream), else — a camera's whole frame — by the order
  // seeded at scene creation (cold order, no split); the order kernel then sorts this frame's
  // packet costs for the next frame
  mark(marks, 0, stream);
  if (!ordered) T.tile_cost = nullptr;
  T.use_order = ordered && P.primary_order ? 1 : 0;
  if (ordered && !T.use_order && P.cold_order && P.num_sel_tiles == P.cold_tiles) {
    T.order_split = 0;
    T.order_stride = per_region;
    T.unit_order = const_cast<int*>(P.cold_order);
    T.use_order = 1;
    oblocks = T.order_regions * T.order_stride;
  }
  // every workgroup holds two tiles of one tile row (tiles_x even, whole 16-pixel rows)
  T.pair_rows = P.pair_rows && kTraceWaves == 2 && kBlockW == 2 && T.tile_block && !T.use_order &&
                !T.tile_major && !T.records && T.tiles_x % 2 == 0 && T.width % 16 == 0 &&
                (reinterpret_cast<uintptr_t>(T.out) & 15) == 0 ? 1 : 0;
  hipLaunchKernelGGL((trace_frame_kernel<FAST, DEEP, SPHERES>), dim3(T.use_order ? oblocks : tblocks),
                     dim3(kTraceWaves * 64), tlds, stream, T, nodes, lights);
  mark(marks, 1, stream);
  if (ordered) hipLaunchKernelGGL(order_kernel, dim3(S.order_regions), dim3(kOrderThreads), 0, stream, S);
  mark(marks, 2, stream);
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
  const int aj = M.row_lo + (int)(blockIdx.y * 16 + (threadIdx.x >> 4));
  if (ai >= M.width || aj >= M.row_hi) return;
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
  if (M.row_hi <= M.row_lo) return hipSuccess;
  const dim3 grid((M.width + 15) / 16, (M.row_hi - M.row_lo + 15) / 16);
  hipLaunchKernelGGL(msaa_resolve_kernel, grid, dim3(256), 0, stream, M);
  return hipGetLastError();
}

// The gathered tiles of a multi-device frame back into rows (UntileParams).  Each 8-pixel row
// of a tile is 96 contiguous bytes in both layouts: six 16-B chunks, one per thread (a wave
// covers 10 tile rows); a tile row on the frame's right edge, or a frame whose rows are not
// 16-B aligned (width % 4 != 0), is copied by pixel instead.
// Gathered tile of frame tile t: rank r's slot tile k (false: a unit of rank 0 under skip_root).
__device__ __forceinline__ bool untile_slot(const UntileParams& U, int t, int tx, int ty, int& r,
                                            int& k) {
  int w = 0;
  const int u = U.blocks ? deal_block_index(U.tiles_x, tx, ty, w) : t;  // deal unit
  r = (u + U.tile_offset) % U.devices;
  if (U.skip_root && r == 0) return false;
  const int b = ((r - U.tile_offset) % U.devices + U.devices) % U.devices;  // rank r's first unit
  k = U.blocks ? 4 * ((u - b) / U.devices) + w : (u - b) / U.devices;  // slot tile
  return true;
}

// (nullptr: a unit of rank 0 under skip_root)
__device__ __forceinline__ const float* untile_src(const UntileParams& U, int t, int tx, int ty) {
  int r, k;
  if (!untile_slot(U, t, tx, ty, r, k)) return nullptr;
  return U.recv + (size_t)(r * U.slot + k) * (kTile * kTile * 3);
}

constexpr int kUntileChunks = 6;  // 16-B chunks per 8-pixel tile row
__global__ __launch_bounds__(256) void untile_kernel(UntileParams U) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long trow = i / kUntileChunks;  // tile row: tile * 8 + row in tile
  const int c = (int)(i - trow * kUntileChunks);
  if (trow >= (long long)U.tiles_total * kTile) return;
  const int t = (int)(trow >> 3), y = (int)(trow & 7);
  const int tx = t % U.tiles_x, ty = t / U.tiles_x;
  const int lr = ty * kTile + y, px0 = tx * kTile;
  if (lr >= U.rows) return;
  const float* src0 = untile_src(U, t, tx, ty);
  if (!src0) return;
  const float* src = src0 + y * (kTile * 3);
  float* dst = U.out + ((size_t)(U.row0 + lr * U.row_stride) * U.width + px0) * 3;
  if (px0 + kTile <= U.width && U.vec) {
    reinterpret_cast<float4*>(dst)[c] = reinterpret_cast<const float4*>(src)[c];
    return;
  }
  // edge tile row / unaligned frame: this thread's four floats, those inside the frame
  const int lim = (U.width - px0) * 3;
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const int f = 4 * c + e;
    if (f < lim) dst[f] = src[f];
  }
}

hipError_t launch_untile(const UntileParams& U, hipStream_t stream) {
  if (U.tiles_total <= 0) return hipSuccess;
  const long long threads = (long long)U.tiles_total * kTile * kUntileChunks;
  hipLaunchKernelGGL(untile_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, stream, U);
  return hipGetLastError();
}

// rt_resolve_device: the gathered pixel records of RT_TILE_RECORDS shares (rt_internal.h) into
// colours of the row-major frame — the shading the frame kernel would have done on the rank that
// traced them, done on the gathering rank.  One thread per pixel, 64 per tile, 4 tiles per
// workgroup.  The hit's t is re-derived by the intersection test the traversal ran (the same ray
// from the same camera arithmetic, the same primitive record, the same operations: the same
// bits), the hit point is o + t * d as trace_ray computes it, and shade_hit is the frame kernel's.
// The colour of pixel (px, py) from its record (not kRecOutside).
template <bool SPHERES>
__device__ __forceinline__ V3 resolve_pixel(const RenderParams& P, unsigned rec, int px, int py) {
  if (rec & kRecMiss) return ld3(P.background);
  const int leaf = (int)(rec & kRecLeafMask);
  const V3 e = ld3(P.cam_e), d = primary_dir(P, px, py);
  const LaneRay ray = make_ray(e, d, P.quot_ok);
  float th = 0.0f;
  (void)leaf_test<SPHERES>(P.prims, leaf, ray, th);
  const unsigned occ = (rec >> kRecLightShift) & kRecLightMask;
  return shade_hit<SPHERES>(P, P.prims, P.normals, P.materials, P.lights, leaf, e + d * th,
                            [&](int li) { return ((occ >> li) & 1u) != 0; });
}

// rt_resolve_rows: row-major pixel records (a row band's, received whole) into the row-major
// frame, rows [row_begin, row_end) of the camera's own frame; one thread per pixel.
#ifndef RT_RESOLVE_PATCH  // (A/B builds: 0 = 256 consecutive pixels of a row per workgroup)
#define RT_RESOLVE_PATCH 1
#endif
#ifndef RT_RESOLVE_PW  // patch width (A/B builds); height 256 / width
#define RT_RESOLVE_PW 32
#endif
constexpr int kResolvePW = RT_RESOLVE_PW, kResolvePH = 256 / RT_RESOLVE_PW;
template <bool SPHERES>
__global__ __launch_bounds__(256) void resolve_rows_kernel(RenderParams P, const unsigned* rec,
                                                           int row_begin, int row_end) {
#if RT_RESOLVE_PATCH
  // a 32 x 8 patch of pixels per workgroup: neighbouring rows' hits share primitives
  const int px = (int)blockIdx.x * kResolvePW + (int)(threadIdx.x % kResolvePW);
  const long long py = row_begin + (long long)blockIdx.y * kResolvePH + (threadIdx.x / kResolvePW);
  if (px >= P.width || py >= row_end) return;
#else
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long py = row_begin + i / P.width;
  if (py >= row_end) return;
  const int px = (int)(i % P.width);
#endif
  const size_t pix = (size_t)py * P.width + px;
  const V3 color = resolve_pixel<SPHERES>(P, rec[pix], px, (int)py);
  float* o = P.out + 3 * pix;
  o[0] = 0.0f + color.x;
  o[1] = 0.0f + color.y;
  o[2] = 0.0f + color.z;
}

hipError_t launch_resolve_rows(const RenderParams& P, const unsigned* rec, int row_begin,
                               int row_end, bool spheres, hipStream_t stream) {
  const long long n = (long long)(row_end - row_begin) * P.width;
  if (n <= 0) return hipSuccess;
  const dim3 grid = RT_RESOLVE_PATCH ? dim3((unsigned)((P.width + kResolvePW - 1) / kResolvePW),
                                            (unsigned)((row_end - row_begin + kResolvePH - 1) / kResolvePH))
                                     : dim3((unsigned)((n + 255) / 256));
  if (spheres)
    hipLaunchKernelGGL(resolve_rows_kernel<true>, grid, dim3(256), 0, stream, P, rec, row_begin, row_end);
  else
    hipLaunchKernelGGL(resolve_rows_kernel<false>, grid, dim3(256), 0, stream, P, rec, row_begin, row_end);
  return hipGetLastError();
}

template <bool SPHERES>
__global__ __launch_bounds__(256) void resolve_kernel(RenderParams P, UntileParams U) {
  const int t = (int)(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (t >= U.tiles_total) return;
  const int lane = (int)(threadIdx.x & 63);
  const int tx = t % U.tiles_x, ty = t / U.tiles_x;
  const int px = tx * kTile + (lane & 7), lr = ty * kTile + (lane >> 3);
  if (px >= U.width || lr >= U.rows) return;
  int r, k;
  if (!untile_slot(U, t, tx, ty, r, k)) return;
  const unsigned rec = reinterpret_cast<const unsigned*>(U.recv)[(size_t)(r * U.slot + k) * (kTile * kTile) + lane];
  if (rec & kRecOutside) return;
  const int py = U.row0 + lr * U.row_stride;
  const V3 color = resolve_pixel<SPHERES>(P, rec, px, py);
  float* o = U.out + 3 * ((size_t)py * U.width + px);
  o[0] = 0.0f + color.x;
  o[1] = 0.0f + color.y;
  o[2] = 0.0f + color.z;
}

hipError_t launch_resolve(const RenderParams& P, const UntileParams& U, bool spheres,
                          hipStream_t stream) {
  if (U.tiles_total <= 0) return hipSuccess;
  const dim3 grid((unsigned)((U.tiles_total + 3) / 4));
  if (spheres)
    hipLaunchKernelGGL(resolve_kernel<true>, grid, dim3(256), 0, stream, P, U);
  else
    hipLaunchKernelGGL(resolve_kernel<false>, grid, dim3(256), 0, stream, P, U);
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
                         bool fast, bool deep, bool spheres, const hipEvent_t* marks,
                         hipStream_t stream) {
  if (P.num_sel_tiles <= 0) return hipSuccess;
  const int blocks = (P.num_sel_tiles + kWavesPerBlock - 1) / kWavesPerBlock;
  // FAST walks the culling tree: only when the scene has one (a root primitive or a tree of
  // one treelet has none, accel_build.cpp)
  fast = fast && P.accel_root >= 0 && P.root_kind == kRootNode && P.leaves != nullptr;
  const int v = (fast ? 4 : 0) | (deep ? 2 : 0) | (spheres ? 1 : 0);
  switch (v) {
#define RT_CASE(F, D, S)                                                                 \
  case (F ? 4 : 0) | (D ? 2 : 0) | (S ? 1 : 0):                                          \
    launch_variant<F, D, S>(P, nodes, prims, normals, mats, lights, blocks, marks, stream); \
    break;
    RT_CASE(true, false, false)
    RT_CASE(true, false, true)
    RT_CASE(true, true, false)
    RT_CASE(true, true, true)
    RT_CASE(false, false, false)
    RT_CASE(false, false, true)
    RT_CASE(false, true, false)
    RT_CASE(false, true, true)
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
// ticks of the 100 MHz clock and (estimated cost << 32 | tile sel, -1 for none).  Returns the number of values
// written, 0 in other builds.
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

// Copies (and clears) the RT_DIAG phase counters (kPhaseSlots values); 0 in other builds.
long long read_reset_phases(unsigned long long* out, long long max_values) {
#ifdef RT_DIAG
  if (max_values < kPhaseSlots) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), kPhaseSlots * sizeof *out) != hipSuccess) return -1;
  unsigned long long z[kPhaseSlots] = {};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof z) != hipSuccess) return -1;
  return kPhaseSlots;
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
