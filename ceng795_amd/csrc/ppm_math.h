// Portable scalar math for the photon-mapping path (PPM), shared by the device kernels and
// the CPU oracle (oracle/ppm_ref.cpp) so that both trace bit-identical photon paths.
//
// The reference calls glibc's sinf/cosf (as sincosf), asinf and powf (PPM/src/Point_light.cpp:
// 20-29, PPM/src/Scene.cpp:15-44 and :153-158, :181-186).  Neither glibc nor ocml is available
// on both sides, so these are written with IEEE +,-,*,/ on doubles only (no FMA: build with
// -ffp-contract=off) plus float sqrt, all of which round identically on x86-64 and gfx950.
// Each evaluates the function in double with error far below 2^-30 and rounds once to float,
// so it returns the correctly rounded float except on rare near-midpoint inputs — the same
// contract glibc's float functions meet; tests/test_ppm_oracle.py measures the agreement.
//
// Random numbers: the reference draws from std::mt19937 seeded by std::random_device
// (non-reproducible, PPM/src/Scene.cpp:17-18,107-108; Point_light.cpp:10-11).  Here each
// photon (and each eye sample) owns a SplitMix64 stream seeded from (seed, stream id), and a
// draw becomes a float exactly as libstdc++'s uniform_real_distribution<float>(0, 1) turns a
// 32-bit engine output into one (generate_canonical<float, 24>: float(u) / 2^32, kept < 1).
#ifndef CENG795_PPM_MATH_H_
#define CENG795_PPM_MATH_H_

#include <cmath>
#include <cstdint>
#include <cstring>

#ifdef __HIPCC__
#define PPM_HD __host__ __device__ __forceinline__
#else
#define PPM_HD inline
#endif

#ifdef __clang__
#pragma clang fp contract(off)
#endif

namespace ppm_math {

constexpr double kPi = 0x1.921fb54442d18p+1;
constexpr double kPio2 = 0x1.921fb54442d18p+0;
constexpr double kInvPio2 = 0x1.45f306dc9c883p-1;
constexpr double kPio2Hi = 0x1.921fb544p+0;   // first 33 bits of pi/2 (k * hi exact, k < 2^20)
constexpr double kPio2Lo = 0x1.0b4611a626331p-34;  // pi/2 - kPio2Hi
constexpr double kLn2Hi = 0x1.62e42feep-1;    // ln 2 split as in fdlibm
constexpr double kLn2Lo = 0x1.a39ef35793c76p-33;
constexpr double kInvLn2 = 0x1.71547652b82fep+0;

PPM_HD uint64_t dbits(double x) {
  uint64_t u;
  std::memcpy(&u, &x, 8);
  return u;
}
PPM_HD double dfrom(uint64_t u) {
  double x;
  std::memcpy(&x, &u, 8);
  return x;
}
PPM_HD double dfloor(double x) {  // floor for |x| < 2^52 without libm
  if (!(x > -4503599627370496.0 && x < 4503599627370496.0)) return x;
  double t = (double)(int64_t)x;
  return t > x ? t - 1.0 : t;
}
PPM_HD double dscale2(double x, int k) {  // x * 2^k for -2000 < k < 2000, no libm
  while (k > 1000) {
    x *= 0x1p+1000;
    k -= 1000;
  }
  while (k < -1000) {
    x *= 0x1p-1000;
    k += 1000;
  }
  return x * dfrom((uint64_t)(k + 1023) << 52);
}

// sin and cos of r, |r| <= pi/4 (Taylor to r^19 / r^18: truncation < 1e-19).
PPM_HD double sin_kernel(double r) {
  const double z = r * r;
  double p = -0x1.2f49b46814157p-57;
  p = p * z + 0x1.952c77030ad4ap-49;
  p = p * z + -0x1.ae7f3e733b81fp-41;
  p = p * z + 0x1.6124613a86d09p-33;
  p = p * z + -0x1.ae64567f544e4p-26;
  p = p * z + 0x1.71de3a556c734p-19;
  p = p * z + -0x1.a01a01a01a01ap-13;
  p = p * z + 0x1.1111111111111p-7;
  p = p * z + -0x1.5555555555555p-3;
  return r + r * (z * p);
}
PPM_HD double cos_kernel(double r) {
  const double z = r * r;
  double p = -0x1.6827863b97d97p-53;
  p = p * z + 0x1.ae7f3e733b81fp-45;
  p = p * z + -0x1.93974a8c07c9dp-37;
  p = p * z + 0x1.1eed8eff8d898p-29;
  p = p * z + -0x1.27e4fb7789f5cp-22;
  p = p * z + 0x1.a01a01a01a01ap-16;
  p = p * z + -0x1.6c16c16c16c17p-10;
  p = p * z + 0x1.5555555555555p-5;
  p = p * z + -0x1.0000000000000p-1;
  return 1.0 + z * p;
}

// sinf / cosf: quadrant reduction x = k*pi/2 + r in double (Cody-Waite, exact for |x| < 2^19).
PPM_HD void sincosf_ieee(float xf, float& s, float& c) {
  const double x = (double)xf;
  if (!(x - x == 0.0)) {  // inf / nan
    s = c = (float)(x - x);
    return;
  }
  const double k = dfloor(x * kInvPio2 + 0.5);
  const double r = (x - k * kPio2Hi) - k * kPio2Lo;
  const double sr = sin_kernel(r), cr = cos_kernel(r);
  const int q = (int)((int64_t)k & 3);
  double sv, cv;
  if (q == 0) {
    sv = sr;
    cv = cr;
  } else if (q == 1) {
    sv = cr;
    cv = -sr;
  } else if (q == 2) {
    sv = -sr;
    cv = -cr;
  } else {
    sv = -cr;
    cv = sr;
  }
  s = (float)sv;
  c = (float)cv;
}
PPM_HD float sinf_ieee(float x) {
  float s, c;
  sincosf_ieee(x, s, c);
  return s;
}
PPM_HD float cosf_ieee(float x) {
  float s, c;
  sincosf_ieee(x, s, c);
  return c;
}

// asin(x) for |x| <= 0.5 by its Taylor series to x^55 (truncation < 1e-18 relative).
PPM_HD double asin_series(double x) {
  const double z = x * x;
  double p = 0x1.018f963c229bfp-9;
  p = p * z + 0x1.1052bc5fa960ap-9;
  p = p * z + 0x1.208d3570ae5a6p-9;
  p = p * z + 0x1.3275586c5f2f0p-9;
  p = p * z + 0x1.464c0950f7d47p-9;
  p = p * z + 0x1.5c5f56efaaaabp-9;
  p = p * z + 0x1.750de64d7d05fp-9;
  p = p * z + 0x1.90cb77f60c7cep-9;
  p = p * z + 0x1.b026f57b13b14p-9;
  p = p * z + 0x1.d3d2a8e0dd67dp-9;
  p = p * z + 0x1.fcaf8fb6db6dbp-9;
  p = p * z + 0x1.15ee9d45d1746p-8;
  p = p * z + 0x1.31683bdef7bdfp-8;
  p = p * z + 0x1.51ba308d3dcb1p-8;
  p = p * z + 0x1.782dda12f684cp-8;
  p = p * z + 0x1.a6863d70a3d71p-8;
  p = p * z + 0x1.df3bd37a6f4dfp-8;
  p = p * z + 0x1.12ef3cf3cf3cfp-7;
  p = p * z + 0x1.3fde50d79435ep-7;
  p = p * z + 0x1.7a87878787878p-7;
  p = p * z + 0x1.c99999999999ap-7;
  p = p * z + 0x1.1c4ec4ec4ec4fp-6;
  p = p * z + 0x1.6e8ba2e8ba2e9p-6;
  p = p * z + 0x1.f1c71c71c71c7p-6;
  p = p * z + 0x1.6db6db6db6db7p-5;
  p = p * z + 0x1.3333333333333p-4;
  p = p * z + 0x1.5555555555555p-3;
  return x + x * (z * p);
}
// sqrt in double from the correctly rounded float sqrt and two Newton steps (IEEE ops only).
PPM_HD double dsqrt(double v) {
  if (!(v > 0.0)) return v == 0.0 ? v : (v - v) / (v - v);
  double y = (double)sqrtf((float)v);
  if (!(y > 0.0)) y = 0x1p-75;
  y = 0.5 * (y + v / y);
  y = 0.5 * (y + v / y);
  return y;
}
PPM_HD float asinf_ieee(float xf) {
  double x = (double)xf;
  const bool neg = x < 0.0;
  if (neg) x = -x;
  if (!(x <= 1.0)) return (float)((x - x) / (x - x));  // |x| > 1 or nan
  double r;
  if (x <= 0.5) {
    r = asin_series(x);
  } else {  // asin x = pi/2 - 2 asin(sqrt((1-x)/2))
    r = kPio2 - 2.0 * asin_series(dsqrt((1.0 - x) * 0.5));
  }
  return (float)(neg ? -r : r);
}

// log(x), x > 0 finite normal or subnormal: x = m 2^e, m in [sqrt(1/2), sqrt 2),
// log m = 2 atanh(s), s = (m-1)/(m+1), |s| < 0.1716 (series to s^27).
PPM_HD double dlog(double x) {
  int e = 0;
  if (x < 0x1p-1022) {
    x *= 0x1p+54;
    e = -54;
  }
  uint64_t u = dbits(x);
  e += (int)((u >> 52) & 0x7ff) - 1023;
  double m = dfrom((u & 0x000fffffffffffffull) | 0x3ff0000000000000ull);
  if (m > 0x1.6a09e667f3bcdp+0) {
    m *= 0.5;
    e += 1;
  }
  const double s = (m - 1.0) / (m + 1.0);
  const double z = s * s;
  double p = 0x1.2f684bda12f68p-4;
  p = p * z + 0x1.47ae147ae147bp-4;
  p = p * z + 0x1.642c8590b2164p-4;
  p = p * z + 0x1.8618618618618p-4;
  p = p * z + 0x1.af286bca1af28p-4;
  p = p * z + 0x1.e1e1e1e1e1e1ep-4;
  p = p * z + 0x1.1111111111111p-3;
  p = p * z + 0x1.3b13b13b13b14p-3;
  p = p * z + 0x1.745d1745d1746p-3;
  p = p * z + 0x1.c71c71c71c71cp-3;
  p = p * z + 0x1.2492492492492p-2;
  p = p * z + 0x1.999999999999ap-2;
  p = p * z + 0x1.5555555555555p-1;
  const double lm = 2.0 * s + s * (z * p);
  return (double)e * kLn2Hi + ((double)e * kLn2Lo + lm);
}
// exp(z): z = k ln2 + r, |r| <= ln2/2, Taylor to r^21.
PPM_HD double dexp(double z) {
  if (z != z) return z;
  if (z > 709.8) return 0x1p+1023 * 0x1p+1023;
  if (z < -745.2) return 0.0;
  const double k = dfloor(z * kInvLn2 + 0.5);
  const double r = (z - k * kLn2Hi) - k * kLn2Lo;
  double p = 0x1.71b8ef6dcf572p-66;
  p = p * r + 0x1.e542ba4020225p-62;
  p = p * r + 0x1.2f49b46814157p-57;
  p = p * r + 0x1.6827863b97d97p-53;
  p = p * r + 0x1.952c77030ad4ap-49;
  p = p * r + 0x1.ae7f3e733b81fp-45;
  p = p * r + 0x1.ae7f3e733b81fp-41;
  p = p * r + 0x1.93974a8c07c9dp-37;
  p = p * r + 0x1.6124613a86d09p-33;
  p = p * r + 0x1.1eed8eff8d898p-29;
  p = p * r + 0x1.ae64567f544e4p-26;
  p = p * r + 0x1.27e4fb7789f5cp-22;
  p = p * r + 0x1.71de3a556c734p-19;
  p = p * r + 0x1.a01a01a01a01ap-16;
  p = p * r + 0x1.a01a01a01a01ap-13;
  p = p * r + 0x1.6c16c16c16c17p-10;
  p = p * r + 0x1.1111111111111p-7;
  p = p * r + 0x1.5555555555555p-5;
  p = p * r + 0x1.5555555555555p-3;
  p = p * r + 0x1.0000000000000p-1;
  const double er = 1.0 + (r + r * (r * p));
  return dscale2(er, (int)k);
}
// powf for the Phong lobes: x >= 0 (the reference clamps with std::max(0.0f, .)).
PPM_HD float powf_ieee(float xf, float yf) {
  const double x = (double)xf, y = (double)yf;
  if (y == 0.0 || x == 1.0) return 1.0f;
  if (x != x || y != y) return (float)(x + y);
  if (y == 1.0) return xf;  // exact (the default PhongExponent)
  if (x == 0.0) return y > 0.0 ? 0.0f : (float)(1.0 / x);
  if (x < 0.0) return (float)((x - x) / (x - x));  // not used by the path (documented)
  if (x - x != 0.0) return y > 0.0 ? xf : 0.0f;    // +inf
  return (float)dexp(y * dlog(x));
}

// ------------------------------------------------------------------ random numbers
PPM_HD uint64_t mix64(uint64_t z) {  // SplitMix64 finaliser
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
struct Rng {  // one SplitMix64 stream per photon / per eye sample
  uint64_t state;
  PPM_HD Rng(uint64_t seed, uint64_t stream) : state(mix64(seed ^ mix64(stream + 0x632BE59BD9B4E019ull))) {}
  PPM_HD uint32_t next_u32() {
    state += 0x9E3779B97F4A7C15ull;
    return (uint32_t)(mix64(state) >> 32);
  }
  // uniform_real_distribution<float>(0, 1) over a 32-bit engine (libstdc++
  // generate_canonical<float, 24>: one draw, float(u) / 2^32, clamped below 1).
  PPM_HD float uniform01() {
    float r = (float)next_u32() / 4294967296.0f;
    if (r >= 1.0f) r = 0x1.fffffep-1f;
    return r;
  }
};
// Stream ids: photons use their index; eye samples set the top bit.
constexpr uint64_t kEyeStream = 0x8000000000000000ull;

}  // namespace ppm_math

#endif
