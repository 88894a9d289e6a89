// ddmath.h — double-double arithmetic for the correctly rounded acos of the FPFH swap test.
//
// Open3D's ComputePairFeatures (reference ransac.py:85 → pcd_fpfh, ply.py:117-120) swaps source
// and target when acos(|a1|) > acos(|a2|).  Mathematically that is |a1| < |a2|; in floating point
// the two acos values of a near tie (|a1|, |a2| a few ulps apart) may round to the same double,
// and then no swap happens — so the decision depends on the libm's rounding.  The device's
// libm (ocml) and glibc differ there; a correctly rounded acos agrees with glibc wherever glibc
// rounds correctly (glibc 2.35: ~99.9 % of arguments, and every swap test of the FPFH parity
// clouds, tools/fpfh_parity.py).  acos_gt below decides the test as the correctly rounded values
// would: far-apart arguments by their order, near ties by acos_cr.
//
// acos_cr(u), 0 ≤ u < 1: θ0 = the libm's acos (error ≤ 2 ulp), then one Newton step on cos θ = u
// with the residual cos θ0 − u = (1 − u) − 2 sin²(θ0 / 2) in double-double — 1 − u exact by
// two_sum, sin by its Taylor series to x²⁹ (x ≤ π/4: truncation < 1e-33) with double-double
// coefficients — so the residual carries ~1e-32 absolute error even where it cancels, and
// θ0 + δ is within ~1e-31 (relative) of acos(u): its rounding is the correct one unless acos(u)
// lies that close to a rounding boundary.  Host and device compile the same code (the host copy
// is exported as m3d_debug_acos_cr for the CPU test against mpmath).
#pragma once

#include <cmath>

#ifndef M3D_HD
#define M3D_HD __host__ __device__ inline
#endif

namespace m3d {

struct dd {
  double hi, lo;
};

M3D_HD dd two_sum(double a, double b) {
  const double s = a + b;
  const double bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}

M3D_HD dd quick_two_sum(double a, double b) {  // |a| ≥ |b|
  const double s = a + b;
  return {s, b - (s - a)};
}

M3D_HD dd two_prod(double a, double b) {
  const double p = a * b;
  return {p, std::fma(a, b, -p)};
}

M3D_HD dd dd_add(dd a, dd b) {
  const dd s = two_sum(a.hi, b.hi);
  const dd t = two_sum(a.lo, b.lo);
  dd r = quick_two_sum(s.hi, s.lo + t.hi);
  return quick_two_sum(r.hi, r.lo + t.lo);
}

M3D_HD dd dd_mul(dd a, dd b) {
  dd p = two_prod(a.hi, b.hi);
  p.lo += a.hi * b.lo + a.lo * b.hi;
  return quick_two_sum(p.hi, p.lo);
}

// sin x, 0 ≤ x ≤ π/4, in double-double: x · Σ_k c_k (x²)^k, Horner from k = 14
M3D_HD dd sin_dd(double x) {
  const double c[14][2] = {
      {-0.16666666666666666, -9.25185853854297e-18},        {0.008333333333333333, 1.1564823173178714e-19},
      {-0.0001984126984126984, -1.7209558293420705e-22},    {2.7557319223985893e-06, -1.858393274046472e-22},
      {-2.505210838544172e-08, 1.448814070935912e-24},      {1.6059043836821613e-10, 1.2585294588752098e-26},
      {-7.647163731819816e-13, -7.03872877733453e-30},      {2.8114572543455206e-15, 1.6508842730861433e-31},
      {-8.22063524662433e-18, -2.2141894119604265e-34},     {1.9572941063391263e-20, -1.3643503830087908e-36},
      {-3.868170170630684e-23, 8.843177655482344e-40},      {6.446950284384474e-26, -1.9330404233703465e-42},
      {-9.183689863795546e-29, -1.4303150396787322e-45},    {1.1309962886447716e-31, 1.0498015412959506e-47}};
  const dd x2 = two_prod(x, x);
  dd p = {c[13][0], c[13][1]};
  for (int k = 12; k >= 0; --k) p = dd_add(dd_mul(p, x2), dd{c[k][0], c[k][1]});
  p = dd_add(dd_mul(p, x2), dd{1.0, 0.0});  // 1 + x²·(…)
  return dd_mul(p, dd{x, 0.0});
}

// correctly rounded acos(u) (see the header); u ≥ 1, u < 0 and NaN go to the libm
M3D_HD double acos_cr(double u) {
  const double t0 = std::acos(u);
  if (!(u >= 0.0 && u < 1.0) || t0 == 0.0) return t0;
  const dd s = sin_dd(0.5 * t0);
  const dd s2 = dd_mul(s, s);
  const dd n = dd_add(two_sum(1.0, -u), dd{-2.0 * s2.hi, -2.0 * s2.lo});  // cos θ0 − u
  const double r = n.hi + n.lo;
  const double st = std::sin(t0), ct = std::cos(t0);
  double d = r / st;                 // Newton: cos(θ0 + δ) = u
  d -= 0.5 * d * d * ct / st;        // its second-order term
  return t0 + d;
}

// CR(acos u) > CR(acos v) for u, v ≥ 0 (the FPFH swap test on |a1|, |a2|)
M3D_HD bool acos_gt(double u, double v) {
  if (!(u < 1.0 && v < 1.0)) return std::acos(u) > std::acos(v);  // 1, > 1 (NaN) and NaN as the libm
  if (u == v) return false;
  // acos has slope ≤ −1: arguments more than 5e-16 apart give values more than 2 ulp (θ < 2)
  // apart, whose roundings — correct, or glibc's within 1 ulp — keep the order
  if (std::fabs(u - v) > 5e-16) return u < v;
  return acos_cr(u) > acos_cr(v);
}

}  // namespace m3d
