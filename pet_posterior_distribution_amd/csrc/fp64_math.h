// fp64 device math shared by the MH and U-Net kernels (no reference counterpart).
#pragma once
#include <hip/hip_runtime.h>

// Natural log of a positive finite x: frexp to m in [1/sqrt 2, sqrt 2), f = m - 1, s = f / (2 + f),
// log m = f - (f^2/2 - s (f^2/2 + R(s^2))) with R the degree-7 minimax of fdlibm's e_log.c (Lg1..Lg7),
// k ln 2 in two parts: <= 1 ulp (checked against numpy / mpmath), about a fifth of ocml's
// instruction count.  Zero, negative, inf and NaN go to ocml's log.
__device__ __forceinline__ double log_pos(double x) {
  if (!(x > 0.0 && x < __builtin_huge_val())) return log(x);
  int e;
  double m = frexp(x, &e);
  if (m < 0.70710678118654752440) {
    m *= 2.0;
    e -= 1;
  }
  const double f = m - 1.0, s = f / (2.0 + f), z = s * s, w = z * z;
  const double t1 = w * (3.999999999940941908e-01 + w * (2.222219843214978396e-01 + w * 1.531383769920937332e-01));
  const double t2 = z * (6.666666666666735130e-01 +
                         w * (2.857142874366239149e-01 + w * (1.818357216161805012e-01 + w * 1.479819860511658591e-01)));
  const double R = t2 + t1, hfsq = 0.5 * f * f, k = (double)e;
  return k * 6.93147180369123816490e-01 - ((hfsq - (s * (hfsq + R) + k * 1.90821492927058770002e-10)) - f);
}


// e^x: x = k ln 2 + r, |r| <= ln 2 / 2 (ln 2 in two parts), e^r by its degree-13 Taylor polynomial
// (truncation 6e-18), 2^k by ldexp: <= 1 ulp (checked against numpy).  Outside (-745, 709.7) and
// NaN: ocml's exp (0 / inf / NaN).
__device__ __forceinline__ double exp_fast(double x) {
  if (!(x > -745.0 && x < 709.7)) return exp(x);
  const double kf = rint(x * 1.4426950408889634);
  double r = fma(-kf, 6.93147180369123816490e-01, x);
  r = fma(-kf, 1.90821492927058770002e-10, r);
  double p = 1.6059043836821613e-10;                       // 1/13!
  p = fma(p, r, 2.08767569878681e-09);                     // 1/12!
  p = fma(p, r, 2.505210838544172e-08);
  p = fma(p, r, 2.755731922398589e-07);
  p = fma(p, r, 2.7557319223985893e-06);
  p = fma(p, r, 2.48015873015873e-05);
  p = fma(p, r, 0.0001984126984126984);
  p = fma(p, r, 0.001388888888888889);
  p = fma(p, r, 0.008333333333333333);
  p = fma(p, r, 0.041666666666666664);
  p = fma(p, r, 0.16666666666666666);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return ldexp(p, (int)kf);
}
