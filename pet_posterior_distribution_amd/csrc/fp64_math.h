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

