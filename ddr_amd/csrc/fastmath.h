// Domain-specialised fp32 math for the routing physics (gfx950).
//
// pow_pos(x, y): x > 0 finite and normal, |y * ln x| < 700.  Evaluated in fp64 -- ln by the atanh
//   series on the reduced mantissa, exp by a Taylor polynomial after ln 2 range reduction --
//   with ~1e-14 relative error before the final rounding to fp32, so the fp32 result is the
//   correctly rounded x^y except when x^y lies within ~1e-14 of a rounding boundary.  The ocml
//   powf it replaces costs ~180 instructions (special cases for every IEEE input class); this
//   is ~44 fp64 operations.  The reference (PyTorch CPU, Sleef powf_u10) is a 1-ulp approximation
//   that differs from the correctly rounded value in ~1.7% of cases; the oracle uses the correctly
//   rounded value.
// div_rn(a, b): IEEE round-to-nearest quotient for normal operands whose quotient is normal (no
//   scaling steps): refined reciprocal + one FMA residual correction (Markstein).  Checked
//   bit-exact against the IEEE division over the physics' operand ranges in tests.
#pragma once

#include <hip/hip_runtime.h>

namespace ddr {

__device__ __forceinline__ float div_rn(float a, float b) {
  float y = __builtin_amdgcn_rcpf(b);
  const float e = fmaf(-b, y, 1.0f);
  y = fmaf(e, y, y);
  const float q = a * y;
  const float r = fmaf(-q, b, a);
  return fmaf(r, y, q);
}

// ln(x) for x > 0 normal, fp64, absolute error ~1e-16 * |ln x| + 1e-16.
__device__ __forceinline__ double ln_pos(double x) {
  int e = __builtin_amdgcn_frexp_exp(x);          // x = m * 2^e, m in [0.5, 1)
  double m = __builtin_amdgcn_frexp_mant(x);
  if (m < 0.70710678118654752440) {
    m = m * 2.0;
    e -= 1;
  }
  const double f = m - 1.0;                        // [-0.2929, 0.4142)
  const double d = m + 1.0;
  // s = f / d with a refined hardware reciprocal (two Newton steps)
  double rd = __builtin_amdgcn_rcp(d);
  rd = fma(fma(-d, rd, 1.0), rd, rd);
  rd = fma(fma(-d, rd, 1.0), rd, rd);
  double s = f * rd;
  s = fma(fma(-s, d, f), rd, s);
  const double s2 = s * s;                         // |s| <= 0.1716
  double p = 1.0 / 17.0;
  p = fma(p, s2, 1.0 / 15.0);
  p = fma(p, s2, 1.0 / 13.0);
  p = fma(p, s2, 1.0 / 11.0);
  p = fma(p, s2, 1.0 / 9.0);
  p = fma(p, s2, 1.0 / 7.0);
  p = fma(p, s2, 1.0 / 5.0);
  p = fma(p, s2, 1.0 / 3.0);
  const double lnm = fma(2.0 * s, s2 * p, 2.0 * s);  // 2 atanh(s)
  constexpr double kLn2Hi = 6.93147180369123816490e-01;
  constexpr double kLn2Lo = 1.90821492927058770002e-10;
  const double de = (double)e;
  return fma(de, kLn2Hi, fma(de, kLn2Lo, lnm));
}

// exp(z) for |z| < 700, fp64, relative error ~1e-15.
__device__ __forceinline__ double exp_f64(double z) {
  constexpr double kLog2e = 1.44269504088896338700e+00;
  constexpr double kLn2Hi = 6.93147180369123816490e-01;
  constexpr double kLn2Lo = 1.90821492927058770002e-10;
  const double k = __builtin_rint(z * kLog2e);
  const double r = fma(-k, kLn2Lo, fma(-k, kLn2Hi, z));  // |r| <= 0.347
  double p = 1.0 / 479001600.0;                          // 1/12!
  p = fma(p, r, 1.0 / 39916800.0);
  p = fma(p, r, 1.0 / 3628800.0);
  p = fma(p, r, 1.0 / 362880.0);
  p = fma(p, r, 1.0 / 40320.0);
  p = fma(p, r, 1.0 / 5040.0);
  p = fma(p, r, 1.0 / 720.0);
  p = fma(p, r, 1.0 / 120.0);
  p = fma(p, r, 1.0 / 24.0);
  p = fma(p, r, 1.0 / 6.0);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return __builtin_amdgcn_ldexp(p, (int)k);
}

// x^y (x > 0) rounded to fp32; ln_out receives ln(x) (fp64) for derivative use.
__device__ __forceinline__ float pow_pos(float x, float y, double* ln_out = nullptr) {
  const double l = ln_pos((double)x);
  if (ln_out) *ln_out = l;
  return (float)exp_f64((double)y * l);
}

}  // namespace ddr
