// Domain-specialised fp32 math for the routing physics (gfx950).
//
// pow_pos(x, y): x > 0 finite and normal (fp32), |y * ln x| < 700.  Evaluated in fp64 with
//   table-driven reductions (tables in LDS, see mathtab.h / load_math_tables):
//     ln x = e ln2 - ln c_j + log1p(m c_j - 1),  j = top 7 mantissa bits, |m c_j - 1| < 2^-8 (exact),
//            log1p by a degree-6 polynomial;
//     exp z = 2^(k >> 7) * 2^((k & 127) / 128) * exp(r),  k = rint(z 128 / ln 2), |r| <= ln2 / 256,
//            exp(r) by a degree-5 polynomial;
//   relative error ~3e-16 before the final rounding to fp32, so the fp32 result is the correctly
//   rounded x^y except when x^y lies within ~3e-16 of a rounding boundary.  ~34 operations and no
//   reciprocal; the ocml powf it replaces costs ~180 instructions (special cases for every IEEE input
//   class).  The reference (PyTorch CPU, Sleef powf_u10) is a 1-ulp approximation that differs from
//   the correctly rounded value in ~1.7% of cases; the oracle uses the correctly rounded value.
// div_rn(a, b): IEEE round-to-nearest quotient for normal operands whose quotient is normal (no
//   scaling steps): refined reciprocal + one FMA residual correction (Markstein).
// Both are checked on the GPU against fp64 references by tools/fm_check.hip.
#pragma once

#include <hip/hip_runtime.h>

#include "mathtab.h"

namespace ddr {

// The tables occupy the first (2 kLnTabN + kExpTabN) doubles of the dynamic LDS of every kernel
// that calls pow_pos (kMathTabBytes in internal.h).
__device__ __forceinline__ double* math_lds() {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  return reinterpret_cast<double*>(smem);
}
// Copy the tables into LDS (all threads of the workgroup; the caller synchronises before use).
__device__ __forceinline__ void load_math_tables() {
  double* t = math_lds();
  for (int i = threadIdx.x; i < 2 * kLnTabN + kExpTabN; i += blockDim.x) t[i] = kMathTab[i];
}

__device__ __forceinline__ float div_rn(float a, float b) {
  float y = __builtin_amdgcn_rcpf(b);
  const float e = fmaf(-b, y, 1.0f);
  y = fmaf(e, y, y);
  const float q = a * y;
  const float r = fmaf(-q, b, a);
  return fmaf(r, y, q);
}

// ln(x) for fp32 x > 0 normal, fp64 result, absolute error ~1e-16 (table-driven).
__device__ __forceinline__ double ln_tab(float x) {
  constexpr double kLn2Hi = 6.93147180369123816490e-01;
  constexpr double kLn2Lo = 1.90821492927058770002e-10;
  const unsigned bits = __float_as_uint(x);
  const int e = (int)(bits >> 23) - 127;
  const unsigned j = (bits >> 16) & 127u;
  const double m = (double)__uint_as_float((bits & 0x7FFFFFu) | 0x3F800000u);  // [1, 2)
  const double2 cl = reinterpret_cast<const double2*>(math_lds())[j];           // (c_j, -ln c_j)
  const double r = fma(m, cl.x, -1.0);                                          // exact
  double t = fma(r, -1.0 / 6.0, 0.2);
  t = fma(t, r, -0.25);
  t = fma(t, r, 1.0 / 3.0);
  t = fma(t, r, -0.5);
  const double l1p = fma(t, r * r, r);
  const double de = (double)e;
  return fma(de, kLn2Hi, fma(de, kLn2Lo, cl.y + l1p));
}

// exp(z) for |z| < 700, fp64, relative error ~2e-16 (table-driven).
__device__ __forceinline__ double exp_tab(double z) {
  constexpr double kInvL = 1.84664965233787316142e+02;        // 128 / ln 2
  constexpr double kLHi = 6.93147180369123816490e-01 / 128.0;  // ln 2 / 128, split (exact products)
  constexpr double kLLo = 1.90821492927058770002e-10 / 128.0;
  const double kd = __builtin_rint(z * kInvL);
  const int k = (int)kd;
  const double r = fma(-kd, kLLo, fma(-kd, kLHi, z));          // |r| <= ln2 / 256
  double t = fma(r, 1.0 / 120.0, 1.0 / 24.0);
  t = fma(t, r, 1.0 / 6.0);
  t = fma(t, r, 0.5);
  t = fma(t, r, 1.0);
  t = fma(t, r, 1.0);                                          // exp(r)
  const double E = math_lds()[2 * kLnTabN + (k & 127)];         // 2^((k & 127) / 128)
  return __builtin_amdgcn_ldexp(E * t, k >> 7);
}

// x^y (x > 0) rounded to fp32; ln_out receives ln(x) (fp64) for derivative use.
__device__ __forceinline__ float pow_pos(float x, float y, double* ln_out = nullptr) {
  const double l = ln_tab(x);
  if (ln_out) *ln_out = l;
  return (float)exp_tab((double)y * l);
}

}  // namespace ddr
