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

// fp64 constants of ln_tab / exp_tab.  fp64 VALU instructions take no literal operands on gfx950,
// so each constant occupies a register pair; the routing kernels pin them in VGPRs (pow_consts_vgpr)
// instead of letting the compiler hoist them into SGPRs, where they displaced the kernel's uniform
// values into v_writelane / v_readlane spill traffic.
struct PowK {
  double ln2hi, ln2lo, l6, l5, l4, l3;  // ln: split ln 2, log1p coefficients -1/6, 1/5, -1/4, 1/3
  double invl, lhi, llo, e5, e4, e3;    // exp: 128/ln 2, split ln 2 / 128, 1/120, 1/24, 1/6
};
__host__ __device__ constexpr PowK pow_consts() {
  return PowK{6.93147180369123816490e-01, 1.90821492927058770002e-10, -1.0 / 6.0, 0.2, -0.25, 1.0 / 3.0,
              1.84664965233787316142e+02, 6.93147180369123816490e-01 / 128.0, 1.90821492927058770002e-10 / 128.0,
              1.0 / 120.0, 1.0 / 24.0, 1.0 / 6.0};
}
template <typename V>
__device__ __forceinline__ V in_vgpr(V x) {
  asm volatile("" : "+v"(x));
  return x;
}
__device__ __forceinline__ PowK pow_consts_vgpr() {
  PowK k = pow_consts();
  k.ln2hi = in_vgpr(k.ln2hi); k.ln2lo = in_vgpr(k.ln2lo); k.l6 = in_vgpr(k.l6); k.l5 = in_vgpr(k.l5);
  k.l4 = in_vgpr(k.l4); k.l3 = in_vgpr(k.l3); k.invl = in_vgpr(k.invl); k.lhi = in_vgpr(k.lhi);
  k.llo = in_vgpr(k.llo); k.e5 = in_vgpr(k.e5); k.e4 = in_vgpr(k.e4); k.e3 = in_vgpr(k.e3);
  return k;
}

__device__ __forceinline__ float div_rn(float a, float b) {
  float y = __builtin_amdgcn_rcpf(b);
  const float e = fmaf(-b, y, 1.0f);
  y = fmaf(e, y, y);
  const float q = a * y;
  const float r = fmaf(-q, b, a);
  return fmaf(r, y, q);
}

// IEEE sqrt (round to nearest) of a normal x >= 2^-96, finite: the hardware square root and the two
// one-ulp neighbour corrections of the library's correctly rounded expansion, without its denormal
// scaling and zero / infinity class fix-ups (the physics takes it of 1 + ss^2 >= 1): 9 instructions
// instead of 15, the same bits.
__device__ __forceinline__ float sqrt_rn_normal(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sm = __int_as_float(__float_as_int(s) - 1);
  const float r1 = fmaf(-sm, s, x);
  const float t = r1 <= 0.0f ? sm : s;
  const float sp = __int_as_float(__float_as_int(s) + 1);
  const float r2 = fmaf(-sp, s, x);
  return r2 > 0.0f ? sp : t;
}

// ln(x) for fp32 x > 0 normal, fp64 result, absolute error ~1e-16 (table-driven).
__device__ __forceinline__ double ln_tab(float x, const PowK& K = pow_consts()) {
  const unsigned bits = __float_as_uint(x);
  const int e = (int)(bits >> 23) - 127;
  const unsigned j = (bits >> 16) & 127u;
  const double m = (double)__uint_as_float((bits & 0x7FFFFFu) | 0x3F800000u);  // [1, 2)
  const double2 cl = reinterpret_cast<const double2*>(math_lds())[j];           // (c_j, -ln c_j)
  const double r = fma(m, cl.x, -1.0);                                          // exact
  double t = fma(r, K.l6, K.l5);
  t = fma(t, r, K.l4);
  t = fma(t, r, K.l3);
  t = fma(t, r, -0.5);
  const double l1p = fma(t, r * r, r);
  const double de = (double)e;
  return fma(de, K.ln2hi, fma(de, K.ln2lo, cl.y + l1p));
}

// exp(z) for |z| < 700, fp64, relative error ~2e-16 (table-driven).
__device__ __forceinline__ double exp_tab(double z, const PowK& K = pow_consts()) {
  const double kd = __builtin_rint(z * K.invl);
  const int k = (int)kd;
  const double r = fma(-kd, K.llo, fma(-kd, K.lhi, z));                      // |r| <= ln2 / 256
  double t = fma(r, K.e5, K.e4);
  t = fma(t, r, K.e3);
  t = fma(t, r, 0.5);
  t = fma(t, r, 1.0);
  t = fma(t, r, 1.0);                                          // exp(r)
  const double E = math_lds()[2 * kLnTabN + (k & 127)];         // 2^((k & 127) / 128)
  return __builtin_amdgcn_ldexp(E * t, k >> 7);
}

// x^y (x > 0) rounded to fp32; ln_out receives ln(x) (fp64) for derivative use.
__device__ __forceinline__ float pow_pos(float x, float y, double* ln_out = nullptr, const PowK& K = pow_consts()) {
  const double l = ln_tab(x, K);
  if (ln_out) *ln_out = l;
  return (float)exp_tab((double)y * l, K);
}

// x^y for x > 0 normal, |y log2 x| < 126, in fp32 arithmetic only (no fp64, no tables): a
// faithful-class pow like the reference's Sleef powf_u10.  x = 2^e m with m in [sqrt(1/2), sqrt(2)),
// so the hardware log2 of m is small and its absolute error tiny; y (e + log2 m) is carried as an
// exact product split (FMA remainders), its integer part goes to the exponent and only the fraction
// (|f| <~ 1) meets v_exp_f32.  Measured against the correctly rounded value: tools/pow_check.hip.
__device__ __forceinline__ float pow_faithful(float x, float y) {
  const int u = __float_as_int(x);
  const int ei = (u - 0x3F3504F3) >> 23;
  const float m = __int_as_float(u - (ei << 23));
  const float l = __builtin_amdgcn_logf(m);
  const float fe = (float)ei;
  const float p = y * fe;
  const float pe = fmaf(y, fe, -p);
  const float q = y * l;
  const float qe = fmaf(y, l, -q);
  const float ip = __builtin_rintf(p);
  const float f = ((p - ip) + q) + (pe + qe);
  return __builtin_amdgcn_ldexpf(__builtin_amdgcn_exp2f(f), (int)ip);
}

// ---- lockstep forms: NP independent evaluations advanced one operation at a time, so a wave
// carries NP dependency chains at once (the routing ticks are latency-bound at 4 waves/SIMD) ----
#define DDR_FOR_NP _Pragma("unroll") for (int h = 0; h < NP; ++h)

template <int NP>
__device__ __forceinline__ void div_rn_np(const float (&a)[NP], const float (&b)[NP], float (&q)[NP]) {
  float y[NP], e[NP], r[NP];
  DDR_FOR_NP y[h] = __builtin_amdgcn_rcpf(b[h]);
  DDR_FOR_NP e[h] = fmaf(-b[h], y[h], 1.0f);
  DDR_FOR_NP y[h] = fmaf(e[h], y[h], y[h]);
  DDR_FOR_NP q[h] = a[h] * y[h];
  DDR_FOR_NP r[h] = fmaf(-q[h], b[h], a[h]);
  DDR_FOR_NP q[h] = fmaf(r[h], y[h], q[h]);
}

// ln x (fp64, table-driven as ln_tab) for NP values in lockstep
template <int NP>
__device__ __forceinline__ void ln_np(const float (&x)[NP], double (&l)[NP], const PowK& K) {
  const double2* lt = reinterpret_cast<const double2*>(math_lds());
  double m[NP], r[NP], t[NP], de[NP];
  double2 cl[NP];
  DDR_FOR_NP {
    const unsigned bits = __float_as_uint(x[h]);
    de[h] = (double)((int)(bits >> 23) - 127);
    cl[h] = lt[(bits >> 16) & 127u];
    m[h] = (double)__uint_as_float((bits & 0x7FFFFFu) | 0x3F800000u);
  }
  DDR_FOR_NP r[h] = fma(m[h], cl[h].x, -1.0);
  DDR_FOR_NP t[h] = fma(r[h], K.l6, K.l5);
  DDR_FOR_NP t[h] = fma(t[h], r[h], K.l4);
  DDR_FOR_NP t[h] = fma(t[h], r[h], K.l3);
  DDR_FOR_NP t[h] = fma(t[h], r[h], -0.5);
  DDR_FOR_NP t[h] = fma(t[h], r[h] * r[h], r[h]);
  DDR_FOR_NP l[h] = fma(de[h], K.ln2hi, fma(de[h], K.ln2lo, cl[h].y + t[h]));
}

// exp z (fp64, table-driven as exp_tab) for NP values in lockstep; E receives the fp64 result
template <int NP>
__device__ __forceinline__ void exp_np(const double (&z)[NP], double (&E)[NP], const PowK& K) {
  const double* et = math_lds() + 2 * kLnTabN;
  double r[NP], t[NP], kd[NP];
  int k[NP];
  DDR_FOR_NP kd[h] = __builtin_rint(z[h] * K.invl);
  DDR_FOR_NP k[h] = (int)kd[h];
  DDR_FOR_NP r[h] = fma(-kd[h], K.llo, fma(-kd[h], K.lhi, z[h]));
  DDR_FOR_NP t[h] = fma(r[h], K.e5, K.e4);
  DDR_FOR_NP t[h] = fma(t[h], r[h], K.e3);
  DDR_FOR_NP t[h] = fma(t[h], r[h], 0.5);
  DDR_FOR_NP t[h] = fma(t[h], r[h], 1.0);
  DDR_FOR_NP t[h] = fma(t[h], r[h], 1.0);
  DDR_FOR_NP E[h] = __builtin_amdgcn_ldexp(et[k[h] & 127] * t[h], k[h] >> 7);
}

template <int NP>
__device__ __forceinline__ void pow_pos_np(const float (&x)[NP], const float (&y)[NP], float (&out)[NP],
                                           const PowK& K) {
  double l[NP], z[NP], E[NP];
  ln_np<NP>(x, l, K);
  DDR_FOR_NP z[h] = (double)y[h] * l[h];
  exp_np<NP>(z, E, K);
  DDR_FOR_NP out[h] = (float)E[h];
}

}  // namespace ddr
