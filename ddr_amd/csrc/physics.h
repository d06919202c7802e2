// Element-wise Muskingum-Cunge physics for one reach and one step, forward and VJP.
//
// Forward (operation order of the reference, each op rounded in R, no FMA contraction -- the
// library is compiled with -ffp-contract=off):
//   geometry/trapezoidal.py:62-97  depth (Manning inversion), top width, side slope, bottom width,
//                                  area, wetted perimeter, hydraulic radius, velocity
//   routing/mmc.py:165-167         celerity c = clamp(v, v_lb, 15) * 5 / 3
//   routing/mmc.py:479-484         Muskingum coefficients c1..c4
// fp32: divisions are IEEE-exact (div_rn), pow is correctly rounded (pow_pos, fastmath.h).
// fp64: plain IEEE division and ocml pow.
// VJP: hand-derived, clamp gradients inclusive at the bounds like
// torch.clamp's backward.
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include "fastmath.h"

namespace ddr {

template <typename R>
struct Consts {
  R dt, qlb, vlb, vub, dlb, bwlb, sslb, ssub;
  PowK pk;        // fp64 constants of the fp32 pow (register-pinned by the routing kernels)
  double ln_dlb;  // ln of the depth lower bound (fp64, host-computed)
  float pinf = __builtin_inff();  // +inf of the one-med3 clamps (rmaxc; an opaque copy at KR = 4)
};

__device__ __forceinline__ float dv(float a, float b) { return div_rn(a, b); }
__device__ __forceinline__ double dv(double a, double b) { return a / b; }
__device__ __forceinline__ float pw(float x, float y, double* ln_x = nullptr, const PowK& K = pow_consts()) {
  return pow_pos(x, y, ln_x, K);
}
__device__ __forceinline__ double pw(double x, double y, double* ln_x = nullptr, const PowK& = pow_consts()) {
  if (ln_x) *ln_x = log(x);
  return pow(x, y);
}
__device__ __forceinline__ float rsqrt_(float a) { return sqrtf(a); }
__device__ __forceinline__ double rsqrt_(double a) { return sqrt(a); }

// Operation set of the physics: Fast = false is the bit-exact set above (forward); Fast = true is
// used by the fp32 adjoint's recompute and VJP, whose tolerance (gradients, 1e-4) allows hardware
// approximations: v_rcp_f32 division (~1.5 ulp), v_log_f32 / v_exp_f32 pow (~1e-6 relative),
// v_sqrt_f32.  The fp64 build always uses the exact set.
template <bool Fast>
__device__ __forceinline__ float dvf(float a, float b) {
  if constexpr (Fast) return a * __builtin_amdgcn_rcpf(b);
  else return div_rn(a, b);
}
template <bool Fast>
__device__ __forceinline__ double dvf(double a, double b) { return a / b; }
template <bool Fast>
__device__ __forceinline__ float pwf(float x, float y, double* ln_x = nullptr, const PowK& K = pow_consts()) {
  if constexpr (Fast) {
    const float l2 = __builtin_amdgcn_logf(x);  // log2 x
    if (ln_x) *ln_x = (double)(l2 * 0.69314718f);
    return __builtin_amdgcn_exp2f(y * l2);
  } else {
    return pow_pos(x, y, ln_x, K);
  }
}
template <bool Fast>
__device__ __forceinline__ double pwf(double x, double y, double* ln_x = nullptr, const PowK& = pow_consts()) {
  return pw(x, y, ln_x);
}
template <bool Fast>
__device__ __forceinline__ float sqf(float a) {
  if constexpr (Fast) return __builtin_amdgcn_sqrtf(a);
  else return sqrtf(a);
}
template <bool Fast>
__device__ __forceinline__ double sqf(double a) { return sqrt(a); }
// sqrt(1 + ss^2) of the wetted perimeter (argument >= 1): IEEE-rounded without the scaling path
__device__ __forceinline__ float sq1p(float a) { return sqrt_rn_normal(a); }
__device__ __forceinline__ double sq1p(double a) { return sqrt(a); }
template <bool Fast>
__device__ __forceinline__ float sqf1p(float a) {
  if constexpr (Fast) return __builtin_amdgcn_sqrtf(a);
  else return sqrt_rn_normal(a);
}
template <bool Fast>
__device__ __forceinline__ double sqf1p(double a) { return sqrt(a); }

template <typename R>
__device__ __forceinline__ R rmax(R a, R b) { return a > b ? a : b; }  // torch.clamp(min=) on finite
template <typename R>
__device__ __forceinline__ R rmin(R a, R b) { return a < b ? a : b; }
template <typename R>
__device__ __forceinline__ R rclamp(R x, R lo, R hi) { return rmin(rmax(x, lo), hi); }
// fp32: one v_med3_f32 each (equal to torch.clamp for the finite values of the physics)
__device__ __forceinline__ float rmax(float a, float b) { return __builtin_amdgcn_fmed3f(a, b, __builtin_inff()); }
__device__ __forceinline__ float rmin(float a, float b) { return __builtin_amdgcn_fmed3f(a, b, -__builtin_inff()); }
// The same with the kernel's infinity (Consts::pinf): with a literal infinity the compiler turns med3(a, b, inf)
// into max(a, b) and, in IEEE mode, canonicalises both operands first (two extra v_max_f32 per clamp); the
// heavy-load kernels (KR = 4) hand it an infinity it cannot see through (opaque_inf, one VGPR), which keeps
// the single med3 -- C5 forward -1.5 %, C3 backward -3 %; at light load the extra VGPR costs more than the
// instructions save, so those kernels keep the literal (profiles/r05/ab_r05.txt)
__device__ __forceinline__ float opaque_inf(float v) {
  asm("" : "+v"(v));  // not volatile: hoisted out of loops like any pure value
  return v;
}
template <typename C>
__device__ __forceinline__ float rmaxc(float a, float b, const C& c) { return __builtin_amdgcn_fmed3f(a, b, c.pinf); }
template <typename C>
__device__ __forceinline__ double rmaxc(double a, double b, const C&) { return rmax(a, b); }
__device__ __forceinline__ float rclamp(float x, float lo, float hi) { return __builtin_amdgcn_fmed3f(x, lo, hi); }

// torch.clamp(min=) with its NaN propagation (v_med3_f32 would return the bound for a NaN): used for
// the routed state and the outputs, so that a failed hand-off's NaN reaches the caller.
template <typename R>
__device__ __forceinline__ R rmax_nan(R x, R lb) { return x < lb ? lb : x; }

// torch: pow(R, 2 / 3) -- the Python double 2/3 is rounded to the tensor dtype.
template <typename R>
__device__ __forceinline__ R two_thirds() { return R(2.0 / 3.0); }

// Per-reach static quantities, computed once per launch exactly as the reference computes them
// at every step (they do not depend on the step).
template <typename R>
struct ReachStatic {
  R n;       // Manning n
  R qe;      // q_spatial + 1e-6                   (trapezoidal.py:62)
  R p;       // p_spatial
  R sqrtS;   // pow(slope, 0.5) == sqrt(slope)      (trapezoidal.py:66, 97)
  R dd;      // p * sqrtS + 1e-8                    (trapezoidal.py:66, 70)
  R expo;    // 3 / (5 + 3 qe)                      (trapezoidal.py:71)
  R inv_n;   // 1 / n                               (trapezoidal.py:97)
  R L;       // length
  R X;       // Muskingum X
  // qe + 1 (trapezoidal.py:65) and 1 - X (mmc.py:480) are recomputed where used (same rounding)
  __device__ __forceinline__ R qe1() const { return qe + R(1); }
  __device__ __forceinline__ R omX() const { return R(1) - X; }
};

// The six stored fields (n, qe, p, sqrtS, L, X) -> the derived ones.  The routing kernels keep only
// the stored fields (in LDS) and call this every tick; the operations are the same as at
// construction, so the values are identical.
template <typename R, bool Fast = false>
__device__ __forceinline__ ReachStatic<R> derive_static(R n, R qe, R p, R sqrtS, R L, R X) {
  ReachStatic<R> s;
  s.n = n;
  s.qe = qe;
  s.p = p;
  s.sqrtS = sqrtS;
  s.dd = (p * sqrtS) + R(1e-8);
  s.expo = dvf<Fast>(R(3), R(5) + R(3) * qe);
  s.inv_n = dvf<Fast>(R(1), n);
  s.L = L;
  s.X = X;
  return s;
}

template <typename R>
__device__ __forceinline__ ReachStatic<R> make_static(R n, R q, R p, R S, R L, R X) {
  return derive_static<R>(n, q + R(1e-6), p, rsqrt_(S), L, X);
}

// Forward intermediates kept for the VJP.
template <typename R>
struct Geom {
  R ratio, pw, depth, dq, tw, ssr, ss, bwr, bw, area, sq, wp, Rh, r23, v, cel, twok, den, ln_ratio, ln_depth;
};

template <typename R, bool Fast = false>
__device__ __forceinline__ void coefficients(const ReachStatic<R>& s, R Q, const Consts<R>& c,
                                             R& c1, R& c2, R& c3, R& c4, R& tw_out, R& ss_out,
                                             Geom<R>* gk = nullptr) {
  double ln_ratio = 0.0, ln_depth = 0.0;
  const R num = (Q * s.n) * s.qe1();
  const R ratio = dvf<Fast>(num, s.dd);
  const R pwv = pwf<Fast>(ratio, s.expo, gk ? &ln_ratio : nullptr, c.pk);
  const R depth = rmaxc(pwv, c.dlb, c);
  const R dq = pwf<Fast>(depth, s.qe, gk ? &ln_depth : nullptr, c.pk);
  const R tw = s.p * dq;
  const R ssr = dvf<Fast>(tw * s.qe, R(2) * depth);
  const R ss = rclamp(ssr, c.sslb, c.ssub);
  const R bwr = tw - (R(2) * ss) * depth;
  const R bw = rmaxc(bwr, c.bwlb, c);
  const R area = ((tw + bw) * depth) * R(0.5);  // x / 2 == x * 0.5 exactly
  const R sq = sqf1p<Fast>(R(1) + ss * ss);
  const R wp = bw + (R(2) * depth) * sq;
  const R Rh = dvf<Fast>(area, wp);
  const R r23 = pwf<Fast>(Rh, two_thirds<R>(), nullptr, c.pk);
  const R v = (s.inv_n * r23) * s.sqrtS;
  const R vc = rclamp(v, c.vlb, c.vub);
  const R cel = dvf<Fast>(vc * R(5), R(3));
  const R k = dvf<Fast>(s.L, cel);
  const R twok = R(2) * k;
  const R omX = s.omX();
  const R den = (twok * omX) + c.dt;
  c1 = dvf<Fast>(c.dt - twok * s.X, den);
  c2 = dvf<Fast>(c.dt + twok * s.X, den);
  c3 = dvf<Fast>((twok * omX) - c.dt, den);
  c4 = dvf<Fast>(R(2) * c.dt, den);
  tw_out = tw;
  ss_out = ss;
  if (gk) {
    gk->ratio = ratio; gk->pw = pwv; gk->depth = depth; gk->dq = dq; gk->tw = tw; gk->ssr = ssr;
    gk->ss = ss; gk->bwr = bwr; gk->bw = bw; gk->area = area; gk->sq = sq; gk->wp = wp; gk->Rh = Rh;
    gk->r23 = r23; gk->v = v; gk->cel = cel; gk->twok = twok; gk->den = den;
    gk->ln_ratio = R(ln_ratio); gk->ln_depth = R(ln_depth);
  }
}

// Lockstep form of coefficients<R> (forward, exact operation set) for NP reaches: every operation
// is issued for all NP reaches before the next, so a wave runs NP independent chains.
template <typename R>
struct PhysOut {
  R c1, c2, c3, c4, tw, ss;
};
template <int NP>
__device__ __forceinline__ void dv_np(const float (&a)[NP], const float (&b)[NP], float (&q)[NP]) { div_rn_np<NP>(a, b, q); }
template <int NP>
__device__ __forceinline__ void dv_np(const double (&a)[NP], const double (&b)[NP], double (&q)[NP]) {
  DDR_FOR_NP q[h] = a[h] / b[h];
}
template <int NP>
__device__ __forceinline__ void pw_np(const float (&x)[NP], const float (&y)[NP], float (&o)[NP], const PowK& K) {
  pow_pos_np<NP>(x, y, o, K);
}
template <int NP>
__device__ __forceinline__ void pw_np(const double (&x)[NP], const double (&y)[NP], double (&o)[NP], const PowK&) {
  DDR_FOR_NP o[h] = pow(x[h], y[h]);
}

template <typename R, int NP>
__device__ __forceinline__ void coefficients_np(const ReachStatic<R> (&s)[NP], const R (&Q)[NP], const Consts<R>& c,
                                                PhysOut<R> (&o)[NP]) {
  R a[NP], b[NP], ratio[NP], depth[NP], dq[NP], e[NP], ssr[NP], ss[NP], bw[NP], area[NP], wp[NP], Rh[NP],
      r23[NP], twok[NP], den[NP];
  DDR_FOR_NP a[h] = (Q[h] * s[h].n) * s[h].qe1();
  DDR_FOR_NP b[h] = s[h].dd;
  dv_np<NP>(a, b, ratio);
  if constexpr (std::is_same<R, float>::value) {
    // pw = ratio^expo and dq = depth^qe share one logarithm: for depth = pw, ln(pw) is derived from
    // the exponent z = expo ln(ratio) and the fp64 value E of the first pow, ln(pw) = z + ln(pw / E)
    // with |pw / E - 1| < 2^-24 (two terms of log1p); for depth = d_lb the constant ln(d_lb).
    double l[NP], z[NP], E[NP];
    ln_np<NP>(ratio, l, c.pk);
    DDR_FOR_NP z[h] = (double)s[h].expo * l[h];
    exp_np<NP>(z, E, c.pk);
    DDR_FOR_NP {
      const float pw = (float)E[h];
      depth[h] = rmaxc(pw, c.dlb, c);
      const double u = ((double)pw - E[h]) * __builtin_amdgcn_rcp(E[h]);
      l[h] = (pw >= c.dlb) ? z[h] + fma(-0.5 * u, u, u) : c.ln_dlb;
      z[h] = (double)s[h].qe * l[h];
    }
    exp_np<NP>(z, E, c.pk);
    DDR_FOR_NP dq[h] = (float)E[h];
  } else {
    DDR_FOR_NP e[h] = s[h].expo;
    pw_np<NP>(ratio, e, depth, c.pk);
    DDR_FOR_NP depth[h] = rmaxc(depth[h], c.dlb, c);
    DDR_FOR_NP e[h] = s[h].qe;
    pw_np<NP>(depth, e, dq, c.pk);
  }
  DDR_FOR_NP o[h].tw = s[h].p * dq[h];
  DDR_FOR_NP a[h] = o[h].tw * s[h].qe;
  DDR_FOR_NP b[h] = R(2) * depth[h];
  dv_np<NP>(a, b, ssr);
  DDR_FOR_NP ss[h] = rclamp(ssr[h], c.sslb, c.ssub);
  DDR_FOR_NP o[h].ss = ss[h];
  DDR_FOR_NP bw[h] = rmaxc(o[h].tw - (R(2) * ss[h]) * depth[h], c.bwlb, c);
  DDR_FOR_NP area[h] = ((o[h].tw + bw[h]) * depth[h]) * R(0.5);
  DDR_FOR_NP a[h] = sq1p(R(1) + ss[h] * ss[h]);
  DDR_FOR_NP wp[h] = bw[h] + (R(2) * depth[h]) * a[h];
  dv_np<NP>(area, wp, Rh);
  DDR_FOR_NP e[h] = two_thirds<R>();
  pw_np<NP>(Rh, e, r23, c.pk);
  DDR_FOR_NP a[h] = rclamp((s[h].inv_n * r23[h]) * s[h].sqrtS, c.vlb, c.vub) * R(5);
  DDR_FOR_NP b[h] = R(3);
  dv_np<NP>(a, b, e);                                  // celerity
  DDR_FOR_NP a[h] = s[h].L;
  dv_np<NP>(a, e, b);                                  // k = L / c
  DDR_FOR_NP twok[h] = R(2) * b[h];
  DDR_FOR_NP den[h] = (twok[h] * s[h].omX()) + c.dt;
  DDR_FOR_NP a[h] = c.dt - twok[h] * s[h].X;
  dv_np<NP>(a, den, b);
  DDR_FOR_NP o[h].c1 = b[h];
  DDR_FOR_NP a[h] = c.dt + twok[h] * s[h].X;
  dv_np<NP>(a, den, b);
  DDR_FOR_NP o[h].c2 = b[h];
  DDR_FOR_NP a[h] = (twok[h] * s[h].omX()) - c.dt;
  dv_np<NP>(a, den, b);
  DDR_FOR_NP o[h].c3 = b[h];
  DDR_FOR_NP a[h] = R(2) * c.dt;
  dv_np<NP>(a, den, b);
  DDR_FOR_NP o[h].c4 = b[h];
}

// Hardware-approximate fp32 form of coefficients_np (v_rcp / v_log / v_exp / v_rsq, the operation
// set of the adjoint's recompute, adjoint_step_fast): ~1e-6 relative per coefficient.
__device__ __forceinline__ PhysOut<float> coefficients_fast(const ReachStatic<float>& s, float Q, const Consts<float>& c) {
  const float qe = s.qe;
  const float ratio = ((Q * s.n) * (qe + 1.0f)) * __builtin_amdgcn_rcpf(s.dd);
  const float pw = __builtin_amdgcn_exp2f(s.expo * __builtin_amdgcn_logf(ratio));
  const float depth = rmaxc(pw, c.dlb, c);
  const float dq = __builtin_amdgcn_exp2f(qe * __builtin_amdgcn_logf(depth));
  PhysOut<float> o;
  o.tw = s.p * dq;
  const float td = depth + depth;
  const float ssr = (o.tw * qe) * __builtin_amdgcn_rcpf(td);
  o.ss = rclamp(ssr, c.sslb, c.ssub);
  const float bw = rmaxc(o.tw - (o.ss + o.ss) * depth, c.bwlb, c);
  const float area = ((o.tw + bw) * depth) * 0.5f;
  const float u = fmaf(o.ss, o.ss, 1.0f);
  const float wp = fmaf(td, u * __builtin_amdgcn_rsqf(u), bw);
  const float Rh = area * __builtin_amdgcn_rcpf(wp);
  const float r23 = __builtin_amdgcn_exp2f(__builtin_amdgcn_logf(Rh) * (2.0f / 3.0f));
  const float cel = rclamp((s.inv_n * r23) * s.sqrtS, c.vlb, c.vub) * (5.0f / 3.0f);
  const float twok = 2.0f * (s.L * __builtin_amdgcn_rcpf(cel));
  const float rden = __builtin_amdgcn_rcpf(fmaf(twok, 1.0f - s.X, c.dt));
  const float tX = twok * s.X;
  o.c1 = (c.dt - tX) * rden;
  o.c2 = (c.dt + tX) * rden;
  o.c4 = (2.0f * c.dt) * rden;
  o.c3 = 1.0f - o.c4;
  return o;
}

// The reference's operation sequence (coefficients_np) with IEEE divisions (div_rn) and square
// root, and the pows in fp32 faithful-class arithmetic (pow_faithful) instead of fp64: no fp64
// instruction and no table lookup on the forward's dependency chain.
__device__ __forceinline__ PhysOut<float> coefficients_faithful(const ReachStatic<float>& s, float Q,
                                                                const Consts<float>& c) {
  PhysOut<float> o;
  const float ratio = div_rn((Q * s.n) * s.qe1(), s.dd);
  const float depth = rmaxc(pow_faithful(ratio, s.expo), c.dlb, c);
  const float dq = pow_faithful(depth, s.qe);
  o.tw = s.p * dq;
  const float ssr = div_rn(o.tw * s.qe, 2.0f * depth);
  o.ss = rclamp(ssr, c.sslb, c.ssub);
  const float bw = rmaxc(o.tw - (2.0f * o.ss) * depth, c.bwlb, c);
  const float area = ((o.tw + bw) * depth) * 0.5f;
  const float wp = bw + (2.0f * depth) * sqrt_rn_normal(1.0f + o.ss * o.ss);
  const float Rh = div_rn(area, wp);
  const float r23 = pow_faithful(Rh, two_thirds<float>());
  const float cel = div_rn(rclamp((s.inv_n * r23) * s.sqrtS, c.vlb, c.vub) * 5.0f, 3.0f);
  const float twok = 2.0f * div_rn(s.L, cel);
  const float den = (twok * s.omX()) + c.dt;
  o.c1 = div_rn(c.dt - twok * s.X, den);
  o.c2 = div_rn(c.dt + twok * s.X, den);
  o.c3 = div_rn((twok * s.omX()) - c.dt, den);
  o.c4 = div_rn(2.0f * c.dt, den);
  return o;
}

// VJP of (c1, c2, c3, c4) w.r.t. (Q, n, q_spatial, p_spatial) at the point described by g.
template <typename R, bool Fast = false>
__device__ __forceinline__ void coefficients_vjp(const ReachStatic<R>& s, R Q, const Consts<R>& c,
                                                 const Geom<R>& g, R c1, R c2, R c3, R c4, R gc1,
                                                 R gc2, R gc3, R gc4, R& gQ, R& gn, R& gq, R& gp) {
  // c_k(twok): d c1 = (-X - c1 (1-X)) / den, d c2 = (X - c2 (1-X)) / den,
  //            d c3 = (1-X)(1 - c3) / den,   d c4 = -c4 (1-X) / den
  const R omX = s.omX();
  const R g_twok = dvf<Fast>(gc1 * (-s.X - c1 * omX) + gc2 * (s.X - c2 * omX) + gc3 * omX * (R(1) - c3) -
                          gc4 * c4 * omX, g.den);
  const R k = g.twok * R(0.5);
  const R g_k = R(2) * g_twok;
  const R g_cel = dvf<Fast>(-g_k * k, g.cel);
  const bool vin = (g.v >= c.vlb) && (g.v <= c.vub);
  const R g_v = vin ? g_cel * dvf<Fast>(R(5), R(3)) : R(0);
  // v = inv_n * R^(2/3) * sqrtS
  const R g_Rh = dvf<Fast>(g_v * s.inv_n * s.sqrtS * two_thirds<R>() * g.r23, g.Rh);
  R g_n = -g_v * g.v * s.inv_n;
  // Rh = area / wp
  const R g_area = dvf<Fast>(g_Rh, g.wp);
  const R g_wp = dvf<Fast>(-g_Rh * g.Rh, g.wp);
  // wp = bw + 2 depth sq
  R g_bw = g_wp;
  R g_depth = g_wp * R(2) * g.sq;
  R g_ss = dvf<Fast>(g_wp * R(2) * g.depth * g.ss, g.sq);
  // area = (tw + bw) depth / 2
  R g_tw = g_area * g.depth * R(0.5);
  g_bw += g_area * g.depth * R(0.5);
  g_depth += g_area * (g.tw + g.bw) * R(0.5);
  // bw = max(tw - 2 ss depth, bw_lb)
  const R g_bwr = (g.bwr >= c.bwlb) ? g_bw : R(0);
  g_tw += g_bwr;
  g_ss -= R(2) * g.depth * g_bwr;
  g_depth -= R(2) * g.ss * g_bwr;
  // ss = clamp(tw qe / (2 depth))
  const R g_ssr = (g.ssr >= c.sslb && g.ssr <= c.ssub) ? g_ss : R(0);
  const R inv2d = dvf<Fast>(R(1), R(2) * g.depth);
  g_tw += g_ssr * s.qe * inv2d;
  R g_qe = g_ssr * g.tw * inv2d;
  g_depth -= g_ssr * g.ssr * R(2) * inv2d;
  // tw = p depth^qe
  R g_p = g_tw * g.dq;
  g_depth += g_tw * g.tw * s.qe * R(2) * inv2d;
  g_qe += g_tw * g.tw * g.ln_depth;
  // depth = max(pw, d_lb)
  const R g_pw = (g.pw >= c.dlb) ? g_depth : R(0);
  // pw = ratio^e ; e = 3 / (5 + 3 qe), de/dqe = -9 / (5 + 3qe)^2 = -e^2
  const R g_ratio = dvf<Fast>(g_pw * s.expo * g.pw, g.ratio);
  const R g_e = g_pw * g.pw * g.ln_ratio;
  g_qe -= g_e * s.expo * s.expo;
  // ratio = num / (p sqrtS + 1e-8)
  const R g_num = dvf<Fast>(g_ratio, s.dd);
  g_p -= dvf<Fast>(g_ratio * g.ratio, s.dd) * s.sqrtS;
  // num = Q n (qe + 1)
  const R qe1 = s.qe1();
  gQ = g_num * s.n * qe1;
  g_n += g_num * Q * qe1;
  g_qe += g_num * Q * s.n;
  gn = g_n;
  gq = g_qe;
  gp = g_p;
}

// ---- fp32 adjoint step (backward kernel, fp32 build): the step's physics recomputed in hardware
// fp32 math and its VJP, folded algebraically.  Equivalent in exact arithmetic to
// coefficients<float, true> + coefficients_vjp<float, true>; per reach-step ~15 transcendental and
// ~90 other instructions.
// dL/d(2k) = sum_k gc_k dc_k/d(2k) is a sum of O(Q) terms that cancels to O(dQ/dt) (its exact value is
// gb / den [X (I - Sx) + (1 - X)(Q - x~)], x~ = c1 Sx + c2 I + c3 Q + c4 qc).  With c1 + c2 = c4 = 1 - c3 it is
//   gb / den [D1 (X + (1 - X) c1) + D2 ((1 - X) c2 - X)],   D1 = Q - qc - Sx,  D2 = Q - qc - I,
// where the coefficients multiply the step's mass imbalances D1, D2 (DF: formed exactly in fp64 by the caller
// from the fp32 states; a1 = D1, a2 = D2), so their ~1e-6 recompute error stays ~1e-6 of the result.  The default
// (a1 = x(t), a2 = Sx, a3 = I) takes Q - x~ from the stored fp32 x(t) -- no q' re-read -- which carries the
// forward's rounding of x (~1e-7 Q) into a quantity of size dQ: 1.6e-3 / 4.7e-3 / 2.4e-3 of the gradient on a
// 2215-deep basin, ~1e-7 on shallow trees (tools/grad_terms.py; DDR_BWD_EXACT_ADJOINT).
struct AdjOut {
  float c1, c2, c3, c4, gQ, gn, gq, gp;
};
template <bool DF>
__device__ __forceinline__ AdjOut adjoint_step_fast(const ReachStatic<float>& s, float Q, const Consts<float>& c,
                                                    float gb, float a1, float a2, float a3) {
  constexpr float kLn2 = 0.69314718055994530942f;
  const float qe = s.qe, qe1 = qe + 1.0f, expo = s.expo;
  // ---- recompute (geometry/trapezoidal.py:62-97, routing/mmc.py:165-167, 479-484) ----
  const float num = (Q * s.n) * qe1;
  const float rdd = __builtin_amdgcn_rcpf(s.dd);
  const float ratio = num * rdd;
  const float l2r = __builtin_amdgcn_logf(ratio);
  const float pw = __builtin_amdgcn_exp2f(expo * l2r);
  const float depth = rmaxc(pw, c.dlb, c);
  const float l2d = __builtin_amdgcn_logf(depth);
  const float dq = __builtin_amdgcn_exp2f(qe * l2d);
  const float tw = s.p * dq;
  const float td = depth + depth;
  const float rtd = __builtin_amdgcn_rcpf(td);
  const float ssr = (tw * qe) * rtd;
  const float ss = rclamp(ssr, c.sslb, c.ssub);
  const float bwr = tw - (ss + ss) * depth;
  const float bw = rmaxc(bwr, c.bwlb, c);
  const float area = ((tw + bw) * depth) * 0.5f;
  const float u = fmaf(ss, ss, 1.0f);
  const float isq = __builtin_amdgcn_rsqf(u);
  const float sq = u * isq;
  const float wp = fmaf(td, sq, bw);
  const float rwp = __builtin_amdgcn_rcpf(wp);
  const float Rh = area * rwp;
  const float r23 = __builtin_amdgcn_exp2f(__builtin_amdgcn_logf(Rh) * (2.0f / 3.0f));
  const float v = (s.inv_n * r23) * s.sqrtS;
  const float cel = rclamp(v, c.vlb, c.vub) * (5.0f / 3.0f);
  const float rcel = __builtin_amdgcn_rcpf(cel);
  const float twok = 2.0f * (s.L * rcel);
  const float omX = 1.0f - s.X;
  const float den = fmaf(twok, omX, c.dt);
  const float rden = __builtin_amdgcn_rcpf(den);
  const float tX = twok * s.X;
  AdjOut o;
  o.c1 = (c.dt - tX) * rden;
  o.c2 = (c.dt + tX) * rden;
  const float c4 = (2.0f * c.dt) * rden;
  o.c3 = 1.0f - c4;
  o.c4 = c4;
  // ---- VJP: gc = gb (Sx, I, Q, qc) ----
  const float g_twok = DF ? (gb * fmaf(a1, fmaf(omX, o.c1, s.X), a2 * fmaf(omX, o.c2, -s.X))) * rden
                          : gb * fmaf(s.X, a3 - a2, omX * (Q - a1)) * rden;
  const float g_cel = -(g_twok * twok) * rcel;                    // k = L / cel
  const bool vin = (v >= c.vlb) && (v <= c.vub);
  const float gvv = vin ? (g_cel * (5.0f / 3.0f)) * v : 0.0f;     // dL/d ln v
  float g_n = -gvv * s.inv_n;
  const float G = gvv * (2.0f / 3.0f);                            // dL/d ln Rh
  const float g_area = G * __builtin_amdgcn_rcpf(area);
  const float g_wp = -G * rwp;
  // wp = bw + 2 depth sq ; area = (tw + bw) depth / 2
  const float ha = (g_area * depth) * 0.5f;
  float g_bw = g_wp + ha;
  float g_tw = ha;
  float g_depth = fmaf(2.0f * sq, g_wp, (G + G) * rtd);             // + G / depth
  float g_ss = ((td * g_wp) * ss) * isq;
  // bw = max(tw - 2 ss depth, bw_lb)
  const float g_bwr = (bwr >= c.bwlb) ? g_bw : 0.0f;
  g_tw += g_bwr;
  g_ss = fmaf(-td, g_bwr, g_ss);
  g_depth = fmaf(-(ss + ss), g_bwr, g_depth);
  // ss = clamp(tw qe / (2 depth))
  const float g_ssr = (ssr >= c.sslb && ssr <= c.ssub) ? g_ss : 0.0f;
  const float gsr = g_ssr * rtd;
  g_tw = fmaf(gsr, qe, g_tw);
  float g_qe = gsr * tw;
  g_depth = fmaf(-(g_ssr + g_ssr) * ssr, rtd, g_depth);
  // tw = p depth^qe
  float g_p = g_tw * dq;
  const float gtt = g_tw * tw;
  g_depth = fmaf((gtt + gtt) * qe, rtd, g_depth);
  g_qe = fmaf(gtt * kLn2, l2d, g_qe);
  // depth = max(ratio^expo, d_lb)
  const float g_pw = (pw >= c.dlb) ? g_depth : 0.0f;
  const float A = (g_pw * expo) * pw;                              // dL/d ln ratio
  g_qe = fmaf(-((g_pw * pw) * (l2r * kLn2)), expo * expo, g_qe);   // d expo / d qe = -expo^2
  // ratio = Q n (qe + 1) / (p sqrtS + 1e-8)
  o.gQ = A * __builtin_amdgcn_rcpf(Q);
  g_n = fmaf(A, s.inv_n, g_n);
  g_qe = fmaf(A, __builtin_amdgcn_rcpf(qe1), g_qe);
  g_p = fmaf(-A * s.sqrtS, rdd, g_p);
  o.gn = g_n;
  o.gq = g_qe;
  o.gp = g_p;
  return o;
}

}  // namespace ddr
