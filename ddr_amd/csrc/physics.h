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

#include "fastmath.h"

namespace ddr {

template <typename R>
struct Consts {
  R dt, qlb, vlb, vub, dlb, bwlb, sslb, ssub;
};

__device__ __forceinline__ float dv(float a, float b) { return div_rn(a, b); }
__device__ __forceinline__ double dv(double a, double b) { return a / b; }
__device__ __forceinline__ float pw(float x, float y, double* ln_x = nullptr) { return pow_pos(x, y, ln_x); }
__device__ __forceinline__ double pw(double x, double y, double* ln_x = nullptr) {
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
__device__ __forceinline__ float pwf(float x, float y, double* ln_x = nullptr) {
  if constexpr (Fast) {
    const float l2 = __builtin_amdgcn_logf(x);  // log2 x
    if (ln_x) *ln_x = (double)(l2 * 0.69314718f);
    return __builtin_amdgcn_exp2f(y * l2);
  } else {
    return pow_pos(x, y, ln_x);
  }
}
template <bool Fast>
__device__ __forceinline__ double pwf(double x, double y, double* ln_x = nullptr) { return pw(x, y, ln_x); }
template <bool Fast>
__device__ __forceinline__ float sqf(float a) {
  if constexpr (Fast) return __builtin_amdgcn_sqrtf(a);
  else return sqrtf(a);
}
template <bool Fast>
__device__ __forceinline__ double sqf(double a) { return sqrt(a); }

template <typename R>
__device__ __forceinline__ R rmax(R a, R b) { return a > b ? a : b; }  // torch.clamp(min=) on finite
template <typename R>
__device__ __forceinline__ R rmin(R a, R b) { return a < b ? a : b; }

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
  const R pwv = pwf<Fast>(ratio, s.expo, gk ? &ln_ratio : nullptr);
  const R depth = rmax(pwv, c.dlb);
  const R dq = pwf<Fast>(depth, s.qe, gk ? &ln_depth : nullptr);
  const R tw = s.p * dq;
  const R ssr = dvf<Fast>(tw * s.qe, R(2) * depth);
  const R ss = rmin(rmax(ssr, c.sslb), c.ssub);
  const R bwr = tw - (R(2) * ss) * depth;
  const R bw = rmax(bwr, c.bwlb);
  const R area = ((tw + bw) * depth) * R(0.5);  // x / 2 == x * 0.5 exactly
  const R sq = sqf<Fast>(R(1) + ss * ss);
  const R wp = bw + (R(2) * depth) * sq;
  const R Rh = dvf<Fast>(area, wp);
  const R r23 = pwf<Fast>(Rh, two_thirds<R>());
  const R v = (s.inv_n * r23) * s.sqrtS;
  const R vc = rmin(rmax(v, c.vlb), c.vub);
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

}  // namespace ddr
