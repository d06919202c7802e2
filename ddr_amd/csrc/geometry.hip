// Per-reach temporal statistics of the trapezoid geometry over daily accumulated discharge
// (reference src/ddr/geometry/statistics.py:20-83, driven by scripts/geometry_predictor.py:193-212).
//
// One wave per reach.  Lane l holds days l, l + 64, ..., (KD per lane, D <= 64 KD).  The wave sorts the
// discharges once (bitonic network: lane shuffles for partners in other lanes, register swaps for
// partners in the same lane), evaluates the geometry (geometry/trapezoidal.py:62-97 in the routing
// kernels' exact operation order, physics.h) at the sorted discharges, and emits min, max, median and
// mean of each of the six variables (depth, top width, bottom width, side slope, hydraulic radius,
// discharge) from fixed positions where the variable is monotone in Q, else after sorting it.  NaN values are skipped like numpy's nanmin / nanmax / nanmedian / nanmean (a reach with
// no valid day gets NaN).  The mean is accumulated in fp64 (numpy's pairwise fp32 sum differs in the
// last bits).  Windows longer than 512 days (multi-year runs) take geometry_stats_long_kernel: one
// workgroup per reach, the values sorted in LDS (up to kGeoLongMaxDays days).
#include "internal.h"
#include "physics.h"

namespace ddr {

namespace {

constexpr int kGeoVars = 6;   // depth, top_width, bottom_width, side_slope, hydraulic_radius, discharge
constexpr int kGeoStats = 4;  // min, max, median, mean

struct GeoArgs {
  const float* qd;   // accumulated discharge, element (reach, day) at reach * rs + day * ds
  int64_t rs, ds;
  int64_t N, D;
  const float* n;
  const float* p;
  int64_t p_stride;
  const float* q;
  const float* S;    // slope, already clamped
  float depth_lb, bw_lb;
  float* out;        // (kGeoVars * kGeoStats, N)
};

__device__ __forceinline__ float shfl_xor_f(float v, int m) {
  return __shfl_xor(v, m, 64);
}

// v of lane ^ J, J a power of two < 64, without the LDS crossbar where a DPP pattern exists (each
// ds_bpermute is an LDS round trip the bitonic stages then wait for): J = 1, 2 quad permutes; 4 a half-row
// mirror then a quad reverse ((l ^ 7) ^ 3 = l ^ 4); 8 a row rotate by 8; 16 a swizzle swap; 32 the
// gfx950 permlane32 swap
template <int J>
__device__ __forceinline__ float xor_lane(float v) {
  const int iv = __float_as_int(v);
  if constexpr (J == 1) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(iv, 0xB1, 0xF, 0xF, true));  // quad_perm [1,0,3,2]
  } else if constexpr (J == 2) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(iv, 0x4E, 0xF, 0xF, true));  // quad_perm [2,3,0,1]
  } else if constexpr (J == 4) {
    const int m = __builtin_amdgcn_mov_dpp(iv, 0x141, 0xF, 0xF, true);        // row_half_mirror
    return __int_as_float(__builtin_amdgcn_mov_dpp(m, 0x1B, 0xF, 0xF, true));  // quad_perm [3,2,1,0]
  } else if constexpr (J == 8) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(iv, 0x128, 0xF, 0xF, true));  // row_ror:8
  } else if constexpr (J == 16) {
    return __int_as_float(__builtin_amdgcn_ds_swizzle(iv, 0x401F));  // swizzle(SWAP, 16)
  } else {
    static_assert(J == 32, "lane xor distance");
    const auto pr = __builtin_amdgcn_permlane32_swap(iv, iv, false, false);
    return __int_as_float((threadIdx.x & 32) ? pr[0] : pr[1]);
  }
}

// v of lane (lane + 1) & 63 (DPP wave_rol:1)
__device__ __forceinline__ float next_lane(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x134, 0xF, 0xF, true));
}
// the wave's sum of x (fp64; every lane gets it), by lane-xor exchanges of the two halves
template <int J>
__device__ __forceinline__ double xor_lane_d(double x) {
  const unsigned long long u = __double_as_longlong(x);
  const float lo = xor_lane<J>(__uint_as_float((unsigned)u));
  const float hi = xor_lane<J>(__uint_as_float((unsigned)(u >> 32)));
  return __longlong_as_double((long long)(((unsigned long long)__float_as_uint(hi) << 32) | __float_as_uint(lo)));
}
__device__ __forceinline__ double wave_sum(double x) {
  x += xor_lane_d<1>(x);
  x += xor_lane_d<2>(x);
  x += xor_lane_d<4>(x);
  x += xor_lane_d<8>(x);
  x += xor_lane_d<16>(x);
  x += xor_lane_d<32>(x);
  return x;
}
// number of lanes with p set
__device__ __forceinline__ int wave_count(bool p) { return __builtin_popcountll(__builtin_amdgcn_ballot_w64(p)); }

// Ascending bitonic sort of the wave's 64 * KD values, element e = i * 64 + lane in v[i].  Each
// compare-exchange is one v_med3_f32 per element: med3(a, b, -inf) = min, med3(a, b, +inf) = max (no NaN
// reaches the sort; a min / max pair plus a select, with the IEEE-mode canonicalisations fminf / fmaxf
// bring, cost 4-5 instructions), the partner in another lane fetched by xor_lane.
template <int KD>
__device__ __forceinline__ void wave_sort(float (&v)[KD], int lane) {
  constexpr int M = 64 * KD;
  const float ninf = -__builtin_inff(), pinf = __builtin_inff();
#pragma unroll
  for (int k = 2; k <= M; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= 64) {
        const int jj = j >> 6;
#pragma unroll
        for (int i = 0; i < KD; ++i) {
          if (i & jj) continue;
          const bool asc = ((i * 64) & k) == 0;  // (k >= 128 here: the lane does not enter)
          const float a = v[i], b = v[i | jj];
          v[i] = __builtin_amdgcn_fmed3f(a, b, asc ? ninf : pinf);
          v[i | jj] = __builtin_amdgcn_fmed3f(a, b, asc ? pinf : ninf);
        }
      } else {
        const bool lower = (lane & j) == 0;
        // every partner fetched before the first exchange: a DPP read of a register the previous VALU
        // instruction wrote needs wait states (s_nop) the stage's other elements fill instead
        float o[KD];
#pragma unroll
        for (int i = 0; i < KD; ++i) {
          switch (j) {  // (j is a compile-time constant of the unrolled loop)
            case 1: o[i] = xor_lane<1>(v[i]); break;
            case 2: o[i] = xor_lane<2>(v[i]); break;
            case 4: o[i] = xor_lane<4>(v[i]); break;
            case 8: o[i] = xor_lane<8>(v[i]); break;
            case 16: o[i] = xor_lane<16>(v[i]); break;
            default: o[i] = xor_lane<32>(v[i]); break;
          }
        }
#pragma unroll
        for (int i = 0; i < KD; ++i) {
          const int e = i * 64 + lane;
          const bool asc = (e & k) == 0;
          v[i] = __builtin_amdgcn_fmed3f(v[i], o[i], (lower == asc) ? ninf : pinf);
        }
      }
    }
  }
}

// Ascending sort of 64 * KD values of which only the first KE slots can be finite (slots KE.. are +inf
// padding): KD = 8, KE = 6 (a 365-day year) sorts slots 0-3 and 4-5 separately, lays the second run out
// descending behind 128 padding values (a bitonic sequence) and merges -- 272 slot-stages instead of the
// full network's 360.  Other shapes take the full network.
template <int KD, int KE>
__device__ __forceinline__ void wave_sort_valid(float (&v)[KD], int lane) {
  if constexpr (KD == 8 && KE == 6) {
    const float pinf = __builtin_inff(), ninf = -__builtin_inff();
    float lo[4] = {v[0], v[1], v[2], v[3]};
    float hi[2] = {-v[4], -v[5]};  // ascending -w is descending w (+inf padding first)
    wave_sort<4>(lo, lane);
    wave_sort<2>(hi, lane);
    v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
    v[4] = pinf; v[5] = pinf; v[6] = -hi[0]; v[7] = -hi[1];
    // bitonic merge (ascending) of the 512-element bitonic sequence
#pragma unroll
    for (int j = 256; j >= 64; j >>= 1) {
      const int jj = j >> 6;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (i & jj) continue;
        const float a = v[i], b = v[i | jj];
        v[i] = __builtin_amdgcn_fmed3f(a, b, ninf);
        v[i | jj] = __builtin_amdgcn_fmed3f(a, b, pinf);
      }
    }
#pragma unroll
    for (int j = 32; j > 0; j >>= 1) {
      const bool lower = (lane & j) == 0;
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        switch (j) {
          case 1: o[i] = xor_lane<1>(v[i]); break;
          case 2: o[i] = xor_lane<2>(v[i]); break;
          case 4: o[i] = xor_lane<4>(v[i]); break;
          case 8: o[i] = xor_lane<8>(v[i]); break;
          case 16: o[i] = xor_lane<16>(v[i]); break;
          default: o[i] = xor_lane<32>(v[i]); break;
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = __builtin_amdgcn_fmed3f(v[i], o[i], lower ? ninf : pinf);
    }
  } else {
    wave_sort<KD>(v, lane);
  }
}

// Element `idx` (wave-uniform) of the sorted values.
template <int KD>
__device__ __forceinline__ float wave_elem(const float (&v)[KD], int idx) {
  const int i = idx >> 6, l = idx & 63;
  float r = v[0];
#pragma unroll
  for (int k = 1; k < KD; ++k)
    if (i == k) r = v[k];
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r), l));  // (idx is wave-uniform)
}

// The trapezoid geometry of one day (trapezoidal.py:62-97): coefficients<float, false>'s operations, in its
// order, up to the hydraulic radius -- the statistics need no velocity and no Muskingum coefficients
// (one pow and six divisions fewer per day than the routing step).  Bit-identical to the values
// coefficients() computes on the way.
struct DayGeom {
  float depth, tw, bw, ss, Rh;
};
__device__ __forceinline__ DayGeom day_geometry(const ReachStatic<float>& s, float Q, const Consts<float>& c) {
  DayGeom g;
  const float num = (Q * s.n) * s.qe1();
  const float ratio = dvf<false>(num, s.dd);
  const float pwv = pwf<false>(ratio, s.expo, nullptr, c.pk);
  g.depth = rmax(pwv, c.dlb);
  const float dq = pwf<false>(g.depth, s.qe, nullptr, c.pk);
  g.tw = s.p * dq;
  const float ssr = dvf<false>(g.tw * s.qe, 2.0f * g.depth);
  g.ss = rclamp(ssr, c.sslb, c.ssub);
  const float bwr = g.tw - (2.0f * g.ss) * g.depth;
  g.bw = rmax(bwr, c.bwlb);
  const float area = ((g.tw + g.bw) * g.depth) * 0.5f;
  const float sq = sqrt_rn_normal(1.0f + g.ss * g.ss);
  const float wp = g.bw + (2.0f * g.depth) * sq;
  g.Rh = dvf<false>(area, wp);
  return g;
}

// The value of `var` (0 depth, 1 top width, 2 bottom width, 3 side slope, 4 hydraulic radius, 5 Q).
__device__ __forceinline__ float geom_var(const DayGeom& g, float Q, int var) {
  return var == 0 ? g.depth : (var == 1 ? g.tw : (var == 2 ? g.bw : (var == 3 ? g.ss : (var == 4 ? g.Rh : Q))));
}

// One wave per reach, days in Q order: the wave sorts the valid discharges once (bitonic, NaN last), then
// evaluates each day's geometry at the sorted Q (the geometry is a function of Q alone), so element e of
// every variable belongs to the e-th smallest discharge.  A variable whose values are monotone along that
// order (the common case: depth and top width are non-decreasing in Q, the others nearly always monotone
// over one reach's year) has its order statistics at fixed positions; the wave checks monotonicity on
// every adjacent pair and sorts only a variable that is not (or has a NaN where Q is valid).  Exact:
// the same min / max / median as a sort of every variable, in every case.  The mean is the fp64 sum of
// the valid values (fp32 values, so the order does not change it where the range stays within 2^29).
template <int KD, int KE>
__device__ __forceinline__ void geometry_stats_reach(const GeoArgs& a, int64_t reach, int lane);

// Persistent workgroups (the math tables are loaded once per workgroup, not once per 4 reaches) over groups
// of 4 consecutive reaches; the groups are dealt out XCD-major -- workgroup w runs on XCD w % 8 and walks a
// contiguous range of groups -- so that the reaches sharing a line of the (day, reach) discharge layout are
// read through one L2, not fetched once per XCD.
// KE = ceil(D / 64) <= KD: the slots that can hold a day (the sort pads to KD with +inf; everything after
// it works on the KE slots).
template <int KD, int KE>
__global__ void __launch_bounds__(256) geometry_stats_kernel(GeoArgs a) {
  load_math_tables();
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t groups = (a.N + 3) / 4;
  const int64_t nwg = gridDim.x;                 // a multiple of 8
  const int64_t per_xcd = nwg / 8;
  const int64_t xcd = blockIdx.x % 8, slot = blockIdx.x / 8;
  const int64_t span = (groups + 7) / 8;         // groups per XCD, contiguous
  const int64_t g0 = xcd * span, g1 = g0 + span < groups ? g0 + span : groups;
  for (int64_t grp = g0 + slot; grp < g1; grp += per_xcd) {
    const int64_t reach = grp * 4 + (threadIdx.x >> 6);
    if (reach < a.N) geometry_stats_reach<KD, KE>(a, reach, lane);
  }
}

template <int KD, int KE>
__device__ __forceinline__ void geometry_stats_reach(const GeoArgs& a, int64_t reach, int lane) {
  Consts<float> cs{};
  cs.dt = 3600.0f;
  cs.qlb = 0.0f;
  cs.vlb = 0.01f;
  cs.vub = 15.0f;
  cs.dlb = a.depth_lb;
  cs.bwlb = a.bw_lb;
  cs.sslb = 0.5f;
  cs.ssub = 50.0f;
  cs.pk = pow_consts();
  cs.ln_dlb = 0.0;
  // trapezoidal.py:62-66: the static part (no length / storage enter the geometry)
  const ReachStatic<float> st = make_static<float>(a.n[reach], a.q[reach], a.p[reach * a.p_stride], a.S[reach],
                                                   1.0f, 0.0f);
  float qv[KD];
  int cq = 0;
#pragma unroll
  for (int i = 0; i < KD; ++i) {
    const int64_t d = (int64_t)i * 64 + lane;
    const float Q = (i < KE && d < a.D) ? a.qd[reach * a.rs + d * a.ds] : __builtin_nanf("");
    const bool valid = Q == Q;  // torch propagates a NaN discharge through every variable
    cq += wave_count(valid);
    qv[i] = valid ? Q : __builtin_inff();  // NaN (and the padding) sorts last, past the valid count
  }
  wave_sort_valid<KD, KE>(qv, lane);
  float vals[kGeoVars][KE];
#pragma unroll
  for (int i = 0; i < KE; ++i) {
    const bool ok = i * 64 + lane < cq;
    if (i * 64 >= cq) {  // (wave-uniform) no valid day in this slot: no geometry to evaluate
#pragma unroll
      for (int var = 0; var < kGeoVars; ++var) vals[var][i] = __builtin_nanf("");
      continue;
    }
    const float Q = ok ? qv[i] : 1.0f;  // (padding: any positive value, the result is discarded)
    const DayGeom g = day_geometry(st, Q, cs);
#pragma unroll
    for (int var = 0; var < kGeoVars; ++var) vals[var][i] = ok ? geom_var(g, Q, var) : __builtin_nanf("");
  }
#pragma unroll 1
  for (int var = 0; var < kGeoVars; ++var) {
    float v[KD];
    int cnt = 0;
    double sum = 0.0;
    bool inc = true, dec = true;
#pragma unroll
    for (int i = KE; i < KD; ++i) v[i] = __builtin_inff();  // (sort padding only)
#pragma unroll
    for (int i = 0; i < KE; ++i) {
      // (var is not an unrolled index: a select chain keeps vals in registers, where vals[var][i] would
      // send the array to scratch)
      const float x = var == 0 ? vals[0][i]
                               : (var == 1 ? vals[1][i]
                                           : (var == 2 ? vals[2][i]
                                                       : (var == 3 ? vals[3][i] : (var == 4 ? vals[4][i] : vals[5][i]))));
      const bool valid = x == x;
      cnt += wave_count(valid);
      sum += valid ? (double)x : 0.0;
      v[i] = x;
    }
    // adjacent pairs (e, e + 1), e + 1 < cq: element e + 1 is lane + 1's v[i] (lane 0's v[i + 1] for lane 63)
    float nx[KE];  // element e + 1 of lane l's element e = i * 64 + l: lane l + 1's v[i], or lane 0's v[i + 1]
#pragma unroll
    for (int i = 0; i < KE; ++i) nx[i] = next_lane(v[i]);
#pragma unroll
    for (int i = 0; i < KE; ++i) {
      const float nb = lane < 63 ? nx[i] : (i + 1 < KE ? nx[i + 1] : 0.0f);
      const bool pair = i * 64 + lane + 1 < cq;
      inc = inc && (!pair || v[i] <= nb);
      dec = dec && (!pair || v[i] >= nb);
    }
    sum = wave_sum(sum);
    const bool all_inc = __builtin_amdgcn_ballot_w64(!inc) == 0;
    const bool all_dec = __builtin_amdgcn_ballot_w64(!dec) == 0;
    float mn, mx, med, mean;
    if (cnt == 0) {
      mn = mx = med = mean = __builtin_nanf("");
    } else {
      int i_mn, i_mx, i_lo, i_hi;  // positions of the order statistics among elements [0, cnt)
      if (cnt == cq && (all_inc || all_dec)) {
        const bool up = all_inc;
        auto at = [&](int j) { return up ? j : cnt - 1 - j; };  // j-th smallest
        i_mn = at(0);
        i_mx = at(cnt - 1);
        i_lo = at((cnt - 1) / 2);
        i_hi = at(cnt / 2);
      } else {
        // not monotone along Q (or NaN where Q is valid): sort this variable
#pragma unroll
        for (int i = 0; i < KE; ++i) v[i] = v[i] == v[i] ? v[i] : __builtin_inff();
        wave_sort_valid<KD, KE>(v, lane);
        i_mn = 0;
        i_mx = cnt - 1;
        i_lo = (cnt - 1) / 2;
        i_hi = cnt / 2;
      }
      mn = wave_elem<KD>(v, i_mn);
      mx = wave_elem<KD>(v, i_mx);
      const float lo = wave_elem<KD>(v, i_lo), hi = wave_elem<KD>(v, i_hi);
      med = (cnt & 1) ? lo : (lo + hi) / 2.0f;  // numpy: mean of the two middle values
      mean = (float)(sum / (double)cnt);
    }
    if (lane == 0) {
      float* o = a.out + (int64_t)(var * kGeoStats) * a.N + reach;
      o[0] = mn;
      o[a.N] = mx;
      o[2 * a.N] = med;
      o[3 * a.N] = mean;
    }
  }
}


// Long windows (D > 512 days, beyond the per-wave register sort): one 1024-thread workgroup per reach,
// one variable at a time.  Every day's geometry is evaluated (recomputed per variable: this path is
// for multi-year runs, not the water year), the valid values go into LDS (NaN -> +inf, sorted past
// the valid count), a bitonic sort over P = next power of two >= D orders them, and min / max /
// median / mean come from the sorted array (mean: fp64 sum, as the wave kernel).  D <= kGeoLongMaxDays.
__device__ __forceinline__ float geo_var(const GeoArgs& a, const ReachStatic<float>& st, const Consts<float>& cs,
                                         int64_t reach, int64_t d, int var) {
  const float Q = a.qd[reach * a.rs + d * a.ds];
  if (var == 5) return Q;
  float c1, c2, c3, c4, tw, ss;
  Geom<float> g;
  coefficients<float, false>(st, Q, cs, c1, c2, c3, c4, tw, ss, &g);
  if (Q != Q) return __builtin_nanf("");
  return var == 0 ? g.depth : (var == 1 ? g.tw : (var == 2 ? g.bw : (var == 3 ? g.ss : g.Rh)));
}

__global__ void __launch_bounds__(1024) geometry_stats_long_kernel(GeoArgs a, int P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char gsm[];
  float* v = reinterpret_cast<float*>(gsm + kMathTabBytes);           // [P]
  double* rs = reinterpret_cast<double*>(gsm + kMathTabBytes + 4 * (size_t)P);  // [16] wave sums
  int* rc = reinterpret_cast<int*>(rs + 16);                          // [16] wave counts
  load_math_tables();
  __syncthreads();
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t reach = blockIdx.x;
  Consts<float> cs{};
  cs.dt = 3600.0f;
  cs.qlb = 0.0f;
  cs.vlb = 0.01f;
  cs.vub = 15.0f;
  cs.dlb = a.depth_lb;
  cs.bwlb = a.bw_lb;
  cs.sslb = 0.5f;
  cs.ssub = 50.0f;
  cs.pk = pow_consts();
  cs.ln_dlb = 0.0;
  const ReachStatic<float> st = make_static<float>(a.n[reach], a.q[reach], a.p[reach * a.p_stride], a.S[reach],
                                                   1.0f, 0.0f);
  for (int var = 0; var < kGeoVars; ++var) {
    int cnt = 0;
    double sum = 0.0;
    for (int i = tid; i < P; i += 1024) {
      const float x = i < a.D ? geo_var(a, st, cs, reach, i, var) : __builtin_nanf("");
      const bool valid = x == x;
      cnt += valid;
      sum += valid ? (double)x : 0.0;
      v[i] = valid ? x : __builtin_inff();
    }
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) cnt += __shfl_xor(cnt, m, 64);
    sum = wave_sum(sum);
    if (lane == 0) {
      rs[wave] = sum;
      rc[wave] = cnt;
    }
    __syncthreads();
    // ascending bitonic sort of v[0, P)
    for (int k = 2; k <= P; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < P; i += 1024) {
          const int l = i ^ j;
          if (l > i) {
            const float x = v[i], y = v[l];
            const bool asc = (i & k) == 0;
            if (asc ? (x > y) : (x < y)) {
              v[i] = y;
              v[l] = x;
            }
          }
        }
        __syncthreads();
      }
    }
    if (tid == 0) {
      int c = 0;
      double s = 0.0;
      for (int w = 0; w < 16; ++w) {
        c += rc[w];
        s += rs[w];
      }
      float mn, mx, med, mean;
      if (c == 0) {
        mn = mx = med = mean = __builtin_nanf("");
      } else {
        mn = v[0];
        mx = v[c - 1];
        const float lo = v[(c - 1) / 2], hi = v[c / 2];
        med = (c & 1) ? lo : (lo + hi) / 2.0f;  // numpy: mean of the two middle values
        mean = (float)(s / (double)c);
      }
      float* o = a.out + (int64_t)(var * kGeoStats) * a.N + reach;
      o[0] = mn;
      o[a.N] = mx;
      o[2 * a.N] = med;
      o[3 * a.N] = mean;
    }
    __syncthreads();  // v and the wave sums are reused by the next variable
  }
}

}  // namespace

hipError_t launch_geometry_stats(const float* qd, int64_t rs, int64_t ds, int64_t N, int64_t D, const float* n,
                                 const float* p, int64_t p_stride, const float* q, const float* S, float depth_lb,
                                 float bw_lb, float* out, hipStream_t stream) {
  if (N == 0) return hipSuccess;
  GeoArgs a{qd, rs, ds, N, D, n, p, p_stride, q, S, depth_lb, bw_lb, out};
  if (D > 512) {
    int P = 1024;
    while (P < D) P <<= 1;
    const size_t smem = kMathTabBytes + 4 * (size_t)P + 16 * 8 + 16 * 4;
    hipError_t e = hipFuncSetAttribute((const void*)geometry_stats_long_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(geometry_stats_long_kernel, dim3((unsigned)N), dim3(1024), smem, stream, a, P);
    return hipGetLastError();
  }
  // persistent: the resident workgroup count (occupancy x CUs; a grid beyond it would run its extra
  // workgroups' whole shares after the first ones), rounded down to a multiple of 8 (the XCD deal)
  const int64_t groups = (N + 3) / 4;
  const dim3 block(256);
  auto launch = [&](auto kern) -> hipError_t {
    int per_cu = 0, dev = 0, cus = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, kMathTabBytes);
    if (e == hipSuccess) e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    int64_t nwg = std::min<int64_t>(groups, (int64_t)std::max(per_cu, 1) * std::max(cus, 8));
    nwg = std::max<int64_t>(nwg / 8 * 8, 8);
    hipLaunchKernelGGL(kern, dim3((unsigned)nwg), block, kMathTabBytes, stream, a);
    return hipGetLastError();
  };
  if (D <= 64) return launch(geometry_stats_kernel<1, 1>);
  if (D <= 128) return launch(geometry_stats_kernel<2, 2>);
  if (D <= 192) return launch(geometry_stats_kernel<4, 3>);
  if (D <= 256) return launch(geometry_stats_kernel<4, 4>);
  if (D <= 320) return launch(geometry_stats_kernel<8, 5>);
  if (D <= 384) return launch(geometry_stats_kernel<8, 6>);
  if (D <= 448) return launch(geometry_stats_kernel<8, 7>);
  return launch(geometry_stats_kernel<8, 8>);
}

}  // namespace ddr
