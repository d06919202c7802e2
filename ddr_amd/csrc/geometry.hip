// Per-reach temporal statistics of the trapezoid geometry over daily accumulated discharge
// (reference src/ddr/geometry/statistics.py:20-83, driven by scripts/geometry_predictor.py:193-212).
//
// One wave per reach.  Lane l holds days l, l + 64, ..., (KD per lane, D <= 64 KD): it evaluates the
// geometry of its days once (geometry/trapezoidal.py:62-97 in the routing kernels' exact operation
// order, physics.h), then for each of the six variables (depth, top width, bottom width, side slope,
// hydraulic radius, discharge) the wave sorts the D values (bitonic network: lane shuffles for
// partners in other lanes, register swaps for partners in the same lane) and emits min, max, median
// and mean.  NaN values are skipped like numpy's nanmin / nanmax / nanmedian / nanmean (a reach with
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

// Ascending bitonic sort of the wave's 64 * KD values, element e = i * 64 + lane in v[i].
template <int KD>
__device__ __forceinline__ void wave_sort(float (&v)[KD], int lane) {
  constexpr int M = 64 * KD;
#pragma unroll
  for (int k = 2; k <= M; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= 64) {
        const int jj = j >> 6;
#pragma unroll
        for (int i = 0; i < KD; ++i) {
          if (i & jj) continue;
          const int e = i * 64 + lane;
          const bool asc = (e & k) == 0;
          const float a = v[i], b = v[i | jj];
          v[i] = asc ? fminf(a, b) : fmaxf(a, b);
          v[i | jj] = asc ? fmaxf(a, b) : fminf(a, b);
        }
      } else {
        const bool lower = (lane & j) == 0;
#pragma unroll
        for (int i = 0; i < KD; ++i) {
          const int e = i * 64 + lane;
          const bool asc = (e & k) == 0;
          const float o = shfl_xor_f(v[i], j);
          v[i] = (lower == asc) ? fminf(v[i], o) : fmaxf(v[i], o);
        }
      }
    }
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
  return __shfl(r, l, 64);
}

template <int KD>
__global__ void __launch_bounds__(256) geometry_stats_kernel(GeoArgs a) {
  load_math_tables();
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t reach = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (reach >= a.N) return;  // whole waves leave together
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
  float vals[kGeoVars][KD];
#pragma unroll
  for (int i = 0; i < KD; ++i) {
    const int64_t d = (int64_t)i * 64 + lane;
    const float Q = d < a.D ? a.qd[reach * a.rs + d * a.ds] : __builtin_nanf("");
    float c1, c2, c3, c4, tw, ss;
    Geom<float> g;
    coefficients<float, false>(st, Q, cs, c1, c2, c3, c4, tw, ss, &g);
    const bool ok = d < a.D && Q == Q;  // torch propagates a NaN discharge through every variable
    vals[0][i] = ok ? g.depth : __builtin_nanf("");
    vals[1][i] = ok ? g.tw : __builtin_nanf("");
    vals[2][i] = ok ? g.bw : __builtin_nanf("");
    vals[3][i] = ok ? g.ss : __builtin_nanf("");
    vals[4][i] = ok ? g.Rh : __builtin_nanf("");
    vals[5][i] = Q;
  }
#pragma unroll
  for (int var = 0; var < kGeoVars; ++var) {
    float v[KD];
    int cnt = 0;
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < KD; ++i) {
      const float x = vals[var][i];
      const bool valid = x == x;
      cnt += valid;
      sum += valid ? (double)x : 0.0;
      v[i] = valid ? x : __builtin_inff();  // NaN sorts last, past the valid count
    }
    // wave totals (every lane ends with the same value)
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
      cnt += __shfl_xor(cnt, m, 64);
      sum += __shfl_xor(sum, m, 64);
    }
    wave_sort<KD>(v, lane);
    float mn, mx, med, mean;
    if (cnt == 0) {
      mn = mx = med = mean = __builtin_nanf("");
    } else {
      mn = wave_elem<KD>(v, 0);
      mx = wave_elem<KD>(v, cnt - 1);
      const float lo = wave_elem<KD>(v, (cnt - 1) / 2), hi = wave_elem<KD>(v, cnt / 2);
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
    for (int m = 1; m < 64; m <<= 1) {
      cnt += __shfl_xor(cnt, m, 64);
      sum += __shfl_xor(sum, m, 64);
    }
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
  const dim3 grid((unsigned)((N + 3) / 4)), block(256);
  if (D <= 64) hipLaunchKernelGGL(geometry_stats_kernel<1>, grid, block, kMathTabBytes, stream, a);
  else if (D <= 128) hipLaunchKernelGGL(geometry_stats_kernel<2>, grid, block, kMathTabBytes, stream, a);
  else if (D <= 256) hipLaunchKernelGGL(geometry_stats_kernel<4>, grid, block, kMathTabBytes, stream, a);
  else hipLaunchKernelGGL(geometry_stats_kernel<8>, grid, block, kMathTabBytes, stream, a);
  return hipGetLastError();
}

}  // namespace ddr
