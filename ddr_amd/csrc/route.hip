// Fused Muskingum-Cunge routing kernels for gfx950 (MI355X): forward over all T steps and the
// reverse-time / reverse-topological adjoint.
//
// One persistent workgroup owns a block of reaches (whole basins, or a connected piece of a large
// basin) for the whole time window.  Reach i runs step t at tick t + off(i) with
// off(i) = dmax - dist_in_piece(i): every upstream reach is exactly one tick ahead, so one
// LDS double-buffer + one workgroup barrier per tick carries all in-block dependencies
// ("as late as possible" wavefront; T + dmax ticks instead of T x depth level syncs).
// Edges between blocks (cut edges) are exchanged through global memory as 8-byte granules that
// are their own ready flag (sentinel = all ones, re-initialised before every launch), imported in
// chunks of kChunk ticks so the hand-off latency is paid once per chunk.
//
// Reference semantics (file:line in /root/reference):
//   forward  src/ddr/routing/mmc.py:365-443, 487-559, 25-66; routing/utils.py:587-600 (fp64 solve)
//   backward routing/utils.py:629-692 + torch autograd of mmc.py/trapezoidal.py (hand adjoint)
#include "internal.h"
#include "physics.h"
#include "route_args.h"

namespace ddr {

namespace {

constexpr unsigned long long kSentinel = ~0ull;

__device__ __forceinline__ void lds_barrier() {
  // LDS hand-off only: global loads issued ahead (prefetch) stay in flight across the barrier.
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ void store_granule(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long load_granule(const double* p) {
  return __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// Spin until the granule is published (bounded; on timeout record it and return 0).
__device__ double wait_granule(const double* p, unsigned* status) {
  unsigned long long v = load_granule(p);
  unsigned spins = 0;
  while (v == kSentinel) {
    __builtin_amdgcn_s_sleep(2);
    v = load_granule(p);
    if (++spins > (1u << 24)) {
      atomicAdd(status, 1u);
      atomicCAS(status + 1, 0u, blockIdx.x + 1u);
      return 0.0;
    }
  }
  return __longlong_as_double(v);
}

template <typename R>
__device__ __forceinline__ Consts<R> consts_of(const RouteArgs& a) {
  return Consts<R>{R(a.c[0]), R(a.c[1]), R(a.c[2]), R(a.c[3]), R(a.c[4]), R(a.c[5]), R(a.c[6]), R(a.c[7])};
}

template <typename R>
__device__ __forceinline__ ReachStatic<R> load_static(const RouteArgs& a, int ref) {
  const R* n = static_cast<const R*>(a.n);
  const R* q = static_cast<const R*>(a.q);
  const R* p = static_cast<const R*>(a.p);
  const R* L = static_cast<const R*>(a.L);
  const R* S = static_cast<const R*>(a.S);
  const R* X = static_cast<const R*>(a.X);
  return make_static<R>(n[ref], q[ref], p[(int64_t)ref * a.p_stride], S[ref], L[ref], X[ref]);
}

template <typename R>
__device__ __forceinline__ R load_qprime(const RouteArgs& a, int64_t row, int ref) {
  const R* qp = static_cast<const R*>(a.qprime);
  R v = qp[row * a.N + ref];
  if (a.fs) v = v * static_cast<const R*>(a.fs)[ref];  // mmc.py:303-304 (q' * flow_scale)
  return v;
}

}  // namespace

// ============================================================================================
// Forward
// ============================================================================================
template <typename R, int KR>
__global__ void __launch_bounds__(kBlockThreads) route_forward_kernel(RouteArgs a) {
  constexpr int BS = kBlockThreads;
  const BlockDesc B = a.s.blocks[blockIdx.x];
  const int tid = threadIdx.x;
  const int S = a.slot_stride;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* sx = reinterpret_cast<double*>(smem);                 // [2][S]  x_j(t) (solve precision)
  R* sq = reinterpret_cast<R*>(sx + 2 * S);                     // [2][S]  Q_j(t-1)
  double* ring = reinterpret_cast<double*>(smem + ((2 * S * (8 + sizeof(R)) + 15) / 16) * 16);
  const Consts<R> cs = consts_of<R>(a);
  const int64_t T = a.T;
  const bool carry = a.flags & DDR_FWD_CARRY;
  const bool save = a.flags & DDR_FWD_SAVE_X;
  const bool write_runoff = !(a.flags & DDR_FWD_NO_RUNOFF) && a.runoff;
  R* runoff = static_cast<R*>(a.runoff);
  R* xsave = static_cast<R*>(a.x_save);
  const int64_t xs_base = T * B.pos0 + B.pre_dn;

  ReachStatic<R> st[KR];
  int ref[KR], off[KR], upb[KR], upc[KR], cut[KR];
  R Q[KR];
  bool has[KR];
#pragma unroll
  for (int k = 0; k < KR; ++k) {
    const int r = tid + k * BS;
    has[k] = r < B.nloc;
    const int P = B.pos0 + (has[k] ? r : 0);
    ref[k] = a.s.ref[P];
    off[k] = a.s.off[P];
    upb[k] = a.s.upb[P];
    upc[k] = a.s.upc[P];
    cut[k] = a.s.cut[P];
    st[k] = load_static<R>(a, ref[k]);
    Q[k] = R(0);
  }
  // virtual inflows: thread v < nvirt owns virtual v
  const bool vown = tid < B.nvirt;
  int v_off = 0;
  R vQ = R(0);
  if (vown) {

    v_off = a.s.v_off[B.virt0 + tid];
  }
  const int TT = (int)T + B.dmax;
  for (int tau = 0; tau < TT; ++tau) {
    const int cur = tau & 1, prv = cur ^ 1;
    if (B.nvirt > 0 && (tau % kChunk) == 0) {
      // import the next chunk of every virtual inflow into its ring half
      const int half = (tau / kChunk) & 1;
      for (int w = tid; w < B.nvirt * kChunk; w += BS) {
        const int v = w / kChunk, sidx = w % kChunk;
        const int e = a.s.v_edge[B.virt0 + v];
        const int t = tau + sidx - a.s.v_off[B.virt0 + v];
        double val = 0.0;
        if (t >= 0 && t < T) val = wait_granule(a.bnd + (int64_t)e * T + t, a.status);
        ring[v * a.ring_stride + half * kChunk + sidx] = val;
      }
      lds_barrier();
    }
    if (vown) {
      const int t = tau - v_off;
      if (t >= 0 && t < T) {
        const double x = ring[tid * a.ring_stride + (tau % (2 * kChunk))];
        sx[cur * S + B.nloc + tid] = x;
        sq[cur * S + B.nloc + tid] = vQ;
        vQ = (t == 0 && carry) ? R(x) : rmax(R(x), cs.qlb);
      }
    }
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      if (!has[k]) continue;
      const int r = tid + k * BS;
      const int64_t t = tau - off[k];
      if (t < 0 || t >= T) continue;
      const R Qprev = Q[k];
      const int nup = upc[k];
      double x;
      R Qn;
      if (t == 0) {
        if (carry) {
          x = (double)static_cast<const R*>(a.q0)[ref[k]];
          Qn = R(x);
        } else {
          // hot start: (I - N) Q0 = q'[0] (mmc.py:25-66), fp64 column sweep, then clamp
          double acc = (double)load_qprime<R>(a, 0, ref[k]);
          for (int j = 0; j < nup; ++j) acc = acc + sx[prv * S + a.s.uplist[upb[k] + j]];
          x = acc;
          Qn = rmax(R(x), cs.qlb);
        }
      } else {
        const R qc = rmax(load_qprime<R>(a, t - 1, ref[k]), cs.qlb);  // mmc.py:421-424
        R c1, c2, c3, c4, tw, ss;
        coefficients<R>(st[k], Qprev, cs, c1, c2, c3, c4, tw, ss);
        R I = R(0);
        for (int j = 0; j < nup; ++j) I = I + sq[prv * S + a.s.uplist[upb[k] + j]];  // N @ Q_t
        const R b = ((c2 * I) + (c3 * Qprev)) + (c4 * qc);                           // mmc.py:538
        double acc = (double)b;
        const double dc1 = (double)c1;
        for (int j = 0; j < nup; ++j) acc = acc + dc1 * sx[prv * S + a.s.uplist[upb[k] + j]];
        x = acc;
        Qn = rmax(R(x), cs.qlb);  // mmc.py:557
        if (t == T - 1) {
          if (a.tw_last) static_cast<R*>(a.tw_last)[ref[k]] = tw;
          if (a.ss_last) static_cast<R*>(a.ss_last)[ref[k]] = ss;
        }
      }
      sx[cur * S + r] = x;
      sq[cur * S + r] = Qprev;
      const R xr = R(x);
      if (save) xsave[xs_base + (int64_t)tau * B.nloc + r] = xr;
      if (write_runoff) runoff[(int64_t)ref[k] * T + t] = (t == 0) ? rmax(xr, cs.qlb) : Qn;
      if (cut[k] >= 0) store_granule(a.bnd + (int64_t)cut[k] * T + t, x);
      if (t == T - 1 && a.q_last) static_cast<R*>(a.q_last)[ref[k]] = Qn;
      Q[k] = Qn;
    }
    lds_barrier();
  }
}

// ============================================================================================
// Backward (adjoint)
// ============================================================================================
template <typename R>
__device__ __forceinline__ R up_x(const RouteArgs& a, const BlockDesc& B, const R* xsave, int64_t xs_base,
                                  int u, int tick, int64_t t) {
  if (u < B.nloc) return xsave[xs_base + (int64_t)tick * B.nloc + u];
  const int e = a.s.v_edge[B.virt0 + (u - B.nloc)];
  return R(a.bnd[(int64_t)e * a.T + t]);
}

template <typename R, int KR>
__global__ void __launch_bounds__(kBlockThreads) route_backward_kernel(RouteArgs a) {
  constexpr int BS = kBlockThreads;
  const BlockDesc B = a.s.blocks[blockIdx.x];
  const int tid = threadIdx.x;
  const int S = a.slot_stride;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* sa = reinterpret_cast<double*>(smem);  // [2][S]  c1_i * gb_i  (fp64, transposed solve)
  R* sb = reinterpret_cast<R*>(sa + 2 * S);       // [2][S]  c2_i * gb_i
  double* ring = reinterpret_cast<double*>(smem + ((2 * S * (8 + sizeof(R)) + 15) / 16) * 16);
  const Consts<R> cs = consts_of<R>(a);
  const int64_t T = a.T;
  const bool carry = a.flags & DDR_FWD_CARRY;
  const R* xsave = static_cast<const R*>(a.x_save);
  const R* gout = static_cast<const R*>(a.grad_out);
  const int64_t xs_base = T * B.pos0 + B.pre_dn;

  ReachStatic<R> st[KR];
  int ref[KR], off[KR], upb[KR], upc[KR], dloc[KR], cut[KR], gb0[KR], gcnt[KR];
  R lam[KR];
  double acc_n[KR], acc_q[KR], acc_p[KR];
  bool has[KR];
#pragma unroll
  for (int k = 0; k < KR; ++k) {
    const int r = tid + k * BS;
    has[k] = r < B.nloc;
    const int P = B.pos0 + (has[k] ? r : 0);
    ref[k] = a.s.ref[P];
    off[k] = a.s.off[P];
    upb[k] = a.s.upb[P];
    upc[k] = a.s.upc[P];
    dloc[k] = a.s.dloc[P];
    cut[k] = a.s.cut[P];
    st[k] = load_static<R>(a, ref[k]);
    lam[k] = R(0);
    acc_n[k] = acc_q[k] = acc_p[k] = 0.0;
    if (a.g_roff) {
      gb0[k] = (int)a.g_roff[ref[k]];
      gcnt[k] = (int)(a.g_roff[ref[k] + 1] - a.g_roff[ref[k]]);
    } else {
      gb0[k] = 0;
      gcnt[k] = -1;
    }
  }
  // cut-out import ring slot: thread c < ncout owns cut-out reach cout_loc[c]
  int my_cout_slot[KR];
#pragma unroll
  for (int k = 0; k < KR; ++k) my_cout_slot[k] = -1;
  for (int c = 0; c < B.ncout; ++c) {
    const int loc = a.s.cout_loc[B.cout0 + c];
#pragma unroll
    for (int k = 0; k < KR; ++k)
      if (has[k] && tid + k * BS == loc) my_cout_slot[k] = c;
  }
  const bool vown = tid < B.nvirt;
  int v_edge = 0, v_off = 0, v_dloc = 0;
  if (vown) {
    v_edge = a.s.v_edge[B.virt0 + tid];
    v_off = a.s.v_off[B.virt0 + tid];
    v_dloc = a.s.v_dloc[B.virt0 + tid];
  }
  const int TT = (int)T + B.dmax;
  for (int tb = 0; tb < TT; ++tb) {
    const int tau = TT - 1 - tb;  // forward tick
    const int cur = tb & 1, prv = cur ^ 1;
    if (B.ncout > 0 && (tb % kChunk) == 0) {
      const int half = (tb / kChunk) & 1;
      for (int w = tid; w < B.ncout * kChunk; w += BS) {
        const int c = w / kChunk, sidx = w % kChunk;
        const int P = B.pos0 + a.s.cout_loc[B.cout0 + c];
        const int e = a.s.cut[P];
        const int t = (tau - sidx) - a.s.off[P];
        double A = 0.0, Bv = 0.0;
        if (t >= 1 && t < T) {
          A = wait_granule(a.bwd_bnd + ((int64_t)e * T + t) * 2, a.status);
          Bv = wait_granule(a.bwd_bnd + ((int64_t)e * T + t) * 2 + 1, a.status);
        }
        ring[c * a.ring_stride + (half * kChunk + sidx) * 2] = A;
        ring[c * a.ring_stride + (half * kChunk + sidx) * 2 + 1] = Bv;
      }
      lds_barrier();
    }
    if (vown) {
      // export the consumer's (c1 gb, c2 gb) of step t to the upstream block
      const int t = tau - v_off;
      if (t >= 1 && t < T) {
        store_granule(a.bwd_bnd + ((int64_t)v_edge * T + t) * 2, sa[prv * S + v_dloc]);
        store_granule(a.bwd_bnd + ((int64_t)v_edge * T + t) * 2 + 1, (double)sb[prv * S + v_dloc]);
      }
    }
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      if (!has[k]) continue;
      const int r = tid + k * BS;
      const int64_t t = tau - off[k];
      if (t < 1 || t >= T) continue;
      // dL/dQ_t += dL/dout[:, t]
      R g;
      if (gcnt[k] < 0) {
        g = gout[(int64_t)ref[k] * T + t];
      } else {
        g = R(0);
        for (int m = 0; m < gcnt[k]; ++m) g = g + gout[a.g_rg[gb0[k] + m] * T + t];
      }
      lam[k] = lam[k] + g;
      const R xt = xsave[xs_base + (int64_t)tau * B.nloc + r];
      const R xp = xsave[xs_base + (int64_t)(tau - 1) * B.nloc + r];
      const R gx = (xt >= cs.qlb) ? lam[k] : R(0);  // clamp backward (inclusive)
      double A = 0.0;
      R Bd = R(0);
      if (dloc[k] >= 0) {
        A = sa[prv * S + dloc[k]];
        Bd = sb[prv * S + dloc[k]];
      } else if (my_cout_slot[k] >= 0) {
        const int sidx = (tb % (2 * kChunk));
        A = ring[my_cout_slot[k] * a.ring_stride + sidx * 2];
        Bd = R(ring[my_cout_slot[k] * a.ring_stride + sidx * 2 + 1]);
      }
      const double gb64 = (double)gx + A;  // (I - C1 N)^T gb = gx, fp64 (utils.py:188-242)
      const R gb = R(gb64);
      const R Qp = (t == 1 && carry) ? xp : rmax(xp, cs.qlb);
      R c1, c2, c3, c4, tw, ss;
      Geom<R> geo;
      coefficients<R>(st[k], Qp, cs, c1, c2, c3, c4, tw, ss, &geo);
      R I = R(0), Sx = R(0);
      const int nup = upc[k];
      for (int j = 0; j < nup; ++j) {
        const int u = a.s.uplist[upb[k] + j];
        const R xu = up_x<R>(a, B, xsave, xs_base, u, tau - 1, t);
        const R xu_p = up_x<R>(a, B, xsave, xs_base, u, tau - 2, t - 1);
        Sx = Sx + xu;
        I = I + ((t == 1 && carry) ? xu_p : rmax(xu_p, cs.qlb));
      }
      const R qc = rmax(load_qprime<R>(a, t - 1, ref[k]), cs.qlb);
      const R gc1 = gb * Sx, gc2 = gb * I, gc3 = gb * Qp, gc4 = gb * qc;
      R gQ, gn, gq, gp;
      coefficients_vjp<R>(st[k], Qp, cs, geo, c1, c2, c3, c4, gc1, gc2, gc3, gc4, gQ, gn, gq, gp);
      acc_n[k] += (double)gn;
      acc_q[k] += (double)gq;
      acc_p[k] += (double)gp;
      sa[cur * S + r] = (double)c1 * gb64;
      sb[cur * S + r] = c2 * gb;
      lam[k] = ((gb * c3) + gQ) + Bd;
    }
    lds_barrier();
  }
#pragma unroll
  for (int k = 0; k < KR; ++k) {
    if (!has[k]) continue;
    static_cast<R*>(a.gn)[ref[k]] = R(acc_n[k]);
    static_cast<R*>(a.gq)[ref[k]] = R(acc_q[k]);
    static_cast<R*>(a.gp)[ref[k]] = R(acc_p[k]);
  }
}

// ============================================================================================
// Gauge reduction: out[g, t] = sum_{k} clamp(x_t[idx_k])  (mmc.py:405-411, 433-439)
// ============================================================================================


template <typename R>
__global__ void gauge_reduce_kernel(GaugeArgs a, const R* xsave, R* out) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= a.G * a.T) return;
  const int64_t g = w / a.T, t = w % a.T;
  R acc = R(0);
  for (int64_t k = a.goff[g]; k < a.goff[g + 1]; ++k) {
    const int P = a.pos_of_ref[a.gidx[k]];
    const BlockDesc B = a.s.blocks[a.block_of_pos[P]];
    const int r = P - B.pos0;
    const int64_t tick = t + a.s.off[P];
    const R x = xsave[a.T * B.pos0 + B.pre_dn + tick * B.nloc + r];
    const R Q = (t == 0 && a.carry) ? x : rmax(x, R(a.qlb));
    acc = acc + Q;
  }
  // output[:, 0] = clamp(initial) (mmc.py:412); later steps are sums of clamped states
  out[g * a.T + t] = (t == 0) ? rmax(acc, R(a.qlb)) : acc;
}

// ============================================================================================
// Host launchers
// ============================================================================================
template <typename R>
size_t route_smem_bytes(const Graph* g, bool backward) {
  const size_t S = (size_t)g->max_slots;
  size_t base = ((2 * S * (8 + sizeof(R)) + 15) / 16) * 16;
  const int nring = backward ? g->max_cout : g->max_virt;
  const size_t ring = backward ? 2 * 2 * kChunk : 2 * kChunk;
  return base + (size_t)nring * ring * sizeof(double);
}

template <typename R, int KR>
hipError_t launch_route_kr(const Graph* g, RouteArgs a, bool backward, hipStream_t stream) {
  const size_t smem = route_smem_bytes<R>(g, backward);
  a.slot_stride = g->max_slots;
  a.ring_stride = backward ? 4 * kChunk : 2 * kChunk;
  const dim3 grid((unsigned)g->blocks.size()), block(kBlockThreads);
  if (backward) {
    auto kern = route_backward_kernel<R, KR>;
    if (smem > 64 * 1024) {
      hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, grid, block, smem, stream, a);
  } else {
    auto kern = route_forward_kernel<R, KR>;
    if (smem > 64 * 1024) {
      hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, grid, block, smem, stream, a);
  }
  return hipGetLastError();
}

template <typename R>
hipError_t launch_route(const Graph* g, const RouteArgs& a, bool backward, hipStream_t stream) {
  switch (g->kr) {
    case 1: return launch_route_kr<R, 1>(g, a, backward, stream);
    case 2: return launch_route_kr<R, 2>(g, a, backward, stream);
    case 4: return launch_route_kr<R, 4>(g, a, backward, stream);
    case 8: return launch_route_kr<R, 8>(g, a, backward, stream);
    default: return launch_route_kr<R, 8>(g, a, backward, stream);
  }
}

template <typename R>
int max_resident_blocks(const Graph* g, bool backward) {
  int nb = 0;
  const size_t smem = route_smem_bytes<R>(g, backward);
  const void* f = nullptr;
#define DDR_PICK(KRV)                                                                   \
  case KRV:                                                                             \
    f = backward ? (const void*)route_backward_kernel<R, KRV> : (const void*)route_forward_kernel<R, KRV>; \
    break;
  switch (g->kr) {
    DDR_PICK(1)
    DDR_PICK(2)
    DDR_PICK(4)
    default:
      f = backward ? (const void*)route_backward_kernel<R, 8> : (const void*)route_forward_kernel<R, 8>;
  }
#undef DDR_PICK
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, kBlockThreads, smem) != hipSuccess) return -1;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, g->device) != hipSuccess) return -1;
  return nb * prop.multiProcessorCount;
}

template <typename R>
hipError_t launch_gauge(const GaugeArgs& a, const R* xsave, R* out, hipStream_t stream) {
  const int64_t total = a.G * a.T;
  if (total == 0) return hipSuccess;
  const int threads = 256;
  const unsigned blocks = (unsigned)((total + threads - 1) / threads);
  hipLaunchKernelGGL(gauge_reduce_kernel<R>, dim3(blocks), dim3(threads), 0, stream, a, xsave, out);
  return hipGetLastError();
}

template hipError_t launch_route<float>(const Graph*, const RouteArgs&, bool, hipStream_t);
template hipError_t launch_route<double>(const Graph*, const RouteArgs&, bool, hipStream_t);
template int max_resident_blocks<float>(const Graph*, bool);
template int max_resident_blocks<double>(const Graph*, bool);
template hipError_t launch_gauge<float>(const GaugeArgs&, const float*, float*, hipStream_t);
template hipError_t launch_gauge<double>(const GaugeArgs&, const double*, double*, hipStream_t);

}  // namespace ddr
