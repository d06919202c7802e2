// Kernel argument blocks and launchers shared by route.hip and capi.cpp.
#pragma once

#include "internal.h"

namespace ddr {

struct RouteArgs {
  DevSchedule s;
  int64_t N, T;
  int64_t n_cut;
  int32_t flags;
  int32_t slot_stride;  // LDS slots per buffer (max nloc + nvirt over blocks)
  int32_t nblocks;      // logical blocks (tickets) of a routing launch
  int32_t xl_off;       // byte offset of the confluence lists in the dynamic LDS
  int32_t own_off;      // backward: byte offset of the hand-off owner words
  int32_t p_stride;
  int32_t qp_hours;               // hourly steps per stored q' row (1, or 24 for a daily store)
  int32_t qp_shift;               // step t reads q' row max(t - qp_shift, 0): 1 routing, 0 accumulation
  // row layout of the gathered q' (a store of qp_hours > 1 steps per row, e.g. daily): per block
  // [qp_rows][nloc] instead of the tick-major [T + dmax][nloc]; row = max(t - shift, 0) / qp_hours,
  // the division as a multiply-high by qp_magic (exact for the window, checked on the host)
  int32_t qs_rows;                // 0: tick-major layout; else rows per block of the row layout
  uint32_t qp_magic;
  const unsigned char* qp_valid;  // optional per-reach mask: 0 -> q' = 0.001 (missing divide)
  const void* n;
  const void* q;
  const void* p;
  const void* L;
  const void* S;
  const void* X;
  const void* fs;
  const void* qprime;
  const void* q0;
  void* runoff;
  void* x_save;
  void* qs;              // lateral inflow in the schedule layout (second half of the x_save workspace)
  double* bnd;
  unsigned* status;
  void* q_last;
  void* tw_last;
  void* ss_last;
  // backward
  const void* grad_out;   // dL/drunoff, (N, T) or (G, T) in gauge mode
  const int64_t* g_roff;
  const int64_t* g_rg;
  double* bwd_bnd;
  void* gn;
  void* gq;
  void* gp;
  // state-gradient backward (route_backward_kernel<.., GS = true>): dL/d(q' * flow_scale) in the
  // schedule layout (as qs), dL/dQ0 (N, carried state), per-gauge t = 0 clamp mask (gauge mode)
  void* gqs;
  void* gq0;
  const unsigned char* gmask0;
  // per-reach state seeds (reference order, R), or null: [0, N) dL/dQ_{T-1} (the final discharge state,
  // mmc.py:441), [N, 2N) dL/dQ_{T-2} (the state the reported geometry reads, mmc.py:161-162); added to
  // dL/dout of those steps (gauge mode: every reach reads its gradient groups)
  const void* gseed;
  unsigned long long* prof;  // debug per-workgroup profile (ddr_set_block_profile), or null
  // split basin (SplitState, internal.h; null when not split): logical blocks of other ranks are
  // skipped, cross-rank cut edges read this rank's receive rows and write the peer's
  const uint8_t* owned;
  const int32_t* xid;
  const int32_t* xcons;
  const int32_t* xprod;
  const int64_t* xedge;
  int32_t xrank;  // this rank's index in the split group
  double* xfwd;
  double* xbwd;
  double* pxfwd[kMaxSplitRanks];
  double* pxbwd[kMaxSplitRanks];
  int32_t xt_off;  // split: byte offset of the block's granule row table in the dynamic LDS (0: none)
  double c[8];  // dt, qlb, vlb, vub, dlb, bwlb, sslb, ssub
  float cf[8];  // the same rounded to fp32 (kernel constants of the fp32 build)
  double ln_dlb;  // ln of the fp32-rounded depth lower bound (fp32 pow derivation, physics.h)
};

struct GaugeArgs {
  DevSchedule s;
  int64_t T;
  int64_t G;
  const int64_t* goff;
  const int64_t* gidx;
  const int32_t* pos_of_ref;  // internal position of each reference reach
  const int32_t* block_of_pos;
  double qlb;
  int32_t carry;
};

template <typename R>
hipError_t launch_route(const Graph* g, const RouteArgs& a, bool backward, hipStream_t stream);
// Q(t) of every reach (reference order) from a forward's saved states (route.hip: state_at_kernel)
template <typename R>
hipError_t launch_state_at(const Graph* g, int64_t T, int64_t t, double qlb, bool carry, const R* xsave, R* out,
                           hipStream_t stream);
// split basin: the epoch hand-shake before a routing launch (route.hip: split_barrier_kernel)
struct SplitBarrierArgs {
  unsigned long long* mine;                  // this rank's epoch words ([2][kMaxSplitRanks])
  unsigned long long* peer[kMaxSplitRanks];  // every rank's epoch words
  int32_t rank, nranks, slot;                // slot 0: forward, 1: backward
  unsigned long long epoch;
  unsigned* status;
};
hipError_t launch_split_barrier(const SplitBarrierArgs& b, hipStream_t stream);
// split basin, after a forward: the cross-rank x rows this rank received are copied into the call's own
// boundary buffer (the backward reads them there, never from the shared receive rows a later forward
// overwrites), and column 0 of the runoff rows of reaches another rank routes is set to NaN
template <typename R>
hipError_t launch_split_finish(const Graph* g, const RouteArgs& a, hipStream_t stream);
// dL/dq' (rows of the caller's store, (rows, N)) from the state-gradient backward's gqs: the adjoint
// of gather_qprime (sum over the steps reading each row, times flow_scale, 0 for a filled divide)
template <typename R>
hipError_t launch_scatter_qprime_grad(const Graph* g, const RouteArgs& a, int64_t rows, R* out, hipStream_t stream);
// per-gauge clamp mask of the t = 0 gauge sum (mmc.py:398-412), for the state-gradient backward
template <typename R>
hipError_t launch_gauge_mask0(const GaugeArgs& a, const R* xsave, unsigned char* mask, hipStream_t stream);
template <typename R>
int max_resident_blocks(const Graph* g, bool backward);
template <typename R>
hipError_t launch_gather_qprime(const Graph* g, RouteArgs& a, hipStream_t stream);
// Sets a.qs_rows / a.qp_magic when the window's q' store has several steps per row and the
// row layout's magic division is exact over the window (otherwise the tick-major layout).
inline void choose_qs_layout(RouteArgs& a) {
  a.qs_rows = 0;
  a.qp_magic = 0;
  const int64_t H = a.qp_hours;
#ifndef DDR_QS_ROWS
#define DDR_QS_ROWS 1
#endif
  if (!DDR_QS_ROWS || H <= 1 || a.T < 1) return;
  const uint64_t m = ((uint64_t(1) << 32) + (uint64_t)H - 1) / (uint64_t)H;  // ceil(2^32 / H)
  const uint64_t err = m * (uint64_t)H - (uint64_t(1) << 32);
  // floor(t m / 2^32) == floor(t / H) for t * err < 2^32 / H
  if (err > 0 && (uint64_t)a.T * err >= ((uint64_t(1) << 32) / (uint64_t)H)) return;
  const int64_t last = a.T - 1 > a.qp_shift ? a.T - 1 - a.qp_shift : 0;
  a.qs_rows = (int32_t)(last / H + 1);
  a.qp_magic = (uint32_t)m;
}
template <typename R>
hipError_t launch_gauge(const GaugeArgs& a, const R* xsave, R* out, hipStream_t stream);
template <typename R>
hipError_t launch_gauge_daily(const GaugeArgs& a, const R* xsave, int64_t t0, int64_t L, int64_t D, R* out,
                              hipStream_t stream);
template <typename R>
hipError_t launch_gauge_daily_seed(int64_t G, int64_t T, int64_t t0, int64_t L, int64_t D, const R* gd, R* gh,
                                   hipStream_t stream);
// pnet.hip: the fused parameter network (C3's KAN stand-in); denorm = host [3][3] (scale, offset, log flag)
int pnet_param_count(int F);
int64_t pnet_work_bytes(int64_t N, int F);
hipError_t launch_pnet_forward(int64_t N, int F, const float* X, const float* P, const float* denorm, float* Z, float* U,
                               float* const out[3], hipStream_t stream);
hipError_t launch_pnet_backward(int64_t N, int F, const float* X, const float* P, const float* denorm, const float* Z,
                                const float* U, const float* const gout[3], float* grad, void* work, hipStream_t stream);
// geometry.hip: windows of up to kGeoLongMaxDays days (~89 years; beyond 512 days one workgroup per
// reach sorts each variable in LDS)
constexpr int64_t kGeoLongMaxDays = 32768;
hipError_t launch_geometry_stats(const float* qd, int64_t rs, int64_t ds, int64_t N, int64_t D, const float* n,
                                 const float* p, int64_t p_stride, const float* q, const float* S, float depth_lb,
                                 float bw_lb, float* out, hipStream_t stream);

}  // namespace ddr
