// Fused Muskingum-Cunge routing kernels for gfx950 (MI355X): forward over all T steps and the
// reverse-time / reverse-topological adjoint.
//
// One persistent workgroup owns a block of reaches (whole basins, or a connected piece of a large
// basin) for the whole time window.  Reach i runs step t at tick t + off(i) with
// off(i) = dmax - dist_in_piece(i): every upstream reach is exactly one tick ahead, so one
// LDS slot per reach + two workgroup barriers per tick carry all in-block dependencies
// ("as late as possible" wavefront; T + dmax ticks instead of T x depth level syncs).
// Edges between blocks (cut edges) are exchanged through global memory as 8-byte granules that
// are their own ready flag (sentinel = all ones, re-initialised before every launch), imported in
// chunks of kChunkFwd / kChunkBwd ticks so the hand-off latency is paid once per chunk.
//
// Workgroups take their logical block from a ticket counter (take_ticket): blocks are numbered in
// piece-height order, so the producers of a running workgroup were taken by workgroups that are
// running or finished, whatever the grid size and the dispatch order.  A schedule with more blocks
// than resident workgroups therefore runs to completion (as "generations"); one that fits runs
// fully time-pipelined.  Every wait is bounded: a timeout records the device status word and yields
// NaN, so a failed hand-off can never pass for a number (capi.cpp reports it as DDR_ERR_TIMEOUT).
//
// Each thread owns KR <= 4 reaches (r = tid + k * 1024); one 1024-thread workgroup per CU (4 waves
// per SIMD).  The per-reach statics live in LDS; registers hold only the per-reach state and one
// tick of prefetched inputs.  Each tick: compute (reads upstream slots) -> barrier -> publish (own
// slot) -> barrier.
//
// Reference semantics (file:line in /root/reference):
//   forward  src/ddr/routing/mmc.py:365-443, 487-559, 25-66; routing/utils.py:587-600 (fp64 solve)
//   backward routing/utils.py:629-692 + torch autograd of mmc.py/trapezoidal.py (hand adjoint)
#include <type_traits>

#include "internal.h"
#include "physics.h"
#include "route_args.h"

namespace ddr {

// Tuning constants (each chosen by an A/B on MI355X; the rejected alternatives live in git history and
// profiles/r0*/ab_*.txt, not here):
// The backward's early loads (the next tick's x(t - 3) and virtual x requested at the top of the tick into a
// second register set) and its double-buffered slots at KR <= 2; KR = 4 has no registers for the second set
constexpr int kBwdEarlyMaxKR = 2;
// The backward's dL/drunoff groups as shift registers at KR <= 2 (c3s8 backward -4 %); at KR = 4 a select on
// t & 3 as two bit tests and three selects (C5 backward 59.5 vs 57.3 ms, profiles/r05/ab_r05.txt)
constexpr int kBwdShiftMaxKR = 2;
// Import waves: a chunk's cut-out granules requested this many ticks before its boundary tick
constexpr int kBwdImpEarly = 4;
// x / gradient helpers: their loads issued this many ticks ahead
constexpr int kBwdHelpAhead = 3;
// The clamps' infinity opaque to the compiler from this KR on (one v_med3_f32 per clamp)
constexpr int kOpqInfMinKR = 4;

namespace {

constexpr unsigned long long kSentinel = ~0ull;
static_assert(kMathTabBytes == (2 * kLnTabN + kExpTabN) * sizeof(double), "math table size");


__device__ __forceinline__ void lds_barrier() {
  // LDS hand-off only: global loads issued ahead (prefetch) stay in flight across the barrier.
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Wave priority by remaining slices: the SIMD's arbiter serves its oldest ready wave
// first, so the workgroup's first waves finish their slices early and the youngest runs its last slices
// alone at the end of every tick, one dependent chain issuing on the SIMD.  A wave at slice k of KR takes
// priority KR - 1 - k (the top of the tick: 3), so the waves with more work left go first and the
// SIMD's waves finish together.  KR = 4 (full load): C5 129.4 -> 126.2 ms, C3 forward 16.0 -> 14.4 ms
// (profiles/r04/ab_r04.txt item 28); at KR = 2 no gain was measured (C4), KR = 1 has one slice.
// (forward at KR = 1) a routing wave runs its step's physics at priority 1 and the rest at 0:
// of the two routing waves on a SIMD, the one ahead yields once its physics is done, so the two finish
// together (c3s8 forward 2.87 -> 2.75 ms; C2 and c5s8r5 within noise; the backward's adjoint showed no
// change; profiles/r04/ab_r04.txt item 30)
__device__ __forceinline__ void set_prio(int p) {
  switch (p) {
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3); break;
  }
}

__device__ __forceinline__ void store_granule(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long load_granule(const double* p) {
  return __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
// Cross-rank granules (split basin): system scope, so a peer GPU's stores into this rank's receive
// rows and this rank's stores into a peer's are seen through neither side's L2
__device__ __forceinline__ void store_granule_sys(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned long long load_granule_sys(const double* p) {
  return __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

// Spin until the granules of a chunk are published (bounded).  On a timeout (or with the debug flag
// that forces one) record it in the status block and return NaN: the corruption then shows in the
// outputs.
// Granules requested together by one import batch (register budget: 2 VGPRs each).
constexpr int kImportBatch = 4;
// Batched form for the chunk imports: the granules row[t0 + s * stride] (s < C; outside [lo, hi):
// 0) are all requested before the first wait, so a chunk costs one memory round trip, not C; only
// the still-unpublished ones are polled again.
template <int C, bool Sys = false>
__device__ __forceinline__ void wait_granules(const double* row, int64_t t0, int stride, int64_t lo, int64_t hi,
                                              double (&out)[C], unsigned* status, int bid, bool force_timeout) {
  auto ld = [](const double* p) { return Sys ? load_granule_sys(p) : load_granule(p); };
  unsigned long long v[C];
  unsigned pend = 0;
#pragma unroll
  for (int s = 0; s < C; ++s) {
    const int64_t t = t0 + (int64_t)s * stride;
    v[s] = (t >= lo && t < hi) ? ld(row + t) : 0ull;  // +0.0 outside the window
  }
#pragma unroll
  for (int s = 0; s < C; ++s) pend |= (v[s] == kSentinel ? 1u : 0u) << s;
  unsigned spins = 0;
  while (pend != 0u || force_timeout) {
    ++spins;
    // a hand-off already failed in this launch (e.g. a split-basin peer that never arrives): give up
    // at once instead of spinning out every later wait too
    const bool failed = (spins & 1023u) == 0u &&
                        __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
    if (force_timeout || failed || spins > (1u << 24)) {
      atomicAdd(status, 1u);
      atomicCAS(status + 1, 0u, (unsigned)bid + 1u);
#pragma unroll
      for (int s = 0; s < C; ++s) {
        const int64_t t = t0 + (int64_t)s * stride;
        const bool nan = ((pend >> s) & 1u) || (force_timeout && t >= lo && t < hi);
        v[s] = nan ? 0x7FF8000000000000ull : v[s];
      }
      break;
    }
    __builtin_amdgcn_s_sleep(2);
#pragma unroll
    for (int s = 0; s < C; ++s) {
      const unsigned long long w = ((pend >> s) & 1u) ? ld(row + (t0 + (int64_t)s * stride)) : v[s];
      v[s] = w;
      pend &= ~((w != kSentinel ? 1u : 0u) << s);
    }
  }
#pragma unroll
  for (int s = 0; s < C; ++s) out[s] = __longlong_as_double(v[s]);
}

// Split form of wait_granules for imports requested a chunk ahead: issue_granules requests the granules
// (no wait: they land while the block runs on), poll_granules waits for the still-unpublished ones with the
// same bounds and failure handling as wait_granules.
template <int C, bool Sys>
__device__ __forceinline__ void issue_granules(const double* row, int64_t t0, int64_t lo, int64_t hi,
                                               unsigned long long (&v)[C]) {
#pragma unroll
  for (int s = 0; s < C; ++s) {
    const int64_t t = t0 + s;
    v[s] = (t >= lo && t < hi) ? (Sys ? load_granule_sys(row + t) : load_granule(row + t)) : 0ull;
  }
}
template <int C, bool Sys>
__device__ __forceinline__ void poll_granules(const double* row, int64_t t0, int64_t lo, int64_t hi,
                                              unsigned long long (&v)[C], double (&out)[C], unsigned* status, int bid,
                                              bool force_timeout) {
  auto ld = [](const double* p) { return Sys ? load_granule_sys(p) : load_granule(p); };
  unsigned pend = 0;
#pragma unroll
  for (int s = 0; s < C; ++s) pend |= (v[s] == kSentinel ? 1u : 0u) << s;
  unsigned spins = 0;
  while (pend != 0u || force_timeout) {
    ++spins;
    const bool failed = (spins & 1023u) == 0u &&
                        __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
    if (force_timeout || failed || spins > (1u << 24)) {
      atomicAdd(status, 1u);
      atomicCAS(status + 1, 0u, (unsigned)bid + 1u);
#pragma unroll
      for (int s = 0; s < C; ++s) {
        const int64_t t = t0 + s;
        const bool nan = ((pend >> s) & 1u) || (force_timeout && t >= lo && t < hi);
        v[s] = nan ? 0x7FF8000000000000ull : v[s];
      }
      break;
    }
    __builtin_amdgcn_s_sleep(2);
#pragma unroll
    for (int s = 0; s < C; ++s) {
      const unsigned long long w = ((pend >> s) & 1u) ? ld(row + (t0 + s)) : v[s];
      v[s] = w;
      pend &= ~((w != kSentinel ? 1u : 0u) << s);
    }
  }
#pragma unroll
  for (int s = 0; s < C; ++s) out[s] = __longlong_as_double(v[s]);
}

// Logical block of this workgroup: the next ticket of the launch (forward: blocks in piece-height
// order, backward: the reverse).  A workgroup waits only on blocks of lower logical index, whose
// tickets were taken by workgroups already running or finished: no co-residency assumption.
// The block descriptor of logical block `bid`, forced into SGPRs (behind the ticket atomic the
// compiler cannot prove the descriptor unclobbered and would load it per lane).
__device__ __forceinline__ BlockDesc block_desc(const BlockDesc* blocks, int bid) {
  const BlockDesc d = blocks[bid];
  BlockDesc u;
  u.pos0 = __builtin_amdgcn_readfirstlane(d.pos0);
  u.nloc = __builtin_amdgcn_readfirstlane(d.nloc);
  u.virt0 = __builtin_amdgcn_readfirstlane(d.virt0);
  u.nvirt = __builtin_amdgcn_readfirstlane(d.nvirt);
  u.cout0 = __builtin_amdgcn_readfirstlane(d.cout0);
  u.ncout = __builtin_amdgcn_readfirstlane(d.ncout);
  u.dmax = __builtin_amdgcn_readfirstlane(d.dmax);
  u.nxl = __builtin_amdgcn_readfirstlane(d.nxl);
  u.xl0 = __builtin_amdgcn_readfirstlane(d.xl0);
  u.pad = 0;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(d.pre_dn & 0xffffffffu));
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((unsigned long long)d.pre_dn >> 32));
  u.pre_dn = (int64_t)(((unsigned long long)hi << 32) | lo);
  return u;
}

// `slot` is a scratch LDS word that nothing else uses before the second barrier.
__device__ __forceinline__ int take_ticket(unsigned* status, int word, int nblocks, bool reverse, int* slot) {
  if (threadIdx.x == 0) {
    const int t = (int)atomicAdd(status + word, 1u);
    *slot = reverse ? nblocks - 1 - t : t;
  }
  __syncthreads();
  const int bid = __builtin_amdgcn_readfirstlane(*slot);
  __syncthreads();
  return bid;
}

// s_waitcnt vmcnt(0) (expcnt, lgkmcnt unconstrained), gfx9 encoding: an explicit wait the compiler's
// waitcnt pass sees (inline asm it would not)
constexpr unsigned kWaitVmcnt0 = 0x0F70;

// Kernel-argument constants in R (pre-rounded on the host, so they stay scalar operands).
// pin_pow: keep the fp64 constants of the correctly rounded pow in VGPRs (kernels that evaluate it).
// opq_inf: the clamps' infinity opaque to the compiler (rmaxc: one v_med3_f32 per clamp; the KR = 4 kernels)
template <typename R>
__device__ __forceinline__ Consts<R> consts_of(const RouteArgs& a, bool pin_pow = true, bool opq_inf = false);
template <>
__device__ __forceinline__ Consts<float> consts_of<float>(const RouteArgs& a, bool pin_pow, bool opq_inf) {
  return Consts<float>{a.cf[0], a.cf[1], a.cf[2], a.cf[3], a.cf[4], a.cf[5], a.cf[6], a.cf[7],
                       pin_pow ? pow_consts_vgpr() : pow_consts(), a.ln_dlb,
                       opq_inf ? opaque_inf(__builtin_inff()) : __builtin_inff()};
}
template <>
__device__ __forceinline__ Consts<double> consts_of<double>(const RouteArgs& a, bool, bool) {
  return Consts<double>{a.c[0], a.c[1], a.c[2], a.c[3], a.c[4], a.c[5], a.c[6], a.c[7], pow_consts(), a.ln_dlb};
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

// Packed upstream descriptor: u0 (13 bits) | f1 (13 bits) << 13 | min(nup, 15) << 26; a missing
// upstream reads slot `none` (the forward's zero slot).  f1 is the second upstream's slot, or for a
// confluence (nup > 2) the offset of its list [c, u1, ..., u_{c-1}] in the block's LDS copy of
// xlist: every upstream index of a tick comes from registers or LDS, never from a global load (whose
// wait would also drain the tick's prefetches, in-order vmcnt).
__device__ __forceinline__ unsigned pack_up(const RouteArgs& a, int P, unsigned none = 0u) {
  const int b = a.s.upb[P], c = a.s.upc[P];
  const unsigned u0 = c > 0 ? (unsigned)a.s.uplist[b] : none;
  const unsigned u1 = c > 2 ? (unsigned)a.s.xoff[P] : (c > 1 ? (unsigned)a.s.uplist[b + 1] : none);
  return u0 | (u1 << 13) | ((unsigned)(c < 15 ? c : 15) << 26);
}
// Copy the block's confluence lists into LDS (all threads; the caller synchronises).
__device__ __forceinline__ void load_xlist(const RouteArgs& a, const BlockDesc& B, int* xl) {
  for (int i = threadIdx.x; i < B.nxl; i += blockDim.x) xl[i] = a.s.xlist[B.xl0 + i];
}
// Make a per-reach value opaque inside the tick loop so the compiler recomputes what it derives
// from it (64-bit addresses, qe + 1, ...) each tick instead of hoisting and keeping it live: at
// KR reaches per thread the hoisted copies, not the state, exhaust the register file.
template <typename V>
__device__ __forceinline__ V opq(V x) {
  asm volatile("" : "+v"(x));
  return x;
}
__device__ __forceinline__ int up_n(unsigned u) { return (int)(u >> 26); }
// 16-B runoff row segments (plain stores: measured faster than 8-B segments and than nt stores)
__device__ __forceinline__ void store4(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
}
// a dL/drunoff group (each 16-B piece of a row is read once per launch; plain loads: nt measured slower)
__device__ __forceinline__ float4 load_grad4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void store4(double* p, double a, double b, double c, double d) {
  reinterpret_cast<double2*>(p)[0] = make_double2(a, b);
  reinterpret_cast<double2*>(p)[1] = make_double2(c, d);
}
__device__ __forceinline__ int up_0(unsigned u) { return (int)(u & 8191u); }
__device__ __forceinline__ int up_f1(unsigned u) { return (int)((u >> 13) & 8191u); }
// slot of the second upstream (a confluence's from its LDS list)
__device__ __forceinline__ int up_1(unsigned u, const int* xl) { return up_n(u) > 2 ? xl[up_f1(u) + 1] : up_f1(u); }

// Debug per-workgroup profile (ddr_set_block_profile): start, end, import wait, hardware id.
// Layout per workgroup: kProfWords uint64 = start, end, wait, hwid, then a timestamp every 1024 ticks.
constexpr int kProfWords = 16;
__device__ __forceinline__ void prof_begin(unsigned long long* p, int bid) {
  p += kProfWords * bid;
  p[0] = __builtin_amdgcn_s_memrealtime();
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
  p[3] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
}
__device__ __forceinline__ void prof_tick(unsigned long long* p, int bid, int tick) {
  if ((tick & 1023) == 0 && (tick >> 10) < kProfWords - 4)
    p[kProfWords * bid + 4 + (tick >> 10)] = __builtin_amdgcn_s_memrealtime();
}
__device__ __forceinline__ void prof_end(unsigned long long* p, int bid, unsigned long long wait) {
  p += kProfWords * bid;
  p[1] = __builtin_amdgcn_s_memrealtime();
  p[2] = wait;
}

// Debug phase profile (-DDDR_PHASE_PROF=1 builds only): every wave accumulates the s_memtime cycles of
// each tick phase; at the end lane 0 writes them after the per-block words of the profile buffer:
// prof[kProfWords * nblocks + (bid * 16 + wave) * kPhases + phase].
#ifndef DDR_PHASE_PROF
#define DDR_PHASE_PROF 0
#endif
struct PhaseProf {
#if DDR_PHASE_PROF
  static constexpr int kPhases = 8;
  unsigned long long acc[kPhases] = {};
  unsigned long long t0 = 0;
  __device__ __forceinline__ void start() { t0 = __builtin_amdgcn_s_memtime(); }
  __device__ __forceinline__ void mark(int ph) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    acc[ph] += t - t0;
    t0 = t;
  }
  __device__ __forceinline__ void flush(unsigned long long* prof, int nblocks, int bid) {
    if (!prof || (threadIdx.x & 63)) return;
    unsigned long long* q = prof + (size_t)kProfWords * nblocks + ((size_t)bid * 16 + (threadIdx.x >> 6)) * kPhases;
    for (int i = 0; i < kPhases; ++i) q[i] = acc[i];
  }
#else
  __device__ __forceinline__ void start() {}
  __device__ __forceinline__ void mark(int) {}
  __device__ __forceinline__ void flush(unsigned long long*, int, int) {}
#endif
};

}  // namespace

// Per-reach statics in LDS, interleaved [slot][6] (n, qe, p, sqrtS, L, X): one get is three
// 2-element LDS reads at immediate offsets (lane stride 24 B: conflict-free).  The derived fields
// (dd, expo, 1/n) are recomputed on read (derive_static), or taken from registers (get_pre).
template <typename R>
struct StatTab {
  R* s;
  using V2 = typename std::conditional<sizeof(R) == 4, float2, double2>::type;
  __device__ __forceinline__ void put(int r, const ReachStatic<R>& v) const {
    R* q = s + 6 * r;
    q[0] = v.n;
    q[1] = v.qe;
    q[2] = v.p;
    q[3] = v.sqrtS;
    q[4] = v.L;
    q[5] = v.X;
  }
  template <bool Fast = false>
  __device__ __forceinline__ ReachStatic<R> get(int r) const {
    const V2* q = reinterpret_cast<const V2*>(s + 6 * r);
    const V2 a = q[0], b = q[1], c = q[2];
    return derive_static<R, Fast>(a.x, a.y, b.x, b.y, c.x, c.y);
  }
  __device__ __forceinline__ ReachStatic<R> get_pre(int r, R expo, R inv_n) const {
    const V2* q = reinterpret_cast<const V2*>(s + 6 * r);
    const V2 a = q[0], b = q[1], c = q[2];
    ReachStatic<R> v;
    v.n = a.x;
    v.qe = a.y;
    v.p = b.x;
    v.sqrtS = b.y;
    v.dd = (b.x * b.y) + R(1e-8);
    v.expo = expo;
    v.inv_n = inv_n;
    v.L = c.x;
    v.X = c.y;
    return v;
  }
};

// The gathered q' * flow_scale of local position r running step t = tau - off at forward tick tau:
// the tick-major schedule layout (row tau), or the row layout of a multi-hour store (choose_qs_layout).
template <typename R>
__device__ __forceinline__ const R* qs_at(const RouteArgs& a, const BlockDesc& B, int64_t xs_base, int tau, int off,
                                          int r) {
  const R* qs = static_cast<const R*>(a.qs);
  if (a.qs_rows > 0) {
    int t = tau - off;
    t = t < 0 ? 0 : (t >= (int)a.T ? (int)a.T - 1 : t);
    t = t > a.qp_shift ? t - a.qp_shift : 0;
    const unsigned row = __umulhi((unsigned)t, a.qp_magic);  // t / qp_hours
    return qs + (int64_t)a.qs_rows * B.pos0 + (int64_t)row * B.nloc + r;
  }
  return qs + xs_base + (int64_t)tau * B.nloc + r;
}

// ============================================================================================
// Forward
// ============================================================================================
// Tick structure (one LDS slot per reach, single-buffered):
//   [import a chunk of virtual inflows]  prefetch q' of the next tick
//   compute: every reach reads its upstream x_j(t) from the slots (written last tick), runs the
//            physics and the fp64 column sweep, keeps x in a register          -- barrier --
//   publish: x into the reach's own slot (and virtual inflows into theirs)      -- barrier --
// The inflow I(t+1) = sum_j Q_j(t) is formed from the same x_j(t) reads (Q_j = clamp(x_j)).
// FM (fp32 only, DDR_FWD_FAST_MATH): the coefficients in hardware-approximate fp32 math
// (coefficients_fast, the operation set of the adjoint's recompute) instead of the reference's exact
// operation sequence; ~1e-6 relative per coefficient, and few enough registers that all of a
// thread's slices run their physics in lockstep.
// MATH: 0 exact (reference op order, correctly rounded pow), 1 fast (DDR_FWD_FAST_MATH), 2 faithful
// (DDR_FWD_FAITHFUL_MATH: exact op order and IEEE divisions, fp32 faithful-class pow).
// XB: the x slots' buffer count when not the KR rule's (fwd_xbuf): 2 = parity-indexed slots and one barrier
// per tick at KR = 4 too, where the launch finds the LDS for them (launch_route_kr)
// PL (plain): the launch has none of the rarely used options -- no split basin, no profile, no daily
// accumulation -- and 1: runoff written with 16-B rows, q' from the tick-major gather; 2: no runoff (gauge mode),
// tick-major q'; 4: no runoff, q' from the row layout (daily q', qs_rows); so their tests and the uniform values
// behind them (held in scalar registers, spilled at KR = 4) leave the tick loop (C5 forward -6 %, C4 -8 %,
// C2 -15 %: profiles/r05/ab_r05.txt item 11)
template <typename R, int KR, int MATH, int XB = 0, int PL = 0>
__global__ void __launch_bounds__(kBlockThreads, kBlocksPerCU * kBlockThreads / 256) route_forward_kernel(RouteArgs a) {
  constexpr int BS = kBlockThreads;
  constexpr bool kFast = MATH == 1 && std::is_same<R, float>::value;
  constexpr bool kFaith = MATH == 2 && std::is_same<R, float>::value;
  // one slice's physics at a time (lockstep slice pairs, plain or in packed halves, measured slower:
  // DESIGN section 4)
  constexpr int NP = 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int bid = take_ticket(a.status, kStatusTicketFwd, a.nblocks, false, reinterpret_cast<int*>(smem));
  if (a.owned && !a.owned[bid]) return;  // split basin: another rank's block
  const BlockDesc B = block_desc(a.s.blocks, bid);
  const int tid = threadIdx.x;
  // first lane of this wave (scalar): waves with no reach in slice k skip it (scalar branch),
  // so a workgroup's tick costs ceil(nloc / 64) wave-slices, not KR * waves
  const int wbase = __builtin_amdgcn_readfirstlane(tid & ~63);
  const int S = a.slot_stride;
  // kDbl: [2][S] x slots by tick parity -- tick tau reads buffer (tau - 1) & 1 and writes its results
  // straight into buffer tau & 1, one workgroup barrier per tick; else [S], written in a publish phase
  // between two barriers
  constexpr int kXBuf = XB > 0 ? XB : fwd_xbuf(KR);
  constexpr bool kDbl = kXBuf == 2;
  double* sx = reinterpret_cast<double*>(smem + kMathTabBytes);         // [kXBuf][S] x_j(t), solve precision
  const StatTab<R> tab{reinterpret_cast<R*>(sx + kXBuf * S)};           // [S][6]
  double* ring = reinterpret_cast<double*>(smem + kMathTabBytes + align16(size_t(S) * (8 * kXBuf + 6 * sizeof(R))));  // [nvirt][kChunkFwd]
  int* xl = reinterpret_cast<int*>(smem + a.xl_off);                     // confluence lists
  const Consts<R> cs = consts_of<R>(a, !kFast && !kFaith, KR >= kOpqInfMinKR);
  const int64_t T = a.T;
  const bool carry = a.flags & DDR_FWD_CARRY;
  const bool accum = !PL && (a.flags & DDR_FWD_ACCUMULATE);  // every step a hot start (daily accumulation)
  auto* const aprof = PL ? nullptr : a.prof;  // per-block tick profile (--block-profile)
  const int32_t xt_off = PL ? 0 : a.xt_off;   // split basin: the export-row table
  const bool force_to = a.flags & kFlagForceTimeout;
  R* xsave = static_cast<R*>(a.x_save);
  const int TTf = (int)T + B.dmax;
  const R* q0p = static_cast<const R*>(a.q0);
  const int64_t xs_base = T * B.pos0 + B.pre_dn;

  // off: tick offset (low 16 bits) | 1 + rank among the block's cut reaches (high 16, 0 = not cut;
  // its boundary granule row is B.cout0 + rank, graph.cpp numbers cut edges that way)
  int ref[KR], off[KR];
  unsigned up[KR];
  auto off_of = [&](int k) { return off[k] & 0xFFFF; };
  R Q[KR], In[KR], qa[KR], qb[KR], ex[KR], inv[KR];  // ex, inv: the static divisions, kept in registers
  // one reach per thread (small blocks: light loads, where a tick is one dependency chain long): the
  // statics stay in registers, off the chain's LDS round trips
  constexpr bool kStatReg = KR == 1 && sizeof(R) == 4;
  ReachStatic<R> sreg[kStatReg ? KR : 1];
  // runoff (N, T) written from here: the last four steps of each reach, stored 16 B at a time
  R ob0[KR], ob1[KR], ob2[KR], ob3[KR];
  R* runoff = static_cast<R*>(a.runoff);
  const bool emit = PL == 1 || (PL == 0 && runoff != nullptr && !(a.flags & DDR_FWD_NO_RUNOFF));
  // rows 16-B aligned: vector stores (per-step 4-B stores measured 1.6x slower for the whole kernel)
  const bool emit4 = PL == 1 || (T & 3) == 0;
  // Storer waves (one reach per thread, blocks of at most half a workgroup): the idle upper half of the
  // workgroup stores each reach's published x (x_save row, runoff) during the next tick, so a compute
  // wave's top-of-tick wait covers only its q' prefetch -- not the acknowledgement of its stores, which
  // is on a light block's critical path (up to 12 % of a C2 tick, profiles/r03/ab_r03.txt item 5).
  // The storers export the cut reaches' granules too: a cut reach's x reaches its consumer one tick later
  // (pipeline latency of that hand-off only), and no compute wave waits for a store at all.
  // Imports requested a chunk ahead (KR <= 2: registers for the chunk's raw granules).
  constexpr bool kPrefImport = KR <= 2;
  unsigned long long pfg[kChunkFwd];
#pragma unroll
  for (int i = 0; i < kChunkFwd; ++i) pfg[i] = 0ull;
  const bool storer_mode = KR == 1 && !(a.flags & kFlagNoStorer) && B.nloc <= BS / 2;
  const bool storer_wave = storer_mode && wbase >= BS / 2;
  const int sr = tid - BS / 2;  // a storer thread's reach
  int sref = 0, soff = 0;  // soff: tick offset | 1 + cut rank << 16, as off[]
  if (storer_wave && sr < B.nloc) {
    sref = a.s.ref[B.pos0 + sr];
    const int e = a.s.cut[B.pos0 + sr];
    soff = a.s.off[B.pos0 + sr] | (e >= 0 ? (e - B.cout0 + 1) << 16 : 0);
  }
#pragma unroll
  for (int k = 0; k < KR; ++k) {
    const int r = tid + k * BS;
    const bool hk = r < B.nloc;
    const int P = B.pos0 + (hk ? r : 0);
    ref[k] = a.s.ref[P];
    const int e = a.s.cut[P];
    off[k] = a.s.off[P] | (e >= 0 ? (e - B.cout0 + 1) << 16 : 0);
    up[k] = pack_up(a, P, (unsigned)(S - 1));  // slot S-1 holds 0: missing upstreams add exactly 0
    Q[k] = In[k] = R(0);
    qa[k] = qb[k] = R(0);
    ob0[k] = ob1[k] = ob2[k] = ob3[k] = R(0);
    const ReachStatic<R> st = load_static<R>(a, ref[k]);
    ex[k] = st.expo;
    inv[k] = st.inv_n;
    if (hk) tab.put(r, st);
    if constexpr (kStatReg) sreg[k] = tab.get_pre(hk ? r : 0, st.expo, st.inv_n);  // the values the LDS path reads
  }
  if (tid == 0) sx[S - 1] = 0.0;
  if (kDbl && tid == 0) sx[2 * S - 1] = 0.0;
  // virtual inflow vi is imported and published by thread BS - 1 - vi: the owners sit in the last
  // waves, which hold fewer wave-slices than wave 0 when nloc is not a multiple of 1024 (the import's
  // global round trip lands on the lighter waves; only the owner reads its ring entries, so the import
  // needs no workgroup barrier)
  const int vi = BS - 1 - tid;
  const bool vown = vi < B.nvirt;
  int v_off = 0, v_edge = 0;
  if (vown) {
    v_off = a.s.v_off[B.virt0 + vi];
    v_edge = a.s.v_edge[B.virt0 + vi];
  }
  load_math_tables();
  load_xlist(a, B, xl);
  uintptr_t* xt = reinterpret_cast<uintptr_t*>(smem + xt_off);  // split: cut-outs' export rows
  if (xt_off) {
    for (int c = tid; c < B.ncout; c += BS) {
      const int64_t e = B.cout0 + c;
      const int xi = a.xid[e];
      xt[c] = xi >= 0 ? (reinterpret_cast<uintptr_t>(a.pxfwd[a.xcons[xi]] + (int64_t)xi * T) | 1u)
                      : reinterpret_cast<uintptr_t>(a.bnd + e * T);
    }
  }
  __syncthreads();
  unsigned long long prof_wait = 0;
  if (aprof && tid == 0) prof_begin(aprof, bid);
  PhaseProf phz;
  phz.start();

  // q'[max(t-1,0)] * flow_scale (gathered into the schedule layout: one row per tick), or the
  // carried Q0 at t = 0, for the step each reach runs at tick `tau`
  const R* qsb = static_cast<const R*>(a.qs) + xs_base;
  const bool qs_rows = PL == 4 || (PL == 0 && a.qs_rows > 0);
  // kSt (steady ticks, below): no reach is at its carried t = 0 step
  auto prefetch = [&](int tau, R(&dst)[KR], int tq0, auto sc) {
    constexpr bool kSt = decltype(sc)::value;
    const R* row = qsb + (int64_t)(tau < TTf ? tau : TTf - 1) * B.nloc;
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      if (wbase + k * BS >= B.nloc) continue;
      const int r = tq0 + k * BS;
      const int rs = r < B.nloc ? r : 0;
      const R v = qs_rows ? *qs_at<R>(a, B, xs_base, tau, off_of(k), rs) : row[rs];
      dst[k] = (!kSt && carry && tau == off_of(k)) ? q0p[ref[k]] : v;
    }
  };

  // sc: std::integral_constant<bool, kSt>.  Steady ticks (tau in [dmax + 1, T - 1]) are those at which
  // every reach of the block runs a step t in [1, T - 1]: no activity tests, no idle-slice ballot, no
  // hot start or carried-state case -- the same operations on the same values as the general tick
  // storer threads: the stores of the x their reach published at tick `taup` (read from its slot before
  // the next publish overwrites it); the same values and rounding as the compute waves' stores
  auto store_pass = [&](int taup) {
    if (sr >= B.nloc) return;
    const int so = opq(soff);
    const int t = taup - (so & 0xFFFF);
    if (t < 0 || t >= T) return;
    const double xd = sx[(kDbl ? (taup & 1) * S : 0) + sr];
    const R xr = R(xd);
    if (B.ncout > 0 && (so >> 16)) {
      const int64_t e = B.cout0 + (so >> 16) - 1;
      if (xt_off) {
        const uintptr_t p = xt[(so >> 16) - 1];
        double* row = reinterpret_cast<double*>(p & ~uintptr_t(1));
        if (p & 1u) store_granule_sys(row + t, xd);
        else store_granule(row + t, xd);
      } else {
        store_granule(a.bnd + e * T + t, xd);
      }
    }
    static_cast<R*>(a.x_save)[xs_base + (int64_t)taup * B.nloc + sr] = xr;
    if (emit) {
      ob0[0] = ob1[0];
      ob1[0] = ob2[0];
      ob2[0] = ob3[0];
      ob3[0] = rmax_nan(xr, cs.qlb);
      R* orow = runoff + (int64_t)opq(sref) * T;
      if (!emit4) orow[t] = ob3[0];
      else if ((t & 3) == 3) store4(orow + (t - 3), ob0[0], ob1[0], ob2[0], ob3[0]);
    }
  };

  // the import of the next chunk of every virtual inflow, at ticks tau = 0 mod kChunkFwd (owners only)
  auto import_chunk = [&](int tau) {
    if (B.nvirt > 0 && (tau % kChunkFwd) == 0) {
      // import the next chunk of every virtual inflow (x of the upstream block's reach): its owner
      // thread requests the kChunkFwd granules at once
      const unsigned long long w0 = aprof ? __builtin_amdgcn_s_memrealtime() : 0;
      if (kPrefImport && vown) {
        // (light and medium loads) the chunk was requested one chunk ago: its granules have landed while
        // the block ran, so the import waits only for those still unpublished, and the next chunk is
        // requested now -- the owner's wave (and the barrier after it) no longer pays a memory round
        // trip every kChunkFwd ticks
        const int xi = (!PL && a.xid) ? a.xid[v_edge] : -1;  // split basin: another rank's block, receive rows
        const double* row = xi >= 0 ? a.xfwd + (int64_t)xi * T : a.bnd + (int64_t)v_edge * T;
        const int64_t t0 = (int64_t)tau - v_off;
        double g[kChunkFwd];
        if (xi >= 0) {
          if (tau == 0) issue_granules<kChunkFwd, true>(row, t0, 0, T, pfg);
          poll_granules<kChunkFwd, true>(row, t0, 0, T, pfg, g, a.status, bid, force_to);
          issue_granules<kChunkFwd, true>(row, t0 + kChunkFwd, 0, T, pfg);
        } else {
          if (tau == 0) issue_granules<kChunkFwd, false>(row, t0, 0, T, pfg);
          poll_granules<kChunkFwd, false>(row, t0, 0, T, pfg, g, a.status, bid, force_to);
          issue_granules<kChunkFwd, false>(row, t0 + kChunkFwd, 0, T, pfg);
        }
#pragma unroll
        for (int i = 0; i < kChunkFwd; ++i) ring[vi * kChunkFwd + i] = g[i];
      } else if (vown) {
        // split basin: a cut edge from another rank's block arrives in this rank's receive rows
        const int xi = (!PL && a.xid) ? a.xid[v_edge] : -1;
        if (xi >= 0) {
#pragma unroll
          for (int h = 0; h < kChunkFwd; h += kImportBatch) {
            double g[kImportBatch];
            wait_granules<kImportBatch, true>(a.xfwd + (int64_t)xi * T, (int64_t)tau - v_off + h, 1, 0, T, g, a.status,
                                              bid, force_to);
#pragma unroll
            for (int i = 0; i < kImportBatch; ++i) ring[vi * kChunkFwd + h + i] = g[i];
          }
        } else {
#pragma unroll
          for (int h = 0; h < kChunkFwd; h += kImportBatch) {
            double g[kImportBatch];
            wait_granules<kImportBatch>(a.bnd + (int64_t)v_edge * T, (int64_t)tau - v_off + h, 1, 0, T, g, a.status,
                                        bid, force_to);
#pragma unroll
            for (int i = 0; i < kImportBatch; ++i) ring[vi * kChunkFwd + h + i] = g[i];
          }
        }
      }
      if (aprof) prof_wait += __builtin_amdgcn_s_memrealtime() - w0;
    }
  };
  // a virtual inflow's value of tick tau into its slot of buffer `dst` (owners only)
  auto publish_virt = [&](int tau, double* dst) {
    if (vown) {
      const int t = tau - v_off;
      if (t >= 0 && t < T) dst[B.nloc + vi] = ring[vi * kChunkFwd + (tau % kChunkFwd)];
    }
  };

  // One tick of the waves that route reaches (every wave outside storer mode)
  auto tick = [&](int tau, R(&qcur)[KR], R(&qnext)[KR], auto sc) {
    constexpr bool kSt = decltype(sc)::value;
    // the previous tick's q' prefetch and stores land here (see the backward kernel's tick); unconditional,
    // so the compiler's own wait analysis sees no load outstanding past it (a wait it could not prove made
    // it wait again, vmcnt(0), at the first use of qcur -- after this tick's prefetch was issued)
    __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
    if constexpr (KR == 4) set_prio(3);
    if constexpr (KR == 1) __builtin_amdgcn_s_setprio(1);
    phz.mark(0);  // the previous tick's loads and stores
    // opaque per tick: everything derived from them (LDS / global offsets, masks) is recomputed
    // instead of being hoisted into registers held across the loop
    const int tq = opq(tid);
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      ref[k] = opq(ref[k]);
      off[k] = opq(off[k]);
      up[k] = opq(up[k]);
      ex[k] = opq(ex[k]);
      inv[k] = opq(inv[k]);
    }
    import_chunk(tau);
    phz.mark(1);  // import
    prefetch(tau + 1, qnext, tq, sc);
    R* xrow = xsave + xs_base + (int64_t)tau * B.nloc;  // this tick's row of the state layout
    double xk[KR];
    const double* sxr = sx + (kDbl ? ((tau + 1) & 1) * S : 0);  // the slots published at tick tau - 1
    double* sxw = sx + (kDbl ? (tau & 1) * S : 0);              // (kDbl) this tick's results
    // ---- compute, NP slices at a time: their physics in lockstep (NP independent dependency
    //      chains per wave: the tick is latency-bound at 4 waves per SIMD), then per slice the
    //      fp64 column sweep and the stores -------------------------------------------------------
#pragma unroll
    for (int k0 = 0; k0 < KR; k0 += NP) {
      if (wbase + k0 * BS >= B.nloc) continue;
      if constexpr (KR == 4) set_prio(KR - 1 - k0);
      if (!kSt) {
        // no lane of the wave runs a step this tick (before its first / after its last step: the
        // first and last dmax ticks of a block, most ticks of a short window): skip the slice
        bool act = false;
#pragma unroll
        for (int h = 0; h < NP; ++h) {
          const int t = tau - off_of(k0 + h);
          act = act || (tq + (k0 + h) * BS < B.nloc && t >= 0 && t < T);
        }
        if (__builtin_amdgcn_ballot_w64(act) == 0) continue;
      }
      ReachStatic<R> st[NP];
      R Qv[NP];
      PhysOut<R> ph[NP];
      // the upstream slots first: they do not depend on the physics, so their LDS latency hides under it
      // (the second upstream's slot is the packed word's f1; a confluence's comes from its list below)
      double x0a[NP], x1a[NP];
#pragma unroll
      for (int h = 0; h < NP; ++h) {
        x0a[h] = sxr[up_0(up[k0 + h])];
        x1a[h] = sxr[up_n(up[k0 + h]) > 2 ? S - 1 : up_f1(up[k0 + h])];  // (a list offset is not a slot)
      }
#pragma unroll
      for (int h = 0; h < NP; ++h) {
        const int r = tq + (k0 + h) * BS;
        if constexpr (kStatReg) st[h] = sreg[k0 + h];
        else st[h] = tab.get_pre(r < B.nloc ? r : 0, ex[k0 + h], inv[k0 + h]);
        Qv[h] = Q[k0 + h];
      }
      if (!accum) {
        if constexpr (kFast) {
#pragma unroll
          for (int h = 0; h < NP; ++h) ph[h] = coefficients_fast(st[h], Qv[h], cs);
        } else if constexpr (kFaith) {
#pragma unroll
          for (int h = 0; h < NP; ++h) ph[h] = coefficients_faithful(st[h], Qv[h], cs);
        } else {
          coefficients_np<R, NP>(st, Qv, cs, ph);
        }
      } else {
#pragma unroll
        for (int h = 0; h < NP; ++h) ph[h] = PhysOut<R>{R(0), R(0), R(0), R(0), R(0), R(0)};
      }
      if constexpr (KR == 1) __builtin_amdgcn_s_setprio(0);
#pragma unroll
      for (int h = 0; h < NP; ++h) {
        const int k = k0 + h;
        const int r = tq + k * BS;
        const bool hk = r < B.nloc;
        const int t = tau - off_of(k);
        const int nup = up_n(up[k]);
        const R qv = qcur[k];  // q' * flow_scale (mmc.py:303-304), applied by the gather
        const R qc = rmaxc(qv, cs.qlb, cs);                                        // mmc.py:421-424
        const R b = ((ph[h].c2 * In[k]) + (ph[h].c3 * Q[k])) + (ph[h].c4 * qc);  // mmc.py:535-538
        const double x0v = x0a[h];
        double x1v = x1a[h];
        if (nup > 2) x1v = sxr[xl[up_f1(up[k]) + 1]];  // a confluence: its list [c, u1, ...]
        // Q_j(t) of the upstream reaches (mmc.py:557; the carried state at t = 0 is not clamped)
        const bool raw = !kSt && (t == 0 && carry);
        auto qf = [&](double x) -> R {
          const R xr = R(x);
          return raw ? xr : rmaxc(xr, cs.qlb, cs);
        };
        const double dc1 = (double)ph[h].c1;
        double acc = (double)b;                                         // utils.py:587-600 (fp64)
        acc = acc + dc1 * x0v;                                          // (+ 0 for a missing upstream)
        acc = acc + dc1 * x1v;
        double hot = 0.0;
        if constexpr (!kSt) {
          hot = (double)qv;                                             // mmc.py:25-66 (hot start)
          hot = hot + x0v;
          hot = hot + x1v;
        }
        R inn = R(0);                                                   // I(t+1) = N @ Q_t, ascending columns
        inn = inn + (nup > 0 ? qf(x0v) : R(0));
        inn = inn + (nup > 1 ? qf(x1v) : R(0));
        if (nup > 2) {
          const int* lst = xl + up_f1(up[k]);
          const int c = lst[0];
          for (int j = 2; j < c; ++j) {
            const double xj = sxr[lst[j]];
            acc = acc + dc1 * xj;
            if constexpr (!kSt) hot = hot + xj;
            inn = inn + qf(xj);
          }
        }
        const double x = kSt ? acc : ((t == 0 && carry) ? (double)qcur[k] : ((t == 0 || accum) ? hot : acc));
        xk[k] = x;
        if (kDbl && hk && (kSt || (t >= 0 && t < T))) sxw[r] = x;  // published: read at tick tau + 1
        if (hk && (kSt || (t >= 0 && t < T))) {
          const R xr = R(x);
          const R Qn = raw ? xr : rmax_nan(xr, cs.qlb);
          const bool own_st = !storer_mode;  // (storer mode: the upper waves store)
          if (own_st) xrow[r] = xr;  // the routing state for the adjoint
          if (emit && own_st) {
            // runoff[ref, t] = max(x(t), qlb)  (mmc.py:412 for t = 0, mmc.py:557 after every step)
            ob0[k] = ob1[k];
            ob1[k] = ob2[k];
            ob2[k] = ob3[k];
            ob3[k] = rmax_nan(xr, cs.qlb);
            R* orow = runoff + (int64_t)ref[k] * T;
            if (!emit4) orow[t] = ob3[k];
            else if ((t & 3) == 3) store4(orow + (t - 3), ob0[k], ob1[k], ob2[k], ob3[k]);
          }
          if (B.ncout > 0 && (off[k] >> 16) && !storer_mode) {
            const int64_t e = B.cout0 + (off[k] >> 16) - 1;
            if (xt_off) {  // split basin: the row from the block's table (another rank's: system scope)
              const uintptr_t p = xt[(off[k] >> 16) - 1];
              double* row = reinterpret_cast<double*>(p & ~uintptr_t(1));
              if (p & 1u) store_granule_sys(row + t, x);
              else store_granule(row + t, x);
            } else {
              store_granule(a.bnd + e * T + t, x);
            }
          }
          // (the last step's Q, top width and side slope: route_last_kernel, from the saved states --
          // no rarely taken stores, and no pointers held across the tick loop for them)
          Q[k] = Qn;
          In[k] = inn;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (kDbl) {
      // the virtual inflows' values of this tick, beside the reaches' (owners only read their own ring)
      publish_virt(tau, sxw);
      phz.mark(2);  // prefetch issue + compute + publish
      lds_barrier();
      phz.mark(3);  // the tick's one barrier
      return;
    }
    phz.mark(2);  // prefetch issue + compute
    lds_barrier();
    phz.mark(3);  // barrier 1
    // ---- publish ------------------------------------------------------------------------------
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      if (wbase + k * BS >= B.nloc) continue;
      const int t = tau - off_of(k);
      const int r = tq + k * BS;
      if (r < B.nloc && (kSt || (t >= 0 && t < T))) sx[r] = xk[k];
    }
    publish_virt(tau, sx);
    phz.mark(4);  // publish
    lds_barrier();
    phz.mark(5);  // barrier 2
  };

  const int TT = (int)T + B.dmax;
  if constexpr (KR == 1) {
    if (storer_wave) {
      // Storer waves (storer mode: the upper half of the workgroup): their own loop -- the import of the
      // virtual inflows they own, the stores of the x their reach published a tick earlier, the virtuals'
      // publish and the tick's barriers -- so the routing waves' tick carries no storer branch
#pragma unroll 1
      for (int tau = 0; tau < TT; ++tau) {
        import_chunk(tau);
        if (tau > 0) store_pass(tau - 1);
        if constexpr (kDbl) {
          publish_virt(tau, sx + (tau & 1) * S);
          lds_barrier();
        } else {
          lds_barrier();
          publish_virt(tau, sx);
          lds_barrier();
        }
      }
      store_pass(TT - 1);  // the last tick's publish (its barrier has passed)
      return;
    }
  }
  using Gen = std::integral_constant<bool, false>;
  using Steady = std::integral_constant<bool, true>;
  prefetch(0, qa, tid, Gen{});
  // two ticks per iteration, the prefetch registers swapping roles: copying the prefetched q'
  // (qa = qb) at the loop latch would wait for the loads just issued, and for every store of the tick.
  // Steady ticks [s0, s1) (even bounds, so the roles keep alternating) between the ramps.
  int s0 = B.dmax + 1, s1 = (int)T & ~1;
  s0 += s0 & 1;
  if ((a.flags & kFlagNoSteady) || accum || s1 <= s0) s0 = s1 = 0;
#pragma unroll 1
  for (int tau = 0; tau < s0; tau += 2) {
    if (aprof && tid == 0) prof_tick(aprof, bid, tau);
    tick(tau, qa, qb, Gen{});
    tick(tau + 1, qb, qa, Gen{});
  }
#pragma unroll 1
  for (int tau = s0; tau < s1; tau += 2) {
    if (aprof && tid == 0) prof_tick(aprof, bid, tau);
    tick(tau, qa, qb, Steady{});
    tick(tau + 1, qb, qa, Steady{});
  }
#pragma unroll 1
  for (int tau = s1; tau < TT; tau += 2) {
    if (aprof && tid == 0) prof_tick(aprof, bid, tau);
    tick(tau, qa, qb, Gen{});
    if (tau + 1 < TT) tick(tau + 1, qb, qa, Gen{});
  }
  if (aprof && tid == 0) prof_end(aprof, bid, prof_wait);
  phz.flush(aprof, a.nblocks, bid);
}

// The forward's last-step outputs (mmc.py:441 _discharge_t, mmc.py:161-162 top_width / side_slope), from
// the saved states: Q(T - 1) = clamp(x(T - 1)), and the geometry of step T - 1, whose physics ran on
// Q(T - 2) -- the same operations on the same values as the routing kernel's, so the same bits.  One
// thread per internal position.
template <typename R, int MATH>
__global__ void __launch_bounds__(256) route_last_kernel(RouteArgs a) {
  load_math_tables();
  __syncthreads();
  const int64_t P = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (P >= a.N) return;
  const BlockDesc B = a.s.blocks[a.s.block_of_pos[P]];
  const int r = (int)(P - B.pos0);
  const int64_t off = a.s.off[P];
  const int ref = a.s.ref[P];
  const int64_t T = a.T;
  if (a.owned && !a.owned[a.s.block_of_pos[P]]) {  // split basin: another rank routes this reach
    const R nan = R(__builtin_nan(""));
    if (a.q_last) static_cast<R*>(a.q_last)[ref] = nan;
    if (a.tw_last) static_cast<R*>(a.tw_last)[ref] = nan;
    if (a.ss_last) static_cast<R*>(a.ss_last)[ref] = nan;
    return;
  }
  const R* xs = static_cast<const R*>(a.x_save) + T * B.pos0 + B.pre_dn;
  const bool carry = a.flags & DDR_FWD_CARRY;
  const bool accum = a.flags & DDR_FWD_ACCUMULATE;
  const Consts<R> cs = consts_of<R>(a, false);
  auto Q_at = [&](int64_t t) {  // Q(t): the carried state at t = 0 is not clamped
    const R x = xs[(t + off) * B.nloc + r];
    return (t == 0 && carry) ? x : rmax_nan(x, cs.qlb);
  };
  if (a.q_last) static_cast<R*>(a.q_last)[ref] = Q_at(T - 1);
  if (T > 1 && !accum && (a.tw_last || a.ss_last)) {
    const ReachStatic<R> st = load_static<R>(a, ref);
    const R Qv = Q_at(T - 2);
    PhysOut<R> ph;
    constexpr bool kFast = MATH == 1 && std::is_same<R, float>::value;
    constexpr bool kFaith = MATH == 2 && std::is_same<R, float>::value;
    if constexpr (kFast) {
      ph = coefficients_fast(st, Qv, cs);
    } else if constexpr (kFaith) {
      ph = coefficients_faithful(st, Qv, cs);
    } else {
      ReachStatic<R> sa[1] = {st};
      R qa[1] = {Qv};
      PhysOut<R> pa[1];
      coefficients_np<R, 1>(sa, qa, cs, pa);
      ph = pa[0];
    }
    if (a.tw_last) static_cast<R*>(a.tw_last)[ref] = ph.tw;
    if (a.ss_last) static_cast<R*>(a.ss_last)[ref] = ph.ss;
  }
}

// Q(t) of every reach, in reference order, from a forward's saved states (ddr_state_f32/f64): clamp(x(t)),
// the carried state at t = 0 unclamped (mmc.py:441, 557) -- e.g. Q(T - 2), the state the reported
// geometry of the last step was computed from (mmc.py:161-162), for that geometry's VJP
template <typename R>
__global__ void state_at_kernel(DevSchedule s, int64_t N, int64_t T, int64_t t, R qlb, int carry, const R* xsave,
                                R* out) {
  const int64_t P = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (P >= N) return;
  const BlockDesc B = s.blocks[s.block_of_pos[P]];
  const R x = xsave[T * B.pos0 + B.pre_dn + (t + s.off[P]) * B.nloc + (P - B.pos0)];
  out[s.ref[P]] = (t == 0 && carry) ? x : rmax_nan(x, qlb);
}

template <typename R>
hipError_t launch_state_at(const Graph* g, int64_t T, int64_t t, double qlb, bool carry, const R* xsave, R* out,
                           hipStream_t stream) {
  if (g->n == 0) return hipSuccess;
  hipLaunchKernelGGL(state_at_kernel<R>, dim3((unsigned)((g->n + 255) / 256)), dim3(256), 0, stream, g->dev, g->n, T, t,
                     R(qlb), carry ? 1 : 0, xsave, out);
  return hipGetLastError();
}
template hipError_t launch_state_at<float>(const Graph*, int64_t, int64_t, double, bool, const float*, float*, hipStream_t);
template hipError_t launch_state_at<double>(const Graph*, int64_t, int64_t, double, bool, const double*, double*,
                                            hipStream_t);

// one reach-step's adjoint outputs: coefficients, dL/dQ_{t-1} and the parameter gradient terms
template <typename R>
struct AdjOutR {
  R c1, c2, c3, c4, gQ, gn, gq, gp;
};

template <typename R>
struct Grad4 {
  R a, b, c, d;
};
template <typename R>
__device__ __forceinline__ Grad4<R> make_grad4(R a, R b, R c, R d) { return Grad4<R>{a, b, c, d}; }

// ============================================================================================
// Backward (adjoint)
// ============================================================================================
// Reverse ticks (backward tick tb runs forward tick tau = TT - 1 - tb: reach i at step
// t = tau - off(i), its upstream reaches at t + 1, its downstream at t - 1); per tick:
//   [import a chunk of (c1 gb, c2 gb) from downstream blocks]
//   read:    publish x(t - 2) of every reach (and of every virtual inflow, from the forward's
//            boundary granules) into its slot; read the downstream reach's (c1_d gb_d, c2_d gb_d)
//            from its slot (or the ring); export the consumers' values of virtual inflows to the
//            upstream blocks                                                          -- barrier --
//   compute: from the upstream slots x_j(t - 1): the inflow I(t) of this step and the upstream sum
//            Sx(t - 1) of the next one (Sx(t) was formed last tick); VJP of one step; own slot
//            <- (c1 gb, c2 gb)                                                         -- barrier --
// Every global load of a tick is issued one tick (own states: two ticks) before its use: the
// states x(t - 3) (the schedule layout, coalesced rows), the virtual inflows' x, and dL/drunoff read
// straight from the API's (N, T) layout in 16-B groups of four steps (gauge mode: summed over the
// reach's gauges from (G, T)).
// GS (state gradients, DDR_BWD_GRAD_*): the sweep also runs step 0 -- the hot start's transposed solve
// (c1 = 1) into dL/d(q' * flow_scale)[0], or dL/dQ0 of a carried state -- and writes dL/d(q' * flow_scale)
// of every step (gb c4 [q' >= q_lb], mmc.py:421-424, 535-538) into gqs, the schedule layout of qs.
// XB: the slot buffers when not the KR rule's (bwd_xbuf): 1 = single-buffered slots where the double buffer
// does not fit the LDS (fp64 at KR = 2, bwd_xb_of)
// PL (plain, as the forward's): no split basin, no profile, no state seeds, 16-B (N, T) rows; 1: dL/drunoff per
// reach, 2: gauge mode -- the tests of those options and the uniform values behind them leave the tick loop
template <typename R, int KR, bool GS, int XB = 0, bool DF = false, int PL = 0>
__global__ void __launch_bounds__(kBlockThreads, kBlocksPerCU * kBlockThreads / 256) route_backward_kernel(RouteArgs a) {
  constexpr int BS = kBlockThreads;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int bid = take_ticket(a.status, kStatusTicketBwd, a.nblocks, true, reinterpret_cast<int*>(smem));
  if (a.owned && !a.owned[bid]) return;  // split basin: another rank's block
  const BlockDesc B = block_desc(a.s.blocks, bid);
  const int tid = threadIdx.x;
  // first lane of this wave (scalar): waves with no reach in slice k skip it (scalar branch),
  // so a workgroup's tick costs ceil(nloc / 64) wave-slices, not KR * waves
  const int wbase = __builtin_amdgcn_readfirstlane(tid & ~63);
  const int S = a.slot_stride;
  // kDbl (KR <= 2): each slot array is [2][S] by tick parity -- a tick reads what its neighbours wrote the
  // tick before (the downstream's (c1 gb, c2 gb) in buffer (tb + 1) & 1, the upstream's x in buffer tb & 1)
  // and writes its own for the next tick into the other buffers: one workgroup barrier per tick.  Else
  // [S] each, a publish phase and a compute phase between two barriers.
  constexpr int kXB = XB > 0 ? XB : bwd_xbuf(KR);
  constexpr bool kDbl = kXB == 2 && KR <= kBwdEarlyMaxKR;
  R* sa = reinterpret_cast<R*>(smem + kMathTabBytes);  // [kXB][S] c1_i gb_i (transposed solve, rounded to R)
  R* sb = sa + kXB * S;                                 // [kXB][S] c2_i gb_i (adjoint of the inflow)
  R* sx = sb + kXB * S;                                 // [kXB][S] x(t - 2) of each reach / virtual inflow; [S-1] = 0
  const StatTab<R> tab{sx + kXB * S};                   // [S][6]
  R* ring = reinterpret_cast<R*>(smem + kMathTabBytes + align16(size_t(S) * (3 * kXB + 6) * sizeof(R)));  // [ncout][kChunkBwd][2]
  int* xl = reinterpret_cast<int*>(smem + a.xl_off);                                            // confluence lists
  const Consts<R> cs = consts_of<R>(a, true, KR >= kOpqInfMinKR);
  const int64_t T = a.T;
  const bool carry = a.flags & DDR_FWD_CARRY;
  const bool force_to = a.flags & kFlagForceTimeout;
  const R* xsave = static_cast<const R*>(a.x_save);
  const R* gout = static_cast<const R*>(a.grad_out);
  const int64_t xs_base = T * B.pos0 + B.pre_dn;
  double* gacc = a.bwd_bnd + 2 * a.n_cut * T;  // (N, 3) fp64 gradient accumulators (zeroed)
  const bool vec4 = PL || (T & 3) == 0;         // (N, T) rows 16-B aligned
  // (expressions at each use, not locals: the general instance then keeps the code and registers it had
  // before the plain ones existed -- locals held across the tick loop spill at KR = 4)
#define gauge (PL == 2 || (PL == 0 && a.g_roff != nullptr))  // dL/dout per gauge (G, T)
#define gseed (PL ? nullptr : a.gseed)                        // state seeds of steps T - 1, T - 2
#define aprof (PL ? nullptr : a.prof)
#define xt_off (PL ? 0 : a.xt_off)
  const int tmin = GS ? 0 : 1;                  // first step of the sweep (step 0: the hot start / Q0)
  R* gqs = static_cast<R*>(a.gqs);

  // od packs the tick offset (bits 16-30), dl (low 16, signed): local downstream (>= 0),
  // -(import slot + 2), or -1, and bit 31: the reach has no dL/drunoff row (gauge mode, ungauged
  // reach: its gradient loads, a dependent chain through the gauge map, are skipped)
  int ref[KR];
  unsigned od[KR];
  auto off_of = [&](int k) { return (int)((od[k] >> 16) & 0x7FFFu); };
  auto has_grad = [&](int k) { return (od[k] >> 31) == 0u; };
  auto dl_of = [&](int k) { return (int)(short)(od[k] & 0xFFFFu); };
  unsigned up[KR];
  // xc = x(t), xa = x(t-1), xb = x(t-2) (published this tick, then reloaded with x(t-3), while
  // x(t-2) stays readable in the reach's own slot); sxn = sum_j x_j(t) (upstream);
  // g0..g3: dL/drunoff of the four steps of t's group (t & ~3 .. t | 3)
  R lam[KR], xc[KR], xa[KR], xb[KR], pn[KR], pq[KR], pp[KR], g0[KR], g1[KR], g2[KR], g3[KR];
  // kDF (DDR_BWD_EXACT_ADJOINT, fp32 fast adjoint): the step's mass imbalances D1 = Q - qc - Sx, D2 = Q - qc - I
  // formed in fp64 from the fp32 states (physics.h adjoint_step_fast): the upstream sums carried in fp64, qc
  // re-read.  Else X (I - Sx) + (1 - X)(Q - x~) with x~ := x(t), the stored state
  constexpr bool kDF = DF && std::is_same<R, float>::value;
  using SxT = typename std::conditional<kDF, double, R>::type;
  SxT sxn[KR];
  // the gradient groups as shift registers (KR <= 2: c3s8 backward -4 %); at KR = 4 the select on t & 3 measured
  // faster (C5 backward 59.5 vs 57.3 ms, profiles/r05/ab_r05.txt)
  constexpr bool kShiftG = KR <= kBwdShiftMaxKR;
  // early loads: the next tick's x(t - 3) and virtual x are requested at the top
  // of the tick into a second register set (roles swap every tick: the loop is unrolled by two), so
  // they have the whole tick to land instead of the part after the first barrier
  R xb2[KR];
  constexpr bool kEarly = KR <= kBwdEarlyMaxKR;
  // gauge mode, KR <= 2: each reach's gauge when it has exactly one (else -1: none, or several -- the
  // reach -> gauge list is walked), so the tick's dL/dout loads are one address computation, not a chain of
  // three dependent loads each followed by a wait
  constexpr bool kGReg = KR <= 2;
  int gsg[kGReg ? KR : 1];
  constexpr bool kQs = GS || kDF;
  R qsv[kQs ? KR : 1];  // q' * flow_scale of this tick's step (prefetched a tick ahead): state gradients, kDF
  // one reach per thread: the derived statics stay in registers (see the forward)
  constexpr bool kStatReg = KR == 1 && sizeof(R) == 4;
  ReachStatic<R> sreg[kStatReg ? KR : 1];
#pragma unroll
  for (int k = 0; k < KR; ++k) {
    const int r = tid + k * BS;
    const bool hk = r < B.nloc;
    const int P = B.pos0 + (hk ? r : 0);
    ref[k] = a.s.ref[P];
    const bool nograd = gauge && a.g_roff[ref[k] + 1] == a.g_roff[ref[k]] && gseed == nullptr;
    if constexpr (kGReg) {
      gsg[k] = -1;
      if (gauge && a.g_roff[ref[k] + 1] - a.g_roff[ref[k]] == 1) gsg[k] = (int)a.g_rg[a.g_roff[ref[k]]];
    }
    od[k] = ((unsigned)a.s.off[P] << 16) | ((unsigned)a.s.dloc[P] & 0xFFFFu) | (nograd ? 0x80000000u : 0u);
    up[k] = pack_up(a, P, (unsigned)(S - 1));  // slot S-1 holds 0: missing upstreams add exactly 0
    lam[k] = R(0);
    sxn[k] = SxT(0);
    xc[k] = xa[k] = xb[k] = R(0);
    pn[k] = pq[k] = pp[k] = R(0);
    g0[k] = g1[k] = g2[k] = g3[k] = R(0);
    if (hk) tab.put(r, load_static<R>(a, ref[k]));
    if constexpr (kStatReg) {
      const ReachStatic<R> ls = load_static<R>(a, ref[k]);
      // the LDS path derives the same fields with the same operations each tick (StatTab::get)
      sreg[k] = derive_static<R, true>(ls.n, ls.qe, ls.p, ls.sqrtS, ls.L, ls.X);
    }
  }
  for (int c = 0; c < B.ncout; ++c) {
    const int loc = a.s.cout_loc[B.cout0 + c];
#pragma unroll
    for (int k = 0; k < KR; ++k)
      if (tid + k * BS == loc) od[k] = (od[k] & 0xFFFF0000u) | ((unsigned)(-(c + 2)) & 0xFFFFu);
  }
  if (tid == 0) sx[S - 1] = R(0);
  if (kDbl && tid == 0) sx[2 * S - 1] = R(0);
  const bool vown = tid < B.nvirt;
  // Import waves (KR = 1, blocks whose reaches, virtuals and chunk imports each fit half the workgroup):
  // the upper half's idle waves run the cut-out imports in a loop of their own, requesting each chunk's
  // granules kBwdImpEarly ticks before its boundary tick, so the routing waves' import phase shrinks
  // to the barrier that hands the ring over
  static_assert(kBwdImpEarly > 0 && kBwdImpEarly < kChunkBwd, "import lead within a chunk");
  const bool help_ok = KR == 1 && kDbl && !(a.flags & kFlagNoStorer) && B.nloc <= BS / 2 && B.nvirt <= BS / 2 &&
                       B.ncout * kChunkBwd <= BS / 2;
  const bool imp_mode = help_ok && B.ncout > 0;
  // x helpers (same blocks): the upper half also loads each reach's x(t - 4) row from x_save, kBwdHelpAhead
  // ticks ahead, and publishes it into the reach's slot, so the routing waves issue no x_save load and do
  // not wait at the tick's top for one
  const bool xhelp = help_ok;
  // gradient helpers (x-helper blocks, per-reach dL/drunoff, statics in registers): the same upper waves also
  // load each reach's dL/drunoff[:, t] kBwdHelpAhead ticks ahead and publish it into a parity-indexed LDS row
  // (the statics table's space, unused when the statics live in registers), so the routing waves issue no
  // global load and wait for none at the tick's top (a cold 16-B group load, one tick ahead, paced the light
  // backward: profiles/r05/ab_r05.txt item 12)
  const bool ghelp = kStatReg && kShiftG && xhelp && !(gauge);
  R* const sg = reinterpret_cast<R*>(sx + kXB * S);  // [2][S] (ghelp): dL/drunoff of each reach's step, by tick parity
  // virtual inflow owners (tid < nvirt): v_edge, v_off in registers; in LDS (own[tid], registers are
  // full) the virtual's consumer slot (low 16 bits) and the tick offset of cut-out `tid` (high 16 bits,
  // tid < ncout: its import owner)
  int v_edge = 0, v_off = 0;
  unsigned* own = reinterpret_cast<unsigned*>(smem + a.own_off);
  if (vown) {
    v_edge = a.s.v_edge[B.virt0 + tid];
    v_off = a.s.v_off[B.virt0 + tid];
  }
  if (tid < B.nvirt || tid < B.ncout)
    own[tid] = (vown ? (unsigned)a.s.v_dloc[B.virt0 + tid] & 0xFFFFu : 0u) |
               (tid < B.ncout ? (unsigned)a.s.off[B.pos0 + a.s.cout_loc[B.cout0 + tid]] << 16 : 0u);
  auto v_dloc_of = [&]() { return (int)(own[tid] & 0xFFFFu); };
  const int TT = (int)T + B.dmax;
  load_math_tables();
  load_xlist(a, B, xl);
  // split basin: [nvirt] the virtuals' export rows (to the producer block's rank), then [ncout] the
  // cut-outs' import rows (this rank's receive rows for edges from another rank's consumer)
  uintptr_t* xtv = reinterpret_cast<uintptr_t*>(smem + xt_off);
  uintptr_t* xtc = xtv + B.nvirt;
  if (xt_off) {
    for (int v = tid; v < B.nvirt; v += BS) {
      const int64_t e = a.s.v_edge[B.virt0 + v];
      const int xi = a.xid[e];
      xtv[v] = xi >= 0 ? (reinterpret_cast<uintptr_t>(a.pxbwd[a.xprod[xi]] + (int64_t)xi * T * 2) | 1u)
                       : reinterpret_cast<uintptr_t>(a.bwd_bnd + e * T * 2);
    }
    for (int c = tid; c < B.ncout; c += BS) {
      const int64_t e = B.cout0 + c;
      const int xi = a.xid[e];
      xtc[c] = xi >= 0 ? (reinterpret_cast<uintptr_t>(a.xbwd + (int64_t)xi * T * 2) | 1u)
                       : reinterpret_cast<uintptr_t>(a.bwd_bnd + e * T * 2);
    }
  }
  __syncthreads();
  unsigned long long prof_wait = 0;
  if (aprof && tid == 0) prof_begin(aprof, bid);
  PhaseProf phz;

  // x of this reach at forward tick `tau` (clamped into the block's rows)
  auto load_own = [&](int tau, R(&dst)[KR], int tq) {
    const int tc = tau < 0 ? 0 : (tau >= TT ? TT - 1 : tau);
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      if (wbase + k * BS >= B.nloc) continue;
      const int r = tq + k * BS;
      dst[k] = xsave[xs_base + (int64_t)tc * B.nloc + (r < B.nloc ? r : 0)];
    }
  };
  // x of a virtual inflow (the upstream reach of cut edge v_edge) at step t, from the forward's
  // boundary granules (t clamped into [0, T))
  // split basin: a virtual whose producer is another rank's block sends its x to this rank's receive rows;
  // split_finish_kernel copied them into this call's bnd after the forward
  const int vxi = (!PL && vown && a.xid) ? a.xid[v_edge] : -1;  // split basin: the virtual's cross-rank row
  auto load_virt = [&](int64_t t) -> double {
    const int64_t tc = t < 0 ? 0 : (t >= T ? T - 1 : t);
    return a.bnd[(int64_t)v_edge * T + tc];
  };
  // dL/drunoff of steps base .. base + 3 of reach slice k (mmc.py:380-412: runoff[ref, t] = Q_t; in
  // gauge mode every gauge sums its reaches' Q_t, mmc.py:405-411, 433-439).  `base` is 4-aligned except
  // for a reach's first group (un: base = T - 4, any alignment; steps outside [0, T) read clamped rows and
  // are never consumed)
  auto load_grad_out = [&](int ref, int64_t base, int gs, bool un) {
    R v0 = R(0), v1 = R(0), v2 = R(0), v3 = R(0);
    const bool v4 = vec4 && !(un && (base & 3) != 0);
    // !un (steady ticks): the group's steps lie in [1, T - 2], so the clamps (int64 compares and selects the
    // compiler hoists above the vec4 branch, run by the whole wave every tick) are dropped -- at KR = 4 (at
    // KR = 1 the light C5-shaped backward measured 6 % slower without them, r05_nc0)
    auto cl = [&](int64_t i) {
      return (!un && KR >= 4) ? i : (i < 0 ? int64_t(0) : (i < T ? i : T - 1));
    };
    const int64_t i0 = cl(base), i1 = cl(base + 1), i2 = cl(base + 2), i3 = cl(base + 3);
    // m0: the gauge's t = 0 sum passed its clamp (state gradients only; mmc.py:398-412)
    auto add_row = [&](const R* row, bool m0) {
      if (v4) {
        if constexpr (sizeof(R) == 4) {
          const float4 v = load_grad4(row + base);
          v0 = v0 + ((m0 || base != 0) ? v.x : 0.0f); v1 = v1 + v.y; v2 = v2 + v.z; v3 = v3 + v.w;
        } else {
          const double2 u = reinterpret_cast<const double2*>(row + base)[0];
          const double2 w = reinterpret_cast<const double2*>(row + base)[1];
          v0 = v0 + ((m0 || base != 0) ? u.x : 0.0); v1 = v1 + u.y; v2 = v2 + w.x; v3 = v3 + w.y;
        }
      } else {
        v0 = v0 + ((m0 || base != 0) ? row[i0] : R(0));
        v1 = v1 + ((m0 || base != -1) ? row[i1] : R(0));
        v2 = v2 + ((m0 || base != -2) ? row[i2] : R(0));
        v3 = v3 + ((m0 || base != -3) ? row[i3] : R(0));
      }
    };
    // a row's four values as loaded: no arithmetic on them in this tick, so the wave does not wait for the load
    // (it lands by the next tick's top; adding them to 0 would consume it now -- a full memory round trip)
    auto raw_row = [&](const R* row) {
      if (v4) {
        if constexpr (sizeof(R) == 4) {
          const float4 v = load_grad4(row + base);
          return make_grad4(v.x, v.y, v.z, v.w);
        } else {
          const double2 u = reinterpret_cast<const double2*>(row + base)[0];
          const double2 w = reinterpret_cast<const double2*>(row + base)[1];
          return make_grad4(u.x, u.y, w.x, w.y);
        }
      }
      return make_grad4(row[i0], row[i1], row[i2], row[i3]);
    };
    if (gauge) {
      const bool z = GS && a.gmask0 && base <= 0;  // the group holds step 0
      if (gs >= 0) {
        // the reach's only gauge (kGReg): the row address needs no dependent index loads in the tick
        // (its values as loaded instead of added to 0, so that this tick does not wait for them: no change
        // at c3s8, r05_gr)
        add_row(gout + (int64_t)gs * T, !(z && a.gmask0[gs] == 0));
        return make_grad4(v0, v1, v2, v3);
      }
      const int64_t q1 = a.g_roff[ref + 1];
      for (int64_t q = a.g_roff[ref]; q < q1; ++q) {
        const int64_t gi = a.g_rg[q];
        add_row(gout + gi * T, !(z && a.gmask0[gi] == 0));
      }
      return make_grad4(v0, v1, v2, v3);
    }
    // one reach row: the loaded values as they are
    return raw_row(gout + (int64_t)ref * T);
  };
  // ... plus the state seeds of steps T - 1 and T - 2 (a.gseed).  Only outside the steady ticks (seeded: the
  // steady range then starts late enough that no steady tick loads the groups of those steps), so the steady
  // loop's code and registers are those of an unseeded launch
  auto load_grad = [&](int ref, int64_t base, int gs, bool seeded) {
    Grad4<R> v = load_grad_out(ref, base, gs, seeded);
    if (seeded && gseed != nullptr && base + 3 >= T - 2) {
      const R* sd = static_cast<const R*>(gseed);
      const R s1 = sd[ref], s2 = sd[a.N + ref];
      auto add = [&](R& g, int64_t t) { g = g + (t == T - 1 ? s1 : (t == T - 2 ? s2 : R(0))); };
      add(v.a, base);
      add(v.b, base + 1);
      add(v.c, base + 2);
      add(v.d, base + 3);
    }
    return v;
  };

  // (ghelp) the value helper w publishes at backward tick tb, read by its reach at tick tb + 1: dL/drunoff of the
  // step t = TT - 2 - tb - off (0 outside [0, T)), plus the state seeds of steps T - 1 and T - 2
  // (rf, off: reach w's reference index and tick offset, loaded once)
  auto ghelp_load = [&](int rf, int off, int tb) -> R {
    const int64_t t = (int64_t)TT - 2 - tb - off;
    if (t < 0 || t >= T) return R(0);
    R v = gout[(int64_t)rf * T + t];
    if (gseed != nullptr && t >= T - 2) v = v + static_cast<const R*>(gseed)[(t == T - 1 ? 0 : a.N) + rf];
    return v;
  };

  // virtual inflow's x(t_v - 2), prefetched one tick ahead (kept as loaded: converting it would
  // wait for the load in the tick that issues it)
  double vx = 0.0, vx2 = 0.0;

  // xbc / vxc: loaded last tick, published now; xbn / vxn: loaded now for the next tick (the same
  // registers without early loads)
  // sc: std::integral_constant<bool, kSt>.  Steady ticks (forward tick tau in [dmax + 2, T - 1]) are
  // those at which every reach runs a step t in [2, T - 1]: no activity tests, no t = 1 carried-state
  // case, no step-0 sweep, the next step's gradient group always in range
  auto tick = [&](int tb, R(&xbc)[KR], R(&xbn)[KR], double& vxc, double& vxn, auto sc) {
    constexpr bool kSt = decltype(sc)::value;
    const int tau = TT - 1 - tb;  // forward tick
    // Every global load of the previous tick (states, virtual inflows, gradient groups) lands
    // here, a whole tick after its issue.  An explicit wait the compiler can see: without it, its
    // conservative count across the divergent load branches waits (vmcnt(0)) at the first use of a
    // previous-tick register, i.e. for the loads issued in THIS tick too.
    __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
    if constexpr (KR == 4) set_prio(3);
    phz.mark(0);  // the previous tick's loads and stores
    const int tq = opq(tid);
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      ref[k] = opq(ref[k]);
      od[k] = opq(od[k]);
      up[k] = opq(up[k]);
    }
    // kDbl: this tick publishes (into the next tick's x buffer) the values loaded last tick, and loads
    // those it publishes next tick -- one tick further ahead than without double buffering
    const R* sar = sa + (kDbl ? ((tb + 1) & 1) * S : 0);  // the downstream's values of the previous tick
    const R* sbr = sb + (kDbl ? ((tb + 1) & 1) * S : 0);
    R* saw = sa + (kDbl ? (tb & 1) * S : 0);              // this tick's (c1 gb, c2 gb)
    R* sbw = sb + (kDbl ? (tb & 1) * S : 0);
    const R* sxr = sx + (kDbl ? (tb & 1) * S : 0);        // x published for this tick
    R* sxw = sx + (kDbl ? ((tb + 1) & 1) * S : 0);        // (kDbl) x published for the next tick
    if constexpr (kEarly) {
      constexpr int ahead = kDbl ? 1 : 0;
      if (!xhelp) load_own(tau - 3 - ahead, xbn, tq);              // x(t - 3) (kDbl: x(t - 4)), published next tick
      if (vown) vxn = load_virt((int64_t)tau - 1 - ahead - v_off - 2);  // the virtual's value for the next tick
    }
    if (B.ncout > 0 && (tb % kChunkBwd) == 0) {
      // one (cut-out, step) per thread and iteration, its (A, B) granule pair requested together; the
      // cut edge of cut-out c is B.cout0 + c (graph.cpp numbers cut edges in block order), its tick
      // offset is in the owner words
      const unsigned long long w0 = aprof ? __builtin_amdgcn_s_memrealtime() : 0;
      for (int w = tid; !imp_mode && w < B.ncout * kChunkBwd; w += BS) {
        const int c = w / kChunkBwd, sidx = w % kChunkBwd;
        const int t = (tau - sidx) - (int)(own[c] >> 16);
        R A = R(0), Bv = R(0);
        if (t >= tmin && t < T) {
          double g[2];
          const uintptr_t p = xt_off ? xtc[c] : reinterpret_cast<uintptr_t>(a.bwd_bnd + (int64_t)(B.cout0 + c) * T * 2);
          const double* row = reinterpret_cast<const double*>(p & ~uintptr_t(1)) + (int64_t)t * 2;
          if (p & 1u) wait_granules<2, true>(row, 0, 1, 0, 2, g, a.status, bid, force_to);  // another rank's consumer
          else wait_granules<2>(row, 0, 1, 0, 2, g, a.status, bid, force_to);
          A = R(g[0]);
          Bv = R(g[1]);
        }
        ring[(c * kChunkBwd + sidx) * 2] = A;
        ring[(c * kChunkBwd + sidx) * 2 + 1] = Bv;
      }
      lds_barrier();
      if (aprof) prof_wait += __builtin_amdgcn_s_memrealtime() - w0;
    }
    phz.mark(1);  // import
    // ---- read / publish ----------------------------------------------------------------------
    if (vown) {
      // export the consumer's (c1 gb, c2 gb) of step t (written last tick, when the consumer ran
      // step tau + 1 - off_c = tau - v_off) to the upstream block; publish the upstream reach's x
      // at the consumer's current step - 1 (kDbl: next step's, into the next tick's buffer)
      const int t = tau - v_off;
      if (t >= tmin && t < T) {
        const int dloc = v_dloc_of();
        if (vxi >= 0) {  // split basin: the producer block is another rank's (row from the block's table)
          double* dst = reinterpret_cast<double*>(xtv[tid] & ~uintptr_t(1)) + (int64_t)t * 2;
          store_granule_sys(dst, (double)sar[dloc]);
          store_granule_sys(dst + 1, (double)sbr[dloc]);
        } else {
          store_granule(a.bwd_bnd + ((int64_t)v_edge * T + t) * 2, (double)sar[dloc]);
          store_granule(a.bwd_bnd + ((int64_t)v_edge * T + t) * 2 + 1, (double)sbr[dloc]);
        }
      }
      sxw[B.nloc + tid] = R(vxc);
    }
    R A[KR], Bd[KR];
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      A[k] = R(0);
      Bd[k] = R(0);
      if (wbase + k * BS >= B.nloc) continue;
      const int r = tq + k * BS;
      // x(t - 2): the upstream value of the downstream reach's step t - 1 (kDbl: next tick's, x(t - 3))
      if (!xhelp && r < B.nloc) sxw[r] = xbc[k];
      const int dl = dl_of(k);
      if (dl >= 0) {
        A[k] = sar[dl];
        Bd[k] = sbr[dl];
      } else if (dl <= -2) {
        const int sidx = tb % kChunkBwd;
        A[k] = ring[((-dl - 2) * kChunkBwd + sidx) * 2];
        Bd[k] = ring[((-dl - 2) * kChunkBwd + sidx) * 2 + 1];
      }
    }
    phz.mark(2);  // read / publish
    if constexpr (!kDbl) lds_barrier();
    phz.mark(3);  // barrier 1
    if constexpr (!kEarly) {
      load_own(tau - 3, xbn, tq);                    // x(t - 3), published next tick
      if (vown) vxn = load_virt((int64_t)tau - 1 - v_off - 2);  // the virtual's value for the next tick
    }
    // ---- compute ------------------------------------------------------------------------------
    // per slice: the step's inputs (pre), its adjoint, its outputs (post) and the next loads (tail)
    struct Pre {
      int r, rs, t;
      bool hk, active, c0;
      R Sx, I, gk, xtk, lm, gb, Qp, D1, D2;
      double gb64;
      ReachStatic<R> st;
    };
    auto pre = [&](int k, Pre& P) {
      P.r = tq + k * BS;
      P.hk = P.r < B.nloc;
      P.rs = P.hk ? P.r : 0;
      P.t = tau - off_of(k);
      P.active = P.hk && (kSt || (P.t >= 1 && P.t < T));
      // upstream x_j(t - 1): I(t) = sum_j Q_j(t - 1) (mmc.py:535, ascending columns; the carried
      // state at t - 1 = 0 is not clamped) and Sx(t - 1) for the next tick
      P.c0 = !kSt && (P.t == 1 && carry);
      const bool c0 = P.c0;
      const int nup = up_n(up[k]);
      const R x0 = sxr[up_0(up[k])];
      const R x1 = sxr[up_1(up[k], xl)];
      SxT sxv = SxT(0) + SxT(x0);
      sxv = sxv + SxT(x1);
      SxT I = SxT(0);
      I = I + SxT(nup > 0 ? (c0 ? x0 : rmaxc(x0, cs.qlb, cs)) : R(0));
      I = I + SxT(nup > 1 ? (c0 ? x1 : rmaxc(x1, cs.qlb, cs)) : R(0));
      if (nup > 2) {
        const int* lst = xl + up_f1(up[k]);
        const int c = lst[0];
        for (int j = 2; j < c; ++j) {
          const R xj = sxr[lst[j]];
          sxv = sxv + SxT(xj);
          I = I + SxT(c0 ? xj : rmaxc(xj, cs.qlb, cs));
        }
      }
      const SxT Sx = sxn[k];  // sum_j x_j(t), the solve's upstream term of this step
      P.I = R(I);
      P.Sx = R(Sx);
      sxn[k] = sxv;
      if constexpr (kShiftG) {
        // dL/drunoff[:, t]: the group's registers shift by one step per tick (g3 holds step t: a group is loaded
        // the tick before its top step runs) -- no per-lane select on t & 3
        P.gk = g3[k];
        g3[k] = g2[k];
        g2[k] = g1[k];
        g1[k] = g0[k];
        if (kStatReg && ghelp) P.gk = sg[(tb & 1) * S + P.rs];  // published by the gradient helpers last tick
      } else {
        const int e4 = P.t & 3;
        // dL/drunoff[:, t] by two bit tests and three selects (a ternary chain on e4 compiles into divergent
        // branches)
        const bool b0 = (e4 & 1) != 0, b1 = (e4 & 2) != 0;
        const R lo = b0 ? g1[k] : g0[k], hi = b0 ? g3[k] : g2[k];
        P.gk = b1 ? hi : lo;
      }
      P.xtk = xc[k];
      P.st = kStatReg ? sreg[k] : tab.template get<true>(P.rs);
      P.lm = lam[k] + P.gk;                                 // dL/dQ_t (+ dL/dout[:, t])
      const R gx = (P.xtk >= cs.qlb) ? P.lm : R(0);         // clamp backward (inclusive)
      P.gb64 = (double)gx + (double)A[k];                   // (I - C1 N)^T gb = gx (utils.py:188-242)
      P.gb = R(P.gb64);
      P.Qp = c0 ? xa[k] : rmaxc(xa[k], cs.qlb, cs);              // Q_{t-1}
      if constexpr (kDF) {
        const SxT Qq = (SxT)P.Qp - (SxT)rmaxc(qsv[kQs ? k : 0], cs.qlb, cs);  // exact in fp64
        P.D1 = R(Qq - Sx);
        P.D2 = R(Qq - I);
      }
    };
    auto adjoint = [&](int k, const Pre& P, AdjOutR<R>& o) {
      if constexpr (std::is_same<R, float>::value) {
        AdjOut f;
        if constexpr (kDF) f = adjoint_step_fast<true>(P.st, P.Qp, cs, P.gb, P.D1, P.D2, R(0));
        else f = adjoint_step_fast<false>(P.st, P.Qp, cs, P.gb, P.xtk, P.Sx, P.I);
        o = AdjOutR<R>{f.c1, f.c2, f.c3, f.c4, f.gQ, f.gn, f.gq, f.gp};
      } else {
        const R qvk = *qs_at<R>(a, B, xs_base, tau, off_of(k), P.rs);  // q'[t-1] * flow_scale
        R tw, ss;
        Geom<R> geo;
        coefficients<R, true>(P.st, P.Qp, cs, o.c1, o.c2, o.c3, o.c4, tw, ss, &geo);
        const R qc = rmaxc(qvk, cs.qlb, cs);
        const R gc1 = P.gb * P.Sx, gc2 = P.gb * P.I, gc3 = P.gb * P.Qp, gc4 = P.gb * qc;
        coefficients_vjp<R, true>(P.st, P.Qp, cs, geo, o.c1, o.c2, o.c3, o.c4, gc1, gc2, gc3, gc4, o.gQ, o.gn,
                                            o.gq, o.gp);
      }
    };
    auto post = [&](int k, const Pre& P, const AdjOutR<R>& o) {
      const int r = P.r, t = P.t;
      const R gb = P.gb;
      if (P.active) {
        pn[k] = pn[k] + o.gn;
        pq[k] = pq[k] + o.gq;
        pp[k] = pp[k] + o.gp;
        // flush the fp32 partial sums into the fp64 accumulators every kGradFlush *steps* (aligned to
        // t, not to ticks, so the summation grouping -- and the result -- is independent of the
        // partition); one owner per address, so the atomics are deterministic
        if ((t % kGradFlush) == 1 || (!kSt && t == 1)) {
          double* g3p = gacc + (int64_t)ref[k] * 3;
          atomicAdd(g3p + 0, (double)pn[k]);
          atomicAdd(g3p + 1, (double)pq[k]);
          atomicAdd(g3p + 2, (double)pp[k]);
          pn[k] = pq[k] = pp[k] = R(0);
        }
        saw[r] = R((double)o.c1 * P.gb64);
        sbw[r] = o.c2 * gb;
        lam[k] = ((gb * o.c3) + o.gQ) + Bd[k];
        // dL/dqc = gb c4 (b = ... + c4 qc), through qc = clamp(q' * flow_scale) (mmc.py:421-424)
        if constexpr (GS) gqs[xs_base + (int64_t)tau * B.nloc + r] = (qsv[k] >= cs.qlb) ? gb * o.c4 : R(0);
      } else if (!kSt && GS && P.hk && t == 0) {
        if (carry) {
          // Q0 = q0 feeds step 1 unclamped; runoff[:, 0] = clamp(q0) per reach, or the gauge sum's clamp
          // (already folded into gk through gmask0)
          if (a.gq0) static_cast<R*>(a.gq0)[ref[k]] = gauge ? P.lm : lam[k] + ((P.xtk >= cs.qlb) ? P.gk : R(0));
          gqs[xs_base + (int64_t)tau * B.nloc + r] = R(0);
          saw[r] = R(0);
          sbw[r] = R(0);
        } else {
          // hot start x(0) = (I - N)^-1 q'[0] (mmc.py:25-66): its transposed solve (c1 = 1) is gb64
          gqs[xs_base + (int64_t)tau * B.nloc + r] = gb;
          saw[r] = gb;
          sbw[r] = R(0);
        }
      }
    };
    auto tail = [&](int k, const Pre& P) {
      if constexpr (kQs) {
        const int tn = tau > 0 ? tau - 1 : 0;  // the next backward tick's row
        qsv[k] = *qs_at<R>(a, B, xs_base, tn, off_of(k), P.rs);
      }
      // dL/drunoff of the next step's group, one tick ahead
      const int tn = P.t - 1;
      if (!ghelp && P.hk && has_grad(k) && (kSt ? (tn & 3) == 3 : (tn >= 0 && tn < T && ((tn & 3) == 3 || tn == T - 1)))) {
        const Grad4<R> v = load_grad(ref[k], kShiftG ? (int64_t)tn - 3 : (int64_t)(tn & ~3),
                                     kGReg ? opq(gsg[kGReg ? k : 0]) : -1, !kSt);
        g0[k] = v.a; g1[k] = v.b; g2[k] = v.c; g3[k] = v.d;
      }
    };
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      if (wbase + k * BS >= B.nloc) continue;
      if constexpr (KR == 4) set_prio(KR - 1 - k);
      Pre P;
      pre(k, P);
      AdjOutR<R> o;
      adjoint(k, P, o);
      post(k, P, o);
      tail(k, P);
      __builtin_amdgcn_sched_barrier(0);
    }
    phz.mark(4);  // loads issue + compute
    // next tick: x(t - 1) -> x(t); x(t - 2), still in the own slot -> x(t - 1).  kDbl: read before the
    // barrier (no one writes this tick's read buffer during the tick; after the barrier the x helpers
    // may already be writing it for the next tick)
    auto shift_x = [&]() {
#pragma unroll
      for (int k = 0; k < KR; ++k) {
        if (wbase + k * BS >= B.nloc) continue;
        const int r = tq + k * BS;
        xc[k] = xa[k];
        xa[k] = r < B.nloc ? sxr[r] : R(0);
      }
    };
    if constexpr (kDbl) shift_x();
    lds_barrier();
    phz.mark(5);  // barrier 2
    if constexpr (!kDbl) shift_x();
  };

  // tick 0 runs forward tick TT-1: x(t) at row TT-1, x(t-1) at row TT-2, x(t-2) at row TT-3
  if constexpr (kQs) {
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const int r = tid + k * BS;
      qsv[k] = *qs_at<R>(a, B, xs_base, TT - 1, off_of(k), r < B.nloc ? r : 0);
    }
  }
  load_own(TT - 1, xc, tid);
  load_own(TT - 2, xa, tid);
  load_own(TT - 3, xb, tid);
  // prologue: Sx of every reach's first step t0 = sum_j x_j(t0), where x_j(t0) is the upstream
  // reach's x one step before its own first step (its xa; a virtual inflow's granule) -- (kDbl) in buffer
  // 1, which tick 0 then overwrites
  R* sxp = sx + (kDbl ? S : 0);
#pragma unroll
  for (int k = 0; k < KR; ++k)
    if (tid + k * BS < B.nloc) sxp[tid + k * BS] = xa[k];
  if (vown) sxp[B.nloc + tid] = R(load_virt((int64_t)(TT - 1) - v_off - 1));
  __syncthreads();
#pragma unroll
  for (int k = 0; k < KR; ++k) {
    const int r = tid + k * BS;
    if (r >= B.nloc) continue;
    SxT v = SxT(0) + SxT(sxp[up_0(up[k])]);
    v = v + SxT(sxp[up_1(up[k], xl)]);
    if (up_n(up[k]) > 2) {
      const int* lst = xl + up_f1(up[k]);
      for (int j = 2; j < lst[0]; ++j) v = v + SxT(sxp[lst[j]]);
    }
    sxn[k] = v;
  }
  __syncthreads();
  if (vown) vx = load_virt((int64_t)(TT - 1) - v_off - 2);
  if constexpr (kDbl) {
    // tick 0's published values (x(t0 - 2), the virtuals') go into its read buffer now; the registers
    // then hold what tick 0 publishes for tick 1
#pragma unroll
    for (int k = 0; k < KR; ++k)
      if (tid + k * BS < B.nloc) sx[tid + k * BS] = xb[k];
    if (vown) sx[B.nloc + tid] = R(vx);
    load_own(TT - 4, xb, tid);
    if (vown) vx = load_virt((int64_t)(TT - 2) - v_off - 2);
    // (ghelp) tick 0's dL/drunoff row, written by the helper thread of each reach
    if (ghelp && tid >= BS / 2 && tid - BS / 2 < B.nloc) {
      const int P = B.pos0 + tid - BS / 2;
      sg[tid - BS / 2] = ghelp_load(a.s.ref[P], a.s.off[P], -1);
    }
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < KR; ++k)
    if (!ghelp && tid + k * BS < B.nloc && has_grad(k) && TT - 1 - off_of(k) == T - 1) {
      const Grad4<R> v = load_grad(ref[k], kShiftG ? T - 4 : (T - 1) & ~int64_t(3), kGReg ? gsg[kGReg ? k : 0] : -1, true);
      g0[k] = v.a; g1[k] = v.b; g2[k] = v.c; g3[k] = v.d;
    }
  if ((imp_mode || xhelp) && wbase >= BS / 2) {
    // import waves: thread w owns (cut-out w / kChunkBwd, step slot w % kChunkBwd) of every chunk; per tick
    // the same barriers as the routing waves' tick (the ring hand-off at a chunk boundary, the tick's end).
    // x helpers: thread w < nloc publishes reach w's x(t - 4) (forward row TT - 4 - tb at tick tb, clamped)
    // into the next tick's x buffer, its loads issued kBwdHelpAhead ticks ahead
    const int w = tid - BS / 2;
    const bool wown = imp_mode && w < B.ncout * kChunkBwd;
    const bool xown = xhelp && w < B.nloc;
    constexpr int XD = kBwdHelpAhead;
    const R* xcol = xsave + xs_base + (xown ? w : 0);
    auto xload = [&](int tb) -> R {
      int tc = TT - 4 - tb;
      tc = tc < 0 ? 0 : (tc >= TT ? TT - 1 : tc);
      return xown ? xcol[(int64_t)tc * B.nloc] : R(0);
    };
    R xp[XD], gp[XD];
    const bool gown = ghelp && w < B.nloc;
    const int grf = gown ? a.s.ref[B.pos0 + w] : 0, goff = gown ? a.s.off[B.pos0 + w] : 0;
#pragma unroll
    for (int i = 0; i < XD; ++i) {
      xp[i] = xload(i);
      gp[i] = gown ? ghelp_load(grf, goff, i) : R(0);
    }
    const int c = wown ? w / kChunkBwd : 0, sidx = w % kChunkBwd;
    const uintptr_t p = !wown ? 0 : xt_off ? xtc[c] : reinterpret_cast<uintptr_t>(a.bwd_bnd + (int64_t)(B.cout0 + c) * T * 2);
    const bool sys = p & 1u;
    const double* prow = reinterpret_cast<const double*>(p & ~uintptr_t(1));
    const int coff = wown ? (int)(own[c] >> 16) : 0;
    auto step_of = [&](int tb) { return (TT - 1 - tb - sidx) - coff; };  // the step chunk tb's slot needs
    unsigned long long eg[2] = {0ull, 0ull};
    bool issued = false;
    auto htick = [&](int tb, R& xr, R& gr) {
      if (B.ncout > 0 && (tb % kChunkBwd) == 0) {
        if (wown) {
          const int t = step_of(tb);
          R A = R(0), Bv = R(0);
          if (t >= tmin && t < T) {
            double g[2];
            const double* row = prow + (int64_t)t * 2;
            if (issued) {
              if (sys) poll_granules<2, true>(row, 0, 0, 2, eg, g, a.status, bid, force_to);
              else poll_granules<2, false>(row, 0, 0, 2, eg, g, a.status, bid, force_to);
            } else {
              if (sys) wait_granules<2, true>(row, 0, 1, 0, 2, g, a.status, bid, force_to);
              else wait_granules<2>(row, 0, 1, 0, 2, g, a.status, bid, force_to);
            }
            A = R(g[0]);
            Bv = R(g[1]);
          }
          ring[(c * kChunkBwd + sidx) * 2] = A;
          ring[(c * kChunkBwd + sidx) * 2 + 1] = Bv;
        }
        issued = false;
        lds_barrier();
      }
      if (xown) {
        sx[((tb + 1) & 1) * S + w] = xr;  // the routing waves read it next tick
        xr = xload(tb + XD);
      }
      if (gown) {
        sg[((tb + 1) & 1) * S + w] = gr;
        gr = ghelp_load(grf, goff, tb + XD);
      }
      const int nb = tb + kBwdImpEarly;
      if (wown && (nb % kChunkBwd) == 0 && nb < TT) {
        const int t = step_of(nb);
        if (t >= tmin && t < T) {
          const double* row = prow + (int64_t)t * 2;
          if (sys) issue_granules<2, true>(row, 0, 0, 2, eg);
          else issue_granules<2, false>(row, 0, 0, 2, eg);
          issued = true;
        }
      }
      lds_barrier();  // the routing waves' tick end
    };
    // unrolled by XD: each prefetch register is consumed in place (a register copy would wait for its load)
#pragma unroll 1
    for (int tb = 0; tb < TT; tb += XD) {
#pragma unroll
      for (int i = 0; i < XD; ++i)
        if (tb + i < TT) htick(tb + i, xp[i], gp[i]);
    }
    return;
  }
  phz.start();
  using Gen = std::integral_constant<bool, false>;
  using Steady = std::integral_constant<bool, true>;
  // steady backward ticks [b0, b1): forward ticks tau = TT - 1 - tb in [dmax + 2, T - 1]
  // (state seeds: from forward tick T - 2 down, so that every load of the groups of steps T - 2 and T - 1 --
  // issued at forward ticks >= T - 1 -- runs in a general tick)
  int b0 = gseed != nullptr ? B.dmax + 1 : B.dmax, b1 = (int)T - 2;
  if (kEarly) {  // even bounds: the register roles keep alternating
    b0 += b0 & 1;
    b1 &= ~1;
  }
  if ((a.flags & kFlagNoSteady) || b1 <= b0) b0 = b1 = 0;
  if constexpr (kEarly) {
#pragma unroll 1
    for (int tb = 0; tb < b0; tb += 2) {
      if (aprof && tid == 0) prof_tick(aprof, bid, tb);
      tick(tb, xb, xb2, vx, vx2, Gen{});
      tick(tb + 1, xb2, xb, vx2, vx, Gen{});
    }
#pragma unroll 1
    for (int tb = b0; tb < b1; tb += 2) {
      if (aprof && tid == 0) prof_tick(aprof, bid, tb);
      tick(tb, xb, xb2, vx, vx2, Steady{});
      tick(tb + 1, xb2, xb, vx2, vx, Steady{});
    }
#pragma unroll 1
    for (int tb = b1; tb < TT; tb += 2) {
      if (aprof && tid == 0) prof_tick(aprof, bid, tb);
      tick(tb, xb, xb2, vx, vx2, Gen{});
      if (tb + 1 < TT) tick(tb + 1, xb2, xb, vx2, vx, Gen{});
    }
  } else {
#pragma unroll 1
    for (int tb = 0; tb < b0; ++tb) {
      if (aprof && tid == 0) prof_tick(aprof, bid, tb);
      tick(tb, xb, xb, vx, vx, Gen{});
    }
#pragma unroll 1
    for (int tb = b0; tb < b1; ++tb) {
      if (aprof && tid == 0) prof_tick(aprof, bid, tb);
      tick(tb, xb, xb, vx, vx, Steady{});
    }
#pragma unroll 1
    for (int tb = b1; tb < TT; ++tb) {
      if (aprof && tid == 0) prof_tick(aprof, bid, tb);
      tick(tb, xb, xb, vx, vx, Gen{});
    }
  }
  if (aprof && tid == 0) prof_end(aprof, bid, prof_wait);
  phz.flush(aprof, a.nblocks, bid);
#undef gauge
#undef gseed
#undef aprof
#undef xt_off
}

// Final fp64 accumulators -> R gradients (reference order).
template <typename R>
__global__ void finish_grads_kernel(int64_t N, const double* gacc, R* gn, R* gq, R* gp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  gn[i] = R(gacc[3 * i + 0]);
  gq[i] = R(gacc[3 * i + 1]);
  gp[i] = R(gacc[3 * i + 2]);
}

// ============================================================================================
// Lateral inflow into the schedule layout of x_save (per workgroup, tick-major: row tau = t + off(r)
// holds its nloc reaches contiguously).  Each thread issues all its loads before the first is
// consumed (memory-level parallelism).
// ============================================================================================

// q'[max(t-1, 0), ref] * flow_scale[ref] -> qs[tick(t, r)] (mmc.py:303-304, 421-424): the routing
// kernels then read one contiguous row per tick instead of scattered 4-byte values of q' rows.
// One workgroup per (block, tile of gather_steps steps): reads walk the block's reaches in
// ascending reference order (runs of adjacent q' columns), writes walk positions (sorted by tick
// offset, so runs of one offset are contiguous in a tick row); the tile is staged in LDS.
// DDR_FWD_CHECK_QPRIME: the reference asserts that the flow-scaled q' holds no NaN before routing
// (mmc.py:335, `assert ~torch.any(torch.isnan(self.q_prime))`); the gathers see every value the window
// reads, so they set status word kStatusNaN instead of a separate pass over q' (28 GB at C5)
__device__ __forceinline__ void flag_nan(const RouteArgs& a, bool nan) {
  if (!(a.flags & DDR_FWD_CHECK_QPRIME)) return;
  if (__builtin_amdgcn_ballot_w64(nan) != 0 && (threadIdx.x & 63) == 0) atomicOr(a.status + kStatusNaN, 1u);
}
// ... and the one row no routing step reads: q' of the window's last hour (its row (T - 1) / qp_hours)
template <typename R>
__global__ void nan_last_row_kernel(RouteArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool nan = false;
  if (i < a.N) {
    const int64_t row = (a.T - 1) / (a.qp_hours > 0 ? a.qp_hours : 1);
    R v = static_cast<const R*>(a.qprime)[row * a.N + i];
    if (a.qp_valid && !a.qp_valid[i]) v = R(0.001f);
    if (a.fs) v = v * static_cast<const R*>(a.fs)[i];
    nan = v != v;
  }
  flag_nan(a, nan);
}

// One workgroup per (block, chunk of `chunk` steps, a multiple of G), G steps per LDS tile: each thread keeps
// its reaches' reference indices, LDS destinations, tick offsets and scale in registers for the whole chunk
// (a workgroup per tile re-read them: 12 B per reach per tile, a third of the q' bytes at G = 8), and the
// next tile's q' loads are in flight while the current tile leaves LDS for the schedule rows.  A chunk's
// tiles run on one CU back to back, so a tick row's segments written by consecutive tiles meet in its L2.
template <typename R, int G, int BS, int KG>
__global__ void __launch_bounds__(BS) gather_qprime_kernel(RouteArgs a, int chunk, int nchunks) {
  extern __shared__ __attribute__((aligned(16))) unsigned char gsm[];
  R* tile = reinterpret_cast<R*>(gsm);  // [G][nloc]
  // one-dimensional grid, chunk-major: the dispatcher starts every block's first chunk before any second one
  // (mapping a contiguous eighth of this list to each XCD, so that blocks sharing q' lines read them through one
  // L2, measured 2.7 % slower: profiles/r06/ab_r06.txt)
  const int nbk = (int)(gridDim.x / (unsigned)nchunks);
  const int bk = (int)(blockIdx.x % (unsigned)nbk);
  if (a.owned && !a.owned[bk]) return;  // split basin: another rank's block
  const BlockDesc B = a.s.blocks[bk];
  const int64_t T = a.T, N = a.N;
  const int64_t tA = (int64_t)(blockIdx.x / (unsigned)nbk) * chunk;
  if (tA >= T) return;
  const int64_t tB = tA + chunk < T ? tA + chunk : T;
  const int nl = B.nloc;
  const int tid = threadIdx.x;
  const R* qp = static_cast<const R*>(a.qprime);
  const R* fs = static_cast<const R*>(a.fs);
  const unsigned char* valid = a.qp_valid;
  // read side (ascending reference order: runs of adjacent q' columns) and write side (positions, sorted by
  // tick offset: runs of one offset are contiguous in a tick row)
  int ref[KG], loc[KG];
  int64_t off[KG];
  R sc[KG];
  bool fill[KG];
#pragma unroll
  for (int k = 0; k < KG; ++k) {
    const int i = tid + k * BS;
    const bool h = i < nl;
    ref[k] = h ? a.s.rs_ref[B.pos0 + i] : 0;
    loc[k] = h ? a.s.rs_loc[B.pos0 + i] : 0;
    off[k] = h ? a.s.off[B.pos0 + i] : 0;
    sc[k] = fs ? fs[ref[k]] : R(1);
    fill[k] = valid && !valid[ref[k]];  // a divide missing from the store: the reader's 0.001 fill (readers.py:523-530)
  }
  // q' row of step t (t clamped into [0, T)): max(t - shift, 0) -- step t routes q'[t - 1] (mmc.py:421-424),
  // shift 0 in accumulation mode -- divided by the hours per stored row (readers.py:513-519)
  // (32-bit: T < 2^31; an int64 division is ~130 instructions per row, a branch around the row's loads)
  const unsigned H = (unsigned)a.qp_hours, shift = (unsigned)a.qp_shift;
  auto rowoff = [&](int64_t t64) {
    unsigned t = (unsigned)(t64 < T ? t64 : T - 1);
    t = t > shift ? t - shift : 0u;
    return (int64_t)(H == 1u ? t : t / H) * N;
  };
  R v[KG][G];
  auto load = [&](int64_t t0) {
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const R* row = qp + rowoff(t0 + j);
#pragma unroll
      for (int k = 0; k < KG; ++k)
        if (tid + k * BS < nl) v[k][j] = row[ref[k]];
    }
  };
  R* qs = static_cast<R*>(a.qs) + T * B.pos0 + B.pre_dn;
  bool nan = false;
  load(tA);
#pragma unroll 1
  for (int64_t t0 = tA; t0 < tB; t0 += G) {
#pragma unroll
    for (int k = 0; k < KG; ++k) {
      if (tid + k * BS >= nl) continue;
#pragma unroll
      for (int j = 0; j < G; ++j) {
        R x = fill[k] ? R(0.001f) : v[k][j];
        if (fs) x = x * sc[k];
        tile[j * nl + loc[k]] = x;
        nan = nan || x != x;
      }
    }
    __syncthreads();
    if (t0 + G < tB) load(t0 + G);  // lands while this tile is written out
    const int jn = (int)(tB - t0 < G ? tB - t0 : G);
#pragma unroll
    for (int k = 0; k < KG; ++k) {
      const int r = tid + k * BS;
      if (r >= nl) continue;
      R* col = qs + (t0 + off[k]) * nl + r;
      if (jn == G) {
#pragma unroll
        for (int j = 0; j < G; ++j) col[(int64_t)j * nl] = tile[j * nl + r];
      } else {
        for (int j = 0; j < jn; ++j) col[(int64_t)j * nl] = tile[j * nl + r];
      }
    }
    __syncthreads();
  }
  flag_nan(a, nan);
}

// Adjoint of gather_qprime: dL/dq'[s, ref] = flow_scale[ref] * sum over the steps t reading row s
// (ascending t) of gqs[tick(t, ref)]; 0 for a divide filled with 0.001 (readers.py:523-530).  Step t
// reads row max(t - 1, 0) / qp_hours (mmc.py:421-424 for t >= 1, the hot start for t = 0).  One
// thread per (row, reference reach): the writes are coalesced rows of q'.
template <typename R>
__global__ void scatter_qprime_grad_kernel(RouteArgs a, int64_t rows, R* out) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t N = a.N, T = a.T, H = a.qp_hours;
  if (w >= rows * N) return;
  const int64_t srow = w / N;
  const int ref = (int)(w % N);
  const int P = a.s.pos_of_ref[ref];
  const BlockDesc B = a.s.blocks[a.s.block_of_pos[P]];
  const int64_t r = P - B.pos0, o = a.s.off[P];
  const R* g = static_cast<const R*>(a.gqs) + T * B.pos0 + B.pre_dn;
  // steps whose row is srow: max(t - 1, 0) in [srow H, srow H + H)
  int64_t t0 = srow * H + 1, t1 = srow * H + H + 1;
  if (srow == 0) t0 = 0;
  t1 = t1 < T ? t1 : T;
  R acc = R(0);
  for (int64_t t = t0; t < t1; ++t) acc = acc + g[(t + o) * B.nloc + r];
  if (a.qp_valid && !a.qp_valid[ref]) acc = R(0);
  if (a.fs) acc = acc * static_cast<const R*>(a.fs)[ref];
  out[w] = acc;
}

// Row layout (a store of qp_hours > 1 steps per row): per block [qs_rows][nloc], row d holds q' row d
// of the store for every local position -- qp_hours times fewer bytes than the tick-major layout.
template <typename R, int G>
__global__ void __launch_bounds__(1024) gather_qprime_rows_kernel(RouteArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char gsm[];
  R* tile = reinterpret_cast<R*>(gsm);  // [G][nloc]
  if (a.owned && !a.owned[blockIdx.x]) return;  // split basin: another rank's block
  const BlockDesc B = a.s.blocks[blockIdx.x];
  const int64_t N = a.N, d0 = (int64_t)blockIdx.y * G;
  const int nl = B.nloc;
  const R* qp = static_cast<const R*>(a.qprime);
  const R* fs = static_cast<const R*>(a.fs);
  const int* rs_loc = a.s.rs_loc + B.pos0;
  const int* rs_ref = a.s.rs_ref + B.pos0;
  const int jn = (int)(a.qs_rows - d0 < G ? a.qs_rows - d0 : G);
  const unsigned char* valid = a.qp_valid;
  bool nan = false;
  for (int i = threadIdx.x; i < nl; i += 1024) {
    const int ref = rs_ref[i], loc = rs_loc[i];
    R v[G];
#pragma unroll
    for (int j = 0; j < G; ++j) v[j] = j < jn ? qp[(d0 + j) * N + ref] : R(0);
    if (valid && !valid[ref]) {
#pragma unroll
      for (int j = 0; j < G; ++j) v[j] = R(0.001f);  // readers.py:523-530
    }
    if (fs) {
      const R f = fs[ref];
#pragma unroll
      for (int j = 0; j < G; ++j) v[j] = v[j] * f;
    }
#pragma unroll
    for (int j = 0; j < G; ++j) {
      tile[j * nl + loc] = v[j];
      nan = nan || (j < jn && v[j] != v[j]);
    }
  }
  flag_nan(a, nan);
  __syncthreads();
  R* qs = static_cast<R*>(a.qs) + (int64_t)a.qs_rows * B.pos0;
  for (int r = threadIdx.x; r < nl; r += 1024) {
#pragma unroll
    for (int j = 0; j < G; ++j)
      if (j < jn) qs[(d0 + j) * nl + r] = tile[j * nl + r];
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
    const R Q = (t == 0 && a.carry) ? x : rmax_nan(x, R(a.qlb));
    acc = acc + Q;
  }
  // output[:, 0] = clamp(initial) (mmc.py:412); later steps are sums of clamped states
  out[g * a.T + t] = (t == 0) ? rmax_nan(acc, R(a.qlb)) : acc;
}

// mask[g] = 1 where the t = 0 gauge sum (before its clamp, as gauge_reduce_kernel) is >= q_lb:
// torch.clamp's backward passes the gradient there (inclusive at the bound).
template <typename R>
__global__ void gauge_mask0_kernel(GaugeArgs a, const R* xsave, unsigned char* mask) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= a.G) return;
  R acc = R(0);
  for (int64_t k = a.goff[g]; k < a.goff[g + 1]; ++k) {
    const int P = a.pos_of_ref[a.gidx[k]];
    const BlockDesc B = a.s.blocks[a.block_of_pos[P]];
    const R x = xsave[a.T * B.pos0 + B.pre_dn + (int64_t)a.s.off[P] * B.nloc + (P - B.pos0)];
    acc = acc + (a.carry ? x : rmax_nan(x, R(a.qlb)));
  }
  mask[g] = (acc >= R(a.qlb)) ? 1 : 0;
}

// ============================================================================================
// Gauge-mode training objective, fused: hourly gauge sums -> trim -> daily area means
// (scripts/train.py:78-82: downsample(runoff[:, 13 : -11 + tau], num_days), io/functions.py:7-23,
// F.interpolate(mode="area") = adaptive average pooling: day d averages hours
// [floor(d L / D), ceil((d + 1) L / D)) of the L-hour trimmed window).  The (G, T) hourly series is
// never materialised; only (G, D) leaves the kernel.
// ============================================================================================
__host__ __device__ inline int64_t pool_start(int64_t d, int64_t L, int64_t D) { return (d * L) / D; }
__host__ __device__ inline int64_t pool_end(int64_t d, int64_t L, int64_t D) { return ((d + 1) * L + D - 1) / D; }

template <typename R>
__device__ __forceinline__ R gauge_hour(const GaugeArgs& a, const R* xsave, int64_t g, int64_t t) {
  R acc = R(0);
  for (int64_t k = a.goff[g]; k < a.goff[g + 1]; ++k) {
    const int P = a.pos_of_ref[a.gidx[k]];
    const BlockDesc B = a.s.blocks[a.block_of_pos[P]];
    const int r = P - B.pos0;
    const int64_t tick = t + a.s.off[P];
    const R x = xsave[a.T * B.pos0 + B.pre_dn + tick * B.nloc + r];
    acc = acc + ((t == 0 && a.carry) ? x : rmax_nan(x, R(a.qlb)));
  }
  return (t == 0) ? rmax_nan(acc, R(a.qlb)) : acc;  // as gauge_reduce_kernel (mmc.py:412, 433-439)
}

template <typename R>
__global__ void gauge_daily_kernel(GaugeArgs a, const R* xsave, int64_t t0, int64_t L, int64_t D, R* out) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= a.G * D) return;
  const int64_t g = w / D, d = w % D;
  const int64_t h0 = pool_start(d, L, D), h1 = pool_end(d, L, D);
  R sum = R(0);
  for (int64_t h = h0; h < h1; ++h) sum = sum + gauge_hour<R>(a, xsave, g, t0 + h);
  out[w] = sum / R(h1 - h0);  // adaptive_avg_pool: sum / kh / kw with kh = 1
}

// Adjoint seed of the pooling: dL/dhourly[g, t] = sum over the days d whose window holds t - t0 of
// dL/ddaily[g, d] / len(d) (ascending d, as adaptive_avg_pool's backward accumulates), 0 outside
// the trimmed window.  Feeds the gauge-mode routing adjoint.
template <typename R>
__global__ void gauge_daily_seed_kernel(int64_t G, int64_t T, int64_t t0, int64_t L, int64_t D, const R* gd, R* gh) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= G * T) return;
  const int64_t g = w / T, t = w % T, h = t - t0;
  R acc = R(0);
  if (h >= 0 && h < L) {
    const int64_t dc = (h * D) / L;
    const int64_t dlo = dc > 0 ? dc - 1 : 0, dhi = dc + 1 < D ? dc + 1 : D - 1;
    for (int64_t d = dlo; d <= dhi; ++d)
      if (h >= pool_start(d, L, D) && h < pool_end(d, L, D)) acc = acc + gd[g * D + d] / R(pool_end(d, L, D) - pool_start(d, L, D));
  }
  gh[w] = acc;
}

// ============================================================================================
// Host launchers
// ============================================================================================
// Split basin: after the layout, each block's granule rows (tagged pointers, bit 0 = another rank's
// memory: system scope): forward, its cut-outs' export rows; backward, its virtuals' export rows then
// its cut-outs' import rows -- resolved once per launch, no dependent global load per hand-off
size_t split_table_bytes(const Graph* g, bool backward) {
  if (g->split.nranks == 0) return 0;
  return 8 * (size_t)(backward ? g->max_virt + g->max_cout : g->max_cout);
}

// The backward's slot buffers on this graph: the KR rule's, unless its double buffer does not fit a CU's
// LDS at this real size (fp64 at KR = 2: 96 B per slot, ~1.6K-reach blocks), then one -- two barriers per
// tick instead of DDR_ERR_CAPACITY (the graph packer sizes blocks for the fp32 layouts)
template <typename R>
int bwd_xb_of(const Graph* g) {
  if (bwd_xbuf(g->kr) == 1) return 1;
  const size_t b2 = route_lds_bytes((size_t)route_slot_stride(g->max_slots), (size_t)g->max_virt,
                                    (size_t)g->max_cout, (size_t)g->max_xl, true, sizeof(R), g->kr, 2);
  return (sizeof(R) == 8 && g->kr == 2 && align16(b2) + split_table_bytes(g, true) > kLdsBudget) ? 1 : 2;
}

template <typename R>
size_t route_smem_bytes(const Graph* g, bool backward) {
  return route_lds_bytes((size_t)route_slot_stride(g->max_slots), (size_t)g->max_virt, (size_t)g->max_cout,
                         (size_t)g->max_xl, backward, sizeof(R), g->kr, backward ? bwd_xb_of<R>(g) : 0);
}

// the backward kernel of this launch (state gradients: GS; single-buffered fp64 KR = 2 slots: bwd_xb_of)
// (exact adjoint of the fp32 trajectory, DDR_BWD_EXACT_ADJOINT: df)
template <typename R, int KR>
const void* backward_kernel_of(const Graph* g, bool gs, bool df = false, int pl = 0) {
  if constexpr (KR == 2 && sizeof(R) == 8) {
    if (bwd_xb_of<R>(g) == 1)
      return gs ? (const void*)route_backward_kernel<R, KR, true, 1> : (const void*)route_backward_kernel<R, KR, false, 1>;
  }
  if constexpr (sizeof(R) == 4) {
    if (df)
      return gs ? (const void*)route_backward_kernel<R, KR, true, 0, true>
                : (const void*)route_backward_kernel<R, KR, false, 0, true>;
  }
  if constexpr (sizeof(R) == 4) {
    if (!gs && pl == 2) return (const void*)route_backward_kernel<R, KR, false, 0, false, 2>;
  }
  return gs ? (const void*)route_backward_kernel<R, KR, true> : (const void*)route_backward_kernel<R, KR, false>;
}
// the plain backward instance a launch can take (route_backward_kernel's PL), 0 when none
inline int backward_plain_of(const Graph* g, const RouteArgs& a) {
  if ((a.flags & kFlagNoPlain) || g->split.nranks > 0 || a.prof != nullptr || a.gseed != nullptr || (a.T & 3) != 0) return 0;
  // gauge mode only: c3s8 backward -4.5 %; per-reach dL/drunoff (PL = 1) measured 0.5-1.5 % slower at C5 and
  // 3 % at light load (r05_plain3, r05_pl1), so that instance is not built
  return a.g_roff != nullptr ? 2 : 0;
}

// the faithful forward instance for a plain code (route_forward_kernel's PL; 0: the general one)
template <typename R, int KR, int XB>
auto forward_faithful_of(int pl) {
  switch (pl) {
    case 1: return route_forward_kernel<R, KR, 2, XB, 1>;
    case 2: return route_forward_kernel<R, KR, 2, XB, 2>;
    case 4: return route_forward_kernel<R, KR, 2, XB, 4>;
    default: return route_forward_kernel<R, KR, 2, XB>;
  }
}

template <typename R, int KR>
hipError_t launch_route_kr(const Graph* g, RouteArgs a, bool backward, hipStream_t stream) {
  const size_t base = route_smem_bytes<R>(g, backward);
  const size_t smem = align16(base) + split_table_bytes(g, backward);
  a.slot_stride = route_slot_stride(g->max_slots);
  a.n_cut = g->n_cut;
  a.nblocks = (int32_t)g->blocks.size();
  a.xl_off = (int32_t)(base - (size_t)g->max_xl * 4);  // the lists close the base LDS layout
  a.own_off = a.xl_off - (int32_t)align16(4 * (size_t)std::max(g->max_virt, g->max_cout));
  a.xt_off = g->split.nranks > 0 ? (int32_t)align16(base) : 0;
  const dim3 grid((unsigned)g->blocks.size()), block(kBlockThreads);
  if (backward) {
    const void* kern = backward_kernel_of<R, KR>(g, a.gqs != nullptr, (a.flags & DDR_BWD_EXACT_ADJOINT) != 0,
                                                  backward_plain_of(g, a));
    hipError_t e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    void* kargs[] = {&a};
    e = hipLaunchKernel(kern, grid, block, kargs, smem, stream);
    if (e != hipSuccess) return e;
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    const unsigned fb = (unsigned)((g->n + 255) / 256);
    hipLaunchKernelGGL(finish_grads_kernel<R>, dim3(fb), dim3(256), 0, stream, g->n,
                       (const double*)(a.bwd_bnd + 2 * g->n_cut * a.T), (R*)a.gn, (R*)a.gq, (R*)a.gp);
  } else {
    auto kern = route_forward_kernel<R, KR, 0>;
    size_t fsmem = smem;
    if constexpr (std::is_same<R, float>::value) {
      // the plain instance (route_forward_kernel's PL) this launch can take: 0 none, 1 runoff rows, 2 none written
      const bool plain_ok = !(a.flags & kFlagNoPlain);
      const bool rows = a.runoff != nullptr && !(a.flags & DDR_FWD_NO_RUNOFF);
      int plain = 0;
      if (plain_ok && g->split.nranks == 0 && a.prof == nullptr && !(a.flags & DDR_FWD_ACCUMULATE)) {
        if (rows) plain = ((a.T & 3) == 0 && a.qs_rows <= 0) ? 1 : 0;
        else plain = a.qs_rows > 0 ? 4 : 2;
      }
      if (a.flags & DDR_FWD_FAST_MATH) kern = route_forward_kernel<R, KR, 1>;
      else if (a.flags & DDR_FWD_FAITHFUL_MATH) kern = forward_faithful_of<R, KR, 0>(plain);
      // KR = 4 (faithful): double-buffered x slots -- one barrier per tick -- where this graph's largest
      // block leaves the LDS for a second buffer (C5's blocks of <= ~3800 reaches; C3's 4096 do not)
      if constexpr (KR == 4) {
        const size_t b2 = route_lds_bytes((size_t)route_slot_stride(g->max_slots), (size_t)g->max_virt,
                                          (size_t)g->max_cout, (size_t)g->max_xl, false, sizeof(R), g->kr, 2);
        const size_t s2 = align16(b2) + split_table_bytes(g, false);
        if ((a.flags & DDR_FWD_FAITHFUL_MATH) && s2 <= kLdsBudget) {
          kern = forward_faithful_of<R, KR, 2>(plain);
          fsmem = s2;
          a.xl_off = (int32_t)(b2 - (size_t)g->max_xl * 4);
          a.own_off = a.xl_off - (int32_t)align16(4 * (size_t)std::max(g->max_virt, g->max_cout));
          a.xt_off = g->split.nranks > 0 ? (int32_t)align16(b2) : 0;
        }
      }
    }
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)fsmem);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, grid, block, fsmem, stream, a);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (a.q_last || a.tw_last || a.ss_last) {
      auto last = route_last_kernel<R, 0>;
      if constexpr (std::is_same<R, float>::value) {
        if (a.flags & DDR_FWD_FAST_MATH) last = route_last_kernel<R, 1>;
        else if (a.flags & DDR_FWD_FAITHFUL_MATH) last = route_last_kernel<R, 2>;
      }
      hipLaunchKernelGGL(last, dim3((unsigned)((g->n + 255) / 256)), dim3(256), kMathTabBytes, stream, a);
    }
  }
  return hipGetLastError();
}

template <typename R>
hipError_t launch_route(const Graph* g, const RouteArgs& a, bool backward, hipStream_t stream) {
  switch (g->kr) {
    case 1: return launch_route_kr<R, 1>(g, a, backward, stream);
    case 2: return launch_route_kr<R, 2>(g, a, backward, stream);
    default: return launch_route_kr<R, 4>(g, a, backward, stream);
  }
}

template <typename R>
int max_resident_blocks(const Graph* g, bool backward) {
  int nb = 0;
  const size_t smem = align16(route_smem_bytes<R>(g, backward)) + split_table_bytes(g, backward);
  const void* f = nullptr;
  switch (g->kr) {
    case 1: f = backward ? backward_kernel_of<R, 1>(g, false) : (const void*)route_forward_kernel<R, 1, 0>; break;
    case 2: f = backward ? backward_kernel_of<R, 2>(g, false) : (const void*)route_forward_kernel<R, 2, 0>; break;
    default: f = backward ? backward_kernel_of<R, 4>(g, false) : (const void*)route_forward_kernel<R, 4, 0>;
  }
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, kBlockThreads, smem) != hipSuccess) return -1;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, g->device) != hipSuccess) return -1;
  return nb * prop.multiProcessorCount;
}

// Split basin: before a routing launch, every rank of the split announces (system-scope store into each
// peer's epoch word) that its receive rows are reset for launch `epoch` and waits until every peer has
// announced the same; only then may a peer's blocks write into them.  Bounded: a peer that never
// arrives is recorded in the status block (DDR_ERR_TIMEOUT at the next library call).
__global__ void split_barrier_kernel(SplitBarrierArgs b) {
  if (threadIdx.x != 0) return;
  for (int p = 0; p < b.nranks; ++p) {
    if (p == b.rank) continue;
    __hip_atomic_store(b.peer[p] + b.slot * kMaxSplitRanks + b.rank, b.epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  for (int p = 0; p < b.nranks; ++p) {
    if (p == b.rank) continue;
    unsigned spins = 0;
    while (__hip_atomic_load(b.mine + b.slot * kMaxSplitRanks + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) <
           b.epoch) {
      if (++spins > (1u << 22)) {  // ~10 s
        atomicAdd(b.status, 1u);
        atomicCAS(b.status + 1, 0u, 0x40000000u + (unsigned)p);
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
  }
}

hipError_t launch_split_barrier(const SplitBarrierArgs& b, hipStream_t stream) {
  hipLaunchKernelGGL(split_barrier_kernel, dim3(1), dim3(64), 0, stream, b);
  return hipGetLastError();
}

// Split basin, after the forward (grid-stride over n_x rows x T): rows received from another rank
// (xcons == this rank) -> bnd[edge] (the per-call boundary buffer the autograd node keeps; a later forward
// on the same graph resets and rewrites the receive rows); and a NaN in column 0 of every runoff row of a
// reach whose block another rank runs (those rows are never written: misuse shows as NaN, not as stale
// memory).  The last-step outputs of those reaches are NaN as well (route_last_kernel).
template <typename R>
__global__ void split_finish_kernel(RouteArgs a, int64_t n_x) {
  const int64_t T = a.T;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < n_x * T; w += stride) {
    const int64_t xi = w / T, t = w % T;
    if (a.xcons[xi] != a.xrank) continue;
    a.bnd[a.xedge[xi] * T + t] = __longlong_as_double(load_granule_sys(a.xfwd + w));
  }
  if (a.runoff) {
    for (int64_t P = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; P < a.N; P += stride)
      if (!a.owned[a.s.block_of_pos[P]]) static_cast<R*>(a.runoff)[(int64_t)a.s.ref[P] * T] = R(__builtin_nan(""));
  }
}

template <typename R>
hipError_t launch_split_finish(const Graph* g, const RouteArgs& a, hipStream_t stream) {
  if (g->split.nranks == 0) return hipSuccess;
  const int64_t work = std::max<int64_t>((int64_t)g->split.n_x * a.T, g->n);
  const unsigned nb = (unsigned)std::min<int64_t>((work + 255) / 256, 4096);
  hipLaunchKernelGGL(split_finish_kernel<R>, dim3(nb), dim3(256), 0, stream, a, (int64_t)g->split.n_x);
  return hipGetLastError();
}

template <typename R>
hipError_t launch_gather_qprime(const Graph* g, RouteArgs& a, hipStream_t stream) {
  if (g->max_nloc == 0 || a.T == 0) return hipSuccess;
  if (a.flags & DDR_FWD_CHECK_QPRIME) {
    hipLaunchKernelGGL(nan_last_row_kernel<R>, dim3((unsigned)((a.N + 255) / 256)), dim3(256), 0, stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  constexpr int G = sizeof(R) == 4 ? 8 : 4;  // G * 4096 reaches * sizeof(R) <= 128 KiB of LDS
  const size_t smem = (size_t)G * g->max_nloc * sizeof(R);
  if (a.qs_rows > 0) {
    auto rk = gather_qprime_rows_kernel<R, G>;
    hipError_t e = hipFuncSetAttribute((const void*)rk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(rk, dim3((unsigned)g->blocks.size(), (unsigned)((a.qs_rows + G - 1) / G)), dim3(1024), smem,
                       stream, a);
    return hipGetLastError();
  }
  // workgroups of (block, chunk of kTilesPerChunk tiles): short enough that the dispatcher balances blocks of
  // unequal size (a chunk of ~1000 steps left a ~1.5-ms tail behind the largest blocks), long enough that the
  // per-chunk index reads are a small fraction of the q' bytes
  auto launch = [&](auto kern, int gsteps, int bs) -> hipError_t {
    const size_t sm = (size_t)gsteps * g->max_nloc * sizeof(R);
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    if (e != hipSuccess) return e;
    constexpr int64_t kTilesPerChunk = 4;  // C5: 13.35 ms (2: 13.34, 8: 13.45, 16: 13.73; r05's tile per workgroup 13.92)
    const int64_t nb = (int64_t)g->blocks.size();
    const int64_t chunk = kTilesPerChunk * gsteps;
    const int64_t y = (a.T + chunk - 1) / chunk;
    hipLaunchKernelGGL(kern, dim3((unsigned)(nb * y)), dim3(bs), sm, stream, a, (int)chunk, (int)y);
    return hipGetLastError();
  };
  if constexpr (sizeof(R) == 4) {
    if (g->max_nloc <= 256) return launch(gather_qprime_kernel<R, 32, 256, 1>, 32, 256);
    if (g->max_nloc <= 512) return launch(gather_qprime_kernel<R, 32, 512, 1>, 32, 512);
    if (g->max_nloc <= 1024) return launch(gather_qprime_kernel<R, 16, 1024, 1>, 16, 1024);
    if (g->max_nloc <= 2048) return launch(gather_qprime_kernel<R, 16, 1024, 2>, 16, 1024);
    return launch(gather_qprime_kernel<R, G, 1024, 4>, G, 1024);
  } else {
    if (g->max_nloc <= 1024) return launch(gather_qprime_kernel<R, G, 1024, 1>, G, 1024);
    if (g->max_nloc <= 2048) return launch(gather_qprime_kernel<R, G, 1024, 2>, G, 1024);
    return launch(gather_qprime_kernel<R, G / 2, 1024, 4>, G / 2, 1024);  // (G = 4: spills at four reaches)
  }
}

template <typename R>
hipError_t launch_scatter_qprime_grad(const Graph* g, const RouteArgs& a, int64_t rows, R* out, hipStream_t stream) {
  const int64_t total = rows * g->n;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(scatter_qprime_grad_kernel<R>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, a,
                     rows, out);
  return hipGetLastError();
}

template <typename R>
hipError_t launch_gauge_mask0(const GaugeArgs& a, const R* xsave, unsigned char* mask, hipStream_t stream) {
  if (a.G == 0) return hipSuccess;
  hipLaunchKernelGGL(gauge_mask0_kernel<R>, dim3((unsigned)((a.G + 255) / 256)), dim3(256), 0, stream, a, xsave, mask);
  return hipGetLastError();
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

template <typename R>
hipError_t launch_gauge_daily(const GaugeArgs& a, const R* xsave, int64_t t0, int64_t L, int64_t D, R* out,
                              hipStream_t stream) {
  const int64_t total = a.G * D;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(gauge_daily_kernel<R>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, a, xsave, t0,
                     L, D, out);
  return hipGetLastError();
}

template <typename R>
hipError_t launch_gauge_daily_seed(int64_t G, int64_t T, int64_t t0, int64_t L, int64_t D, const R* gd, R* gh,
                                   hipStream_t stream) {
  const int64_t total = G * T;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(gauge_daily_seed_kernel<R>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, G, T, t0,
                     L, D, gd, gh);
  return hipGetLastError();
}

template hipError_t launch_route<float>(const Graph*, const RouteArgs&, bool, hipStream_t);
template hipError_t launch_route<double>(const Graph*, const RouteArgs&, bool, hipStream_t);
template int max_resident_blocks<float>(const Graph*, bool);
template int max_resident_blocks<double>(const Graph*, bool);
template hipError_t launch_split_finish<float>(const Graph*, const RouteArgs&, hipStream_t);
template hipError_t launch_split_finish<double>(const Graph*, const RouteArgs&, hipStream_t);
template hipError_t launch_gather_qprime<float>(const Graph*, RouteArgs&, hipStream_t);
template hipError_t launch_gather_qprime<double>(const Graph*, RouteArgs&, hipStream_t);
template hipError_t launch_scatter_qprime_grad<float>(const Graph*, const RouteArgs&, int64_t, float*, hipStream_t);
template hipError_t launch_scatter_qprime_grad<double>(const Graph*, const RouteArgs&, int64_t, double*, hipStream_t);
template hipError_t launch_gauge_mask0<float>(const GaugeArgs&, const float*, unsigned char*, hipStream_t);
template hipError_t launch_gauge_mask0<double>(const GaugeArgs&, const double*, unsigned char*, hipStream_t);
template hipError_t launch_gauge<float>(const GaugeArgs&, const float*, float*, hipStream_t);
template hipError_t launch_gauge<double>(const GaugeArgs&, const double*, double*, hipStream_t);

template hipError_t launch_gauge_daily<float>(const GaugeArgs&, const float*, int64_t, int64_t, int64_t, float*, hipStream_t);
template hipError_t launch_gauge_daily<double>(const GaugeArgs&, const double*, int64_t, int64_t, int64_t, double*,
                                               hipStream_t);
template hipError_t launch_gauge_daily_seed<float>(int64_t, int64_t, int64_t, int64_t, int64_t, const float*, float*,
                                                   hipStream_t);
template hipError_t launch_gauge_daily_seed<double>(int64_t, int64_t, int64_t, int64_t, int64_t, const double*, double*,
                                                    hipStream_t);

}  // namespace ddr
