// C ABI of libddr_mc.so (include/ddr_mc.h).  No exception crosses this boundary; errors are
// returned as ddr_status codes with a thread-local message (ddr_last_error).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <mutex>
#include <string>

#include "internal.h"
#include "route_args.h"
#include "train.h"

namespace ddr {

namespace {
thread_local std::string g_last_error;
}

void set_error(const std::string& msg) { g_last_error = msg; }
ddr_status fail(ddr_status code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
const char* last_error_cstr() { return g_last_error.c_str(); }
ddr_status hip_fail(hipError_t e, const char* where) {
  g_last_error = std::string(where) + ": " + hipGetErrorString(e);
  return DDR_ERR_HIP;
}

}  // namespace ddr


using namespace ddr;

namespace {

// Measurement hooks (ddr_set_kernel_timing / ddr_set_block_profile): process-wide, not for
// concurrent use from several host threads.
struct KernelTiming {
  bool on = false;
  hipEvent_t ev[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
  bool recorded[2] = {false, false};
} g_timing;
unsigned long long* g_prof[2] = {nullptr, nullptr};
int32_t g_debug = [] {  // ddr_set_debug_flags (DDR_NO_STEADY=1: the general tick path only, for A/B)
  auto on = [](const char* name) {
    const char* v = std::getenv(name);
    return v && v[0] == '1';
  };
  return (on("DDR_NO_STEADY") ? kFlagNoSteady : 0) | (on("DDR_NO_STORER") ? kFlagNoStorer : 0) |
         (on("DDR_NO_PLAIN") ? kFlagNoPlain : 0);
}();

// Hand-off failures surface without a host sync on the hot path: after every routing launch the
// status block's first words are copied (async, same stream) into a pinned slot with an event
// behind it.  Every later entry point polls the completed slots and returns DDR_ERR_TIMEOUT for
// a launch that timed out; ddr_status_check(1) waits for all of them.
struct PendingStatus {
  static constexpr int kSlots = 64;
  std::mutex mu;
  unsigned* host = nullptr;  // pinned, kSlots x 4 words
  hipEvent_t ev[kSlots] = {};
  const char* what[kSlots] = {};
  const void* graph[kSlots] = {};  // the launch's graph and stream, named in the error message
  hipStream_t stream[kSlots] = {};
  unsigned long long seq[kSlots] = {};
  unsigned long long launches = 0;  // routing launches enqueued by this process
  int head = 0;
  bool failed = false;
  std::string msg;

  void harvest(int k) {
    const unsigned* w = host + 4 * k;
    if (w[0] && !failed) {
      failed = true;
      char id[96];
      snprintf(id, sizeof(id), " (graph %p, stream %p, routing launch #%llu of this process)", graph[k],
               (void*)stream[k], seq[k]);
      // word 1: first failing logical block + 1, or 0x40000000 + rank for a split basin's peer that never
      // arrived at the launch's epoch hand-shake (route.hip: split_barrier_kernel)
      const std::string where = w[1] >= 0x40000000u
                                    ? "split-basin hand-shake: rank " + std::to_string((int)(w[1] - 0x40000000u)) +
                                          " never arrived"
                                    : "first logical block " + std::to_string((int)w[1] - 1);
      msg = std::to_string(w[0]) + " inter-workgroup hand-offs of a " + what[k] + " launch" + id + " timed out (" +
            where + "); its outputs hold NaN. Reported by the next library call: call ddr_status_check(1) at the "
            "end of a run so that a timeout in the last launch is not missed";
    }
    (void)hipEventDestroy(ev[k]);
    ev[k] = nullptr;
  }
  // caller holds mu
  void poll(bool wait) {
    for (int k = 0; k < kSlots; ++k) {
      if (!ev[k]) continue;
      if (wait) (void)hipEventSynchronize(ev[k]);
      if (hipEventQuery(ev[k]) == hipSuccess) harvest(k);
    }
  }
  ddr_status take_error() {
    if (!failed) return DDR_OK;
    failed = false;
    return fail(DDR_ERR_TIMEOUT, msg);
  }
  ddr_status enqueue(const void* status, hipStream_t s, const char* which, const void* g) {
    std::lock_guard<std::mutex> lk(mu);
    if (!host) DDR_HIP(hipHostMalloc(reinterpret_cast<void**>(&host), sizeof(unsigned) * 4 * kSlots, hipHostMallocDefault));
    const int k = head;
    head = (head + 1) % kSlots;
    if (ev[k]) {
      (void)hipEventSynchronize(ev[k]);
      harvest(k);
    }
    DDR_HIP(hipMemcpyAsync(host + 4 * k, status, 2 * sizeof(unsigned), hipMemcpyDeviceToHost, s));
    DDR_HIP(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
    what[k] = which;
    graph[k] = g;
    stream[k] = s;
    seq[k] = ++launches;
    DDR_HIP(hipEventRecord(ev[k], s));
    return DDR_OK;
  }
  ddr_status check(bool wait) {
    std::lock_guard<std::mutex> lk(mu);
    if (host) poll(wait);
    return take_error();
  }
} g_pending;

// Restores the calling thread's current device on scope exit (entry points that act on a graph's own
// device, which need not be the caller's current one)
struct DeviceGuard {
  int prev = -1;
  hipError_t error = hipSuccess;
  explicit DeviceGuard(int dev) {
    error = hipGetDevice(&prev);
    if (error == hipSuccess && prev != dev) error = hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// DDR_FWD_CHECK_QPRIME: per host thread and device, the NaN word of its last checked forward, copied to
// pinned memory behind the q' gather, and the event after that copy (ddr_qprime_nan_wait waits for the
// gather only).  Keyed by device: an event belongs to the device current at its creation, so a thread
// routing on several GPUs records each launch's event on that launch's own device
constexpr int kNanDevices = 64;
struct NanCheck {
  unsigned* host = nullptr;
  hipEvent_t ev = nullptr;
  bool armed = false;
};
thread_local NanCheck t_nan[kNanDevices];
thread_local int t_nan_dev = -1;  // device of the calling thread's last checked forward

hipError_t nan_check_mark(const void* status, hipStream_t s) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= kNanDevices) return hipErrorInvalidDevice;
  NanCheck& c = t_nan[dev];
  if (!c.host) {
    e = hipHostMalloc(reinterpret_cast<void**>(&c.host), 16, hipHostMallocDefault);
    if (e != hipSuccess) return e;
  }
  if (!c.ev) {
    e = hipEventCreateWithFlags(&c.ev, hipEventDisableTiming);
    if (e != hipSuccess) return e;
  }
  e = hipMemcpyAsync(c.host, static_cast<const unsigned*>(status) + kStatusNaN, sizeof(unsigned),
                     hipMemcpyDeviceToHost, s);
  if (e != hipSuccess) return e;
  if (t_nan_dev >= 0) t_nan[t_nan_dev].armed = false;  // "the last checked forward" is this one
  c.armed = true;
  t_nan_dev = dev;
  return hipEventRecord(c.ev, s);
}

// Stream capture (a hipGraph of a whole training step, e.g. torch.cuda.graph): the launches are recorded and
// replayed later, so the host-side bookkeeping of a launch -- the status harvest (a D2H copy and an event per
// launch, polled by later calls), the kernel timers, the wait for the graph's upload event (recorded outside
// the capture: capture a step only after the graph has been used once) -- is skipped while the stream
// captures.  A timed-out hand-off inside a replayed step still writes NaN into its outputs.
bool capturing(hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}
// Order `s` after the graph's build.  A capture cannot wait on the upload event (recorded outside it), so a
// device- or stream-built graph whose completion no launch outside a capture has waited for yet is refused
// there: its first replay could read a half-uploaded schedule.
ddr_status ready_for(const Graph* g, hipStream_t s) {
  if (capturing(s)) {
    if (g->ready && !g->ready_waited.load(std::memory_order_acquire))
      return fail(DDR_ERR_ARG, "graph used inside a stream capture before any launch outside it waited for its build: "
                               "route with it once outside the capture first");
    return DDR_OK;
  }
  DDR_HIP(graph_ready(g, s));
  g->ready_waited.store(true, std::memory_order_release);
  return DDR_OK;
}
#define DDR_TRY(call)                   \
  do {                                  \
    const ddr_status _st = (call);      \
    if (_st != DDR_OK) return _st;      \
  } while (0)

hipError_t timing_mark(int which, int edge, hipStream_t s) {
  if (!g_timing.on || capturing(s)) return hipSuccess;
  hipEvent_t& e = g_timing.ev[which][edge];
  if (!e) {
    hipError_t r = hipEventCreate(&e);
    if (r != hipSuccess) return r;
  }
  if (edge == 1) g_timing.recorded[which] = true;
  return hipEventRecord(e, s);
}

template <typename R>
ddr_status check_common(const ddr_graph* gh, const ddr_mc_consts* c, const ddr_mc_reaches* r, int64_t T) {
  if (!gh || !c || !r) return fail(DDR_ERR_ARG, "null graph/consts/reaches");
  if (T < 1) return fail(DDR_ERR_ARG, "T must be >= 1");
  if (!r->n || !r->q_spatial || !r->p_spatial || !r->length || !r->slope || !r->x_storage)
    return fail(DDR_ERR_ARG, "null per-reach input");
  if (r->p_stride != 0 && r->p_stride != 1) return fail(DDR_ERR_ARG, "p_stride must be 0 or 1");
  if (r->qprime_hours < 0 || r->qprime_hours > (int64_t(1) << 20)) return fail(DDR_ERR_ARG, "bad qprime_hours");
  const Graph* g = reinterpret_cast<const Graph*>(gh);
  if (!g->uploaded) return fail(DDR_ERR_ARG, "graph was built host-only: upload it first (ddr_graph_upload)");
  if (T * (g->n + 1) > (int64_t(1) << 62)) return fail(DDR_ERR_ARG, "T * N overflows");
  return DDR_OK;
}

template <typename R>
void fill_common(RouteArgs& a, const Graph* g, const ddr_mc_consts* c, const ddr_mc_reaches* r, int64_t T,
                 const R* qprime, int32_t flags) {
  std::memset(&a, 0, sizeof(a));
  a.s = g->dev;
  a.N = g->n;
  a.T = T;
  a.flags = flags;
  a.p_stride = (int32_t)r->p_stride;
  a.n = r->n;
  a.q = r->q_spatial;
  a.p = r->p_spatial;
  a.L = r->length;
  a.S = r->slope;
  a.X = r->x_storage;
  a.fs = r->flow_scale;
  a.qp_hours = r->qprime_hours > 1 ? (int32_t)r->qprime_hours : 1;
  a.qp_shift = (flags & DDR_FWD_ACCUMULATE) ? 0 : 1;
  a.qp_valid = r->qprime_valid;
  choose_qs_layout(a);  // needs T, qp_hours, qp_shift
  a.qprime = qprime;
  a.c[0] = c->dt;
  a.c[1] = c->discharge_lb;
  a.c[2] = c->velocity_lb;
  a.c[3] = c->velocity_ub;
  a.c[4] = c->depth_lb;
  a.c[5] = c->bottom_width_lb;
  a.c[6] = c->side_slope_lb;
  a.c[7] = c->side_slope_ub;
  for (int i = 0; i < 8; ++i) a.cf[i] = (float)a.c[i];
  a.ln_dlb = std::log(sizeof(R) == 4 ? (double)a.cf[4] : a.c[4]);
}

// The routing kernels need no co-residency (ticket-ordered blocks, route.hip), only that one
// workgroup fits a CU with the schedule's LDS.
template <typename R>
ddr_status check_launchable(const Graph* g, bool backward) {
  const int cap = max_resident_blocks<R>(g, backward);
  if (cap < 0) return fail(DDR_ERR_HIP, "occupancy query failed");
  if (cap == 0)
    return fail(DDR_ERR_CAPACITY, std::string("the ") + (backward ? "backward" : "forward") +
                                      " routing kernel does not fit a CU at this schedule's LDS size" +
                                      (sizeof(R) == 8 ? " (fp64: use a smaller max_block_reaches)" : ""));
  return DDR_OK;
}

// Split basin (SplitState): the launch's split arguments, its receive rows reset, and the epoch hand-shake
// with the other ranks of the split (slot 0: forward, 1: backward), all stream-ordered before the launch.
ddr_status split_prepare(const Graph* g, RouteArgs& a, int64_t T, int slot, hipStream_t s) {
  SplitState& sp = const_cast<Graph*>(g)->split;
  if (sp.nranks == 0) return DDR_OK;
  if (T > sp.t_cap) return fail(DDR_ERR_ARG, "split basin: T exceeds the receive rows' capacity (ddr_graph_set_split t_cap)");
  a.owned = sp.owned;
  a.xid = sp.xid;
  a.xcons = sp.xcons;
  a.xprod = sp.xprod;
  a.xedge = sp.xedge;
  a.xrank = sp.rank;
  auto rows = [&](char* base, int which) {
    double* f = reinterpret_cast<double*>(base + xmem_flags_bytes());
    return which == 0 ? f : f + sp.n_x * T;
  };
  a.xfwd = rows(sp.local, 0);
  a.xbwd = rows(sp.local, 1);
  SplitBarrierArgs b;
  std::memset(&b, 0, sizeof(b));
  for (int p = 0; p < sp.nranks; ++p) {
    a.pxfwd[p] = rows(sp.peers[p], 0);
    a.pxbwd[p] = rows(sp.peers[p], 1);
    b.peer[p] = reinterpret_cast<unsigned long long*>(sp.peers[p]);
  }
  if (sp.n_x > 0) {
    double* mine = slot == 0 ? a.xfwd : a.xbwd;
    DDR_HIP(hipMemsetAsync(mine, 0xFF, sizeof(double) * (size_t)(sp.n_x * T) * (slot == 0 ? 1 : 2), s));
  }
  b.mine = reinterpret_cast<unsigned long long*>(sp.local);
  b.rank = sp.rank;
  b.nranks = sp.nranks;
  b.slot = slot;
  b.epoch = ++sp.epoch[slot];
  b.status = a.status;
  DDR_HIP(launch_split_barrier(b, s));
  return DDR_OK;
}

template <typename R>
ddr_status forward_impl(const ddr_graph* gh, const ddr_mc_consts* c, const ddr_mc_reaches* r, const R* qprime,
                        int64_t T, const R* q0, R* runoff, R* x_save, double* bnd, void* status, R* q_last,
                        R* tw, R* ss, int32_t flags, void* stream) {
  ddr_status st = check_common<R>(gh, c, r, T);
  if (st) return st;
  const Graph* g = reinterpret_cast<const Graph*>(gh);
  if (!qprime) return fail(DDR_ERR_ARG, "null qprime");
  if ((flags & DDR_FWD_CARRY) && !q0) return fail(DDR_ERR_ARG, "DDR_FWD_CARRY needs q0");
  if ((flags & DDR_FWD_CARRY) && (flags & DDR_FWD_ACCUMULATE))
    return fail(DDR_ERR_ARG, "DDR_FWD_ACCUMULATE has no carried state");
  if (!x_save) return fail(DDR_ERR_ARG, "x_save is required (routing state, and the staging of runoff)");
  if (g->n_cut > 0 && !bnd) return fail(DDR_ERR_ARG, "graph has cut edges: bnd buffer required");
  if (!status) return fail(DDR_ERR_ARG, "null status block");
  // a split basin's launches hand-shake per launch epoch with every peer: a launch only this rank makes
  // (a hot start, the daily accumulation) would leave the epochs of all later launches off by one
  if (g->split.nranks > 0 && (T < 2 || (flags & DDR_FWD_ACCUMULATE)))
    return fail(DDR_ERR_ARG, "split basin: hot-start (T = 1) and accumulation launches are not supported");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool cap = capturing(s);
  if (cap && (g->split.nranks > 0 || (flags & DDR_FWD_CHECK_QPRIME)))
    return fail(DDR_ERR_ARG, "stream capture: split-basin launches and the q' NaN check cannot be captured");
  if (!cap && (st = g_pending.check(false))) return st;
  if ((st = check_launchable<R>(g, false))) return st;
  DDR_TRY(ready_for(g, s));
  DDR_HIP(hipMemsetAsync(status, 0, kStatusBytes, s));
  if (g->n_cut > 0) DDR_HIP(hipMemsetAsync(bnd, 0xFF, sizeof(double) * g->n_cut * T, s));
  RouteArgs a;
  fill_common<R>(a, g, c, r, T, qprime, flags | g_debug);
  a.q0 = q0;
  a.runoff = (flags & DDR_FWD_NO_RUNOFF) ? nullptr : runoff;
  a.x_save = x_save;
  a.bnd = bnd;
  a.status = static_cast<unsigned*>(status);
  a.q_last = q_last;
  a.tw_last = tw;
  a.ss_last = ss;
  a.prof = g_prof[0];
  a.qs = x_save + (g->n * T + g->sum_dn);
  if ((st = split_prepare(g, a, T, 0, s))) return st;
  DDR_HIP(launch_gather_qprime<R>(g, a, s));
  if (flags & DDR_FWD_CHECK_QPRIME) DDR_HIP(nan_check_mark(status, s));
  DDR_HIP(timing_mark(0, 0, s));
  DDR_HIP(launch_route<R>(g, a, false, s));
  DDR_HIP(timing_mark(0, 1, s));
  DDR_HIP(launch_split_finish<R>(g, a, s));
  // runoff (N, T) is written by the routing kernel itself (16-B row segments every 4 steps)
  return cap ? DDR_OK : g_pending.enqueue(status, s, "forward", gh);
}

template <typename R>
ddr_status gauge_args(const ddr_graph* gh, const R* x_save, int64_t T, const ddr_gauges* gz, double qlb,
                      int32_t flags, GaugeArgs& a);

// Workspace of the state-gradient backward: dL/d(q' * flow_scale) in the schedule layout, then one
// byte per gauge (the t = 0 clamp mask).
int64_t state_work_bytes(const Graph* g, int64_t T, int64_t n_gauges, size_t rsize) {
  return (int64_t)align16(rsize * (size_t)(g->n * T + g->sum_dn)) + n_gauges;
}

template <typename R>
ddr_status backward_impl(const ddr_graph* gh, const ddr_mc_consts* c, const ddr_mc_reaches* r, const R* qprime,
                         int64_t T, const R* x_save, const double* bnd, const R* grad, const ddr_gauges* gauges,
                         double* bwd_bnd, void* status, R* gn, R* gq, R* gp, int32_t flags, void* stream,
                         int64_t qp_rows = 0, R* gqp = nullptr, R* gq0 = nullptr, void* work = nullptr,
                         const R* seed = nullptr) {
  ddr_status st = check_common<R>(gh, c, r, T);
  if (st) return st;
  const Graph* g = reinterpret_cast<const Graph*>(gh);
  if (!qprime || !x_save || !grad || !gn || !gq || !gp || !status)
    return fail(DDR_ERR_ARG, "null backward argument");
  if (g->n_cut > 0 && !bnd) return fail(DDR_ERR_ARG, "graph has cut edges: forward boundary buffer required");
  if (!bwd_bnd) return fail(DDR_ERR_ARG, "backward workspace required");
  if (flags & DDR_FWD_ACCUMULATE) return fail(DDR_ERR_ARG, "DDR_FWD_ACCUMULATE launches have no adjoint");
  if (gauges && (!gauges->reach_offsets || !gauges->reach_gauges))
    return fail(DDR_ERR_ARG, "gauge mode backward needs the reach->gauge map");
  if (g->split.nranks > 0 && (gauges || gqp || gq0))
    return fail(DDR_ERR_ARG, "split basin: gauge mode and state gradients are not supported");
  const bool state = gqp || gq0;
  if (state) {
    if (!work) return fail(DDR_ERR_ARG, "state gradients need the workspace (ddr_state_work_bytes)");
    if (gq0 && !(flags & DDR_FWD_CARRY)) return fail(DDR_ERR_ARG, "grad_q0 needs a carried-state forward (DDR_FWD_CARRY)");
    if (gqp && qp_rows < (T + std::max<int64_t>(1, r->qprime_hours) - 1) / std::max<int64_t>(1, r->qprime_hours))
      return fail(DDR_ERR_ARG, "grad_qprime has fewer rows than the window reads");
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool cap = capturing(s);
  if (cap && g->split.nranks > 0) return fail(DDR_ERR_ARG, "stream capture: split-basin launches cannot be captured");
  if (!cap && (st = g_pending.check(false))) return st;
  if ((st = check_launchable<R>(g, true))) return st;
  DDR_TRY(ready_for(g, s));
  DDR_HIP(hipMemsetAsync(status, 0, kStatusBytes, s));
  if (g->n_cut > 0) DDR_HIP(hipMemsetAsync(bwd_bnd, 0xFF, sizeof(double) * 2 * g->n_cut * T, s));
  DDR_HIP(hipMemsetAsync(bwd_bnd + 2 * g->n_cut * T, 0, sizeof(double) * 3 * g->n, s));
  RouteArgs a;
  fill_common<R>(a, g, c, r, T, qprime, flags | g_debug);
  a.x_save = const_cast<R*>(x_save);
  a.qs = const_cast<R*>(x_save) + (g->n * T + g->sum_dn);
  a.bnd = const_cast<double*>(bnd);
  a.status = static_cast<unsigned*>(status);
  a.grad_out = grad;
  a.g_roff = gauges ? gauges->reach_offsets : nullptr;
  a.g_rg = gauges ? gauges->reach_gauges : nullptr;
  a.gseed = seed;
  a.bwd_bnd = bwd_bnd;
  a.gn = gn;
  a.gq = gq;
  a.gp = gp;
  // workspace: [2 n_cut T f64 boundary][3 N f64 accumulators]; the kernel reads grad (N, T) itself
  a.prof = g_prof[1];
  if (state) {
    a.gqs = work;
    a.gq0 = gq0;
    if (gauges && gauges->n_gauges > 0) {
      // the gauge sums' clamp at t = 0 (mmc.py:398-412) gates dL/dout[:, 0]
      GaugeArgs ga;
      if ((st = gauge_args<R>(gh, x_save, T, gauges, c->discharge_lb, flags, ga))) return st;
      unsigned char* mask = static_cast<unsigned char*>(work) + align16(sizeof(R) * (size_t)(g->n * T + g->sum_dn));
      DDR_HIP(launch_gauge_mask0<R>(ga, x_save, mask, s));
      a.gmask0 = mask;
    }
  }
  if ((st = split_prepare(g, a, T, 1, s))) return st;
  DDR_HIP(timing_mark(1, 0, s));
  DDR_HIP(launch_route<R>(g, a, true, s));
  DDR_HIP(timing_mark(1, 1, s));
  if (gqp) DDR_HIP(launch_scatter_qprime_grad<R>(g, a, qp_rows, gqp, s));
  return cap ? DDR_OK : g_pending.enqueue(status, s, "backward", gh);
}

template <typename R>
ddr_status gauge_args(const ddr_graph* gh, const R* x_save, int64_t T, const ddr_gauges* gz, double qlb,
                      int32_t flags, GaugeArgs& a) {
  if (!gh || !x_save || !gz || T < 1) return fail(DDR_ERR_ARG, "bad gauge arguments");
  if (gz->n_gauges > 0 && (!gz->offsets || !gz->index)) return fail(DDR_ERR_ARG, "null gauge arrays");
  const Graph* g = reinterpret_cast<const Graph*>(gh);
  if (!g->uploaded) return fail(DDR_ERR_ARG, "graph was built host-only: upload it first (ddr_graph_upload)");
  // a split rank holds the states of its own blocks only: a gauge sum would read rows no launch wrote
  if (g->split.nranks > 0) return fail(DDR_ERR_ARG, "split basin: gauge mode is not supported");
  std::memset(&a, 0, sizeof(a));
  a.s = g->dev;
  a.T = T;
  a.G = gz->n_gauges;
  a.goff = gz->offsets;
  a.gidx = gz->index;
  a.pos_of_ref = g->dev.pos_of_ref;
  a.block_of_pos = g->dev.block_of_pos;
  a.qlb = qlb;
  a.carry = (flags & DDR_FWD_CARRY) ? 1 : 0;
  return DDR_OK;
}

template <typename R>
ddr_status gauge_impl(const ddr_graph* gh, const R* x_save, int64_t T, const ddr_gauges* gz, double qlb,
                      int32_t flags, R* out, void* stream) {
  GaugeArgs a;
  ddr_status st = gauge_args<R>(gh, x_save, T, gz, qlb, flags, a);
  if (st) return st;
  if (!out) return fail(DDR_ERR_ARG, "null gauge output");
  DDR_TRY(ready_for(reinterpret_cast<const Graph*>(gh), static_cast<hipStream_t>(stream)));
  DDR_HIP(launch_gauge<R>(a, x_save, out, static_cast<hipStream_t>(stream)));
  return DDR_OK;
}

ddr_status check_window(int64_t T, int64_t t0, int64_t L, int64_t D) {
  if (t0 < 0 || L < 1 || t0 + L > T || D < 1 || D > L)
    return fail(DDR_ERR_ARG, "daily window must satisfy 0 <= t0, t0 + L <= T, 1 <= D <= L");
  return DDR_OK;
}

template <typename R>
ddr_status gauge_daily_impl(const ddr_graph* gh, const R* x_save, int64_t T, const ddr_gauges* gz, double qlb,
                            int32_t flags, int64_t t0, int64_t L, int64_t D, R* out, void* stream) {
  GaugeArgs a;
  ddr_status st = gauge_args<R>(gh, x_save, T, gz, qlb, flags, a);
  if (st) return st;
  if ((st = check_window(T, t0, L, D))) return st;
  if (!out) return fail(DDR_ERR_ARG, "null daily output");
  DDR_TRY(ready_for(reinterpret_cast<const Graph*>(gh), static_cast<hipStream_t>(stream)));
  DDR_HIP(launch_gauge_daily<R>(a, x_save, t0, L, D, out, static_cast<hipStream_t>(stream)));
  return DDR_OK;
}

template <typename R>
ddr_status gauge_daily_seed_impl(int64_t G, int64_t T, int64_t t0, int64_t L, int64_t D, const R* gd, R* gh,
                                 void* stream) {
  ddr_status st = check_window(T, t0, L, D);
  if (st) return st;
  if (G < 0 || (G > 0 && (!gd || !gh))) return fail(DDR_ERR_ARG, "bad daily seed arguments");
  DDR_HIP(launch_gauge_daily_seed<R>(G, T, t0, L, D, gd, gh, static_cast<hipStream_t>(stream)));
  return DDR_OK;
}

}  // namespace

#define DDR_GUARD(body)                                  \
  try {                                                  \
    body                                                 \
  } catch (const std::exception& ex) {                   \
    return fail(DDR_ERR_ARG, std::string("internal: ") + ex.what()); \
  } catch (...) {                                        \
    return fail(DDR_ERR_ARG, "internal error");          \
  }

ddr_status pnet_forward_impl(int64_t n_rows, int32_t n_features, const float* x, const float* params,
                             const float* denorm, float* z_save, float* u_save, float* out_n, float* out_q,
                             float* out_p, void* stream) {
  if (n_rows < 0 || n_features < 1 || n_features > 12) return fail(DDR_ERR_ARG, "pnet: 0 <= rows, 1 <= features <= 12");
  if (n_rows > 0 && (!x || !params || !denorm || !z_save || !u_save || !out_n || !out_q || !out_p))
    return fail(DDR_ERR_ARG, "pnet: null argument");
  if (n_rows >= (int64_t(1) << 31) / 64 * 64) return fail(DDR_ERR_ARG, "pnet: too many rows");
  float* out[3] = {out_n, out_q, out_p};
  DDR_HIP(launch_pnet_forward(n_rows, n_features, x, params, denorm, z_save, u_save, out, static_cast<hipStream_t>(stream)));
  return DDR_OK;
}
ddr_status pnet_backward_impl(int64_t n_rows, int32_t n_features, const float* x, const float* params,
                              const float* denorm, const float* z_save, const float* u_save, const float* grad_n,
                              const float* grad_q, const float* grad_p, float* grad_params, void* work, void* stream) {
  if (n_rows < 0 || n_features < 1 || n_features > 12) return fail(DDR_ERR_ARG, "pnet: 0 <= rows, 1 <= features <= 12");
  if (!grad_params || !params || !denorm) return fail(DDR_ERR_ARG, "pnet: null argument");
  if (n_rows > 0 && (!x || !z_save || !u_save || !grad_n || !grad_q || !grad_p || !work))
    return fail(DDR_ERR_ARG, "pnet: null argument");
  if (n_rows >= (int64_t(1) << 31) / 64 * 64) return fail(DDR_ERR_ARG, "pnet: too many rows");
  const float* g[3] = {grad_n, grad_q, grad_p};
  DDR_HIP(launch_pnet_backward(n_rows, n_features, x, params, denorm, z_save, u_save, g, grad_params, work,
                               static_cast<hipStream_t>(stream)));
  return DDR_OK;
}

ddr_status daily_l1_impl(int64_t n_gauges, int64_t n_days, int64_t warmup, const float* daily, const float* obs,
                         float inv_count, float* loss, float* grad, void* stream) {
  if (n_gauges < 0 || n_days < 0 || warmup < 0) return fail(DDR_ERR_ARG, "daily_l1: negative size");
  if (!loss || (n_gauges * n_days > 0 && (!daily || !obs))) return fail(DDR_ERR_ARG, "daily_l1: null argument");
  DDR_HIP(launch_daily_l1(n_gauges, n_days, warmup, daily, obs, inv_count, loss, grad, static_cast<hipStream_t>(stream)));
  return DDR_OK;
}
ddr_status clip_adam_impl(int64_t n, float* params, const float* grad, float* m, float* v, float lr, float beta1,
                          float beta2, float eps, float* step, float max_norm, float* norm_out, void* work,
                          void* stream) {
  if (n < 0) return fail(DDR_ERR_ARG, "clip_adam: negative size");
  if (n > 0 && (!params || !grad || !m || !v)) return fail(DDR_ERR_ARG, "clip_adam: null argument");
  if (!(beta1 >= 0.0f && beta1 < 1.0f) || !(beta2 >= 0.0f && beta2 < 1.0f)) return fail(DDR_ERR_ARG, "clip_adam: betas in [0, 1)");
  if (!step || !work) return fail(DDR_ERR_ARG, "clip_adam: null step counter or workspace (ddr_clip_adam_work_bytes)");
  DDR_HIP(launch_clip_adam(n, params, grad, m, v, lr, beta1, beta2, eps, step, max_norm, norm_out, work,
                           static_cast<hipStream_t>(stream)));
  return DDR_OK;
}

template <typename R>
ddr_status state_impl(const ddr_graph* gh, const R* x_save, int64_t T, int64_t t, double qlb, int32_t flags, R* out,
                      void* stream) {
  if (!gh || !x_save || !out) return fail(DDR_ERR_ARG, "null state argument");
  const Graph* g = reinterpret_cast<const Graph*>(gh);
  if (!g->uploaded) return fail(DDR_ERR_ARG, "graph was built host-only: upload it first (ddr_graph_upload)");
  if (T < 1 || t < 0 || t >= T) return fail(DDR_ERR_ARG, "state step out of [0, T)");
  // a split rank holds the states of its own blocks only
  if (g->split.nranks > 0) return fail(DDR_ERR_ARG, "split basin: the saved states are per rank");
  hipStream_t s = static_cast<hipStream_t>(stream);
  DDR_TRY(ready_for(g, s));
  DDR_HIP(launch_state_at<R>(g, T, t, qlb, (flags & DDR_FWD_CARRY) != 0, x_save, out, s));
  return DDR_OK;
}

extern "C" {

ddr_status ddr_graph_build(int64_t n, int64_t e, const int32_t* rows, const int32_t* cols, const ddr_build_opts* opts,
                           ddr_graph** out) {
  DDR_GUARD({
    if (!out) return fail(DDR_ERR_ARG, "null out");
    Graph* g = nullptr;
    ddr_status st = build_graph(n, e, rows, cols, opts, &g);
    if (st) return st;
    *out = reinterpret_cast<ddr_graph*>(g);
    return DDR_OK;
  })
}

ddr_status ddr_graph_build_device(int64_t n, int64_t e, const int32_t* rows, const int32_t* cols,
                                  const ddr_build_opts* opts, void* stream, ddr_graph** out) {
  DDR_GUARD({
    if (!out) return fail(DDR_ERR_ARG, "null out");
    Graph* g = nullptr;
    ddr_status st = build_graph_device(n, e, rows, cols, opts, static_cast<hipStream_t>(stream), &g);
    if (st) return st;
    *out = reinterpret_cast<ddr_graph*>(g);
    return DDR_OK;
  })
}

ddr_status ddr_graph_build_device_begin(int64_t n, int64_t e, const int32_t* rows, const int32_t* cols,
                                        const ddr_build_opts* opts, void* stream, ddr_graph_pending** out) {
  DDR_GUARD({
    if (!out) return fail(DDR_ERR_ARG, "null out");
    DevBuild* b = nullptr;
    ddr_status st = build_graph_device_begin(n, e, rows, cols, opts, static_cast<hipStream_t>(stream), &b);
    if (st) return st;
    *out = reinterpret_cast<ddr_graph_pending*>(b);
    return DDR_OK;
  })
}

ddr_status ddr_graph_build_device_finish(ddr_graph_pending* p, ddr_graph** out) {
  DDR_GUARD({
    if (!p) return fail(DDR_ERR_ARG, "null pending build");
    if (!out) {
      build_graph_device_cancel(reinterpret_cast<DevBuild*>(p));
      return fail(DDR_ERR_ARG, "null out");
    }
    Graph* g = nullptr;
    ddr_status st = build_graph_device_finish(reinterpret_cast<DevBuild*>(p), &g);
    if (st) return st;
    *out = reinterpret_cast<ddr_graph*>(g);
    return DDR_OK;
  })
}

ddr_status ddr_graph_build_device_cancel(ddr_graph_pending* p) {
  DDR_GUARD({
    build_graph_device_cancel(reinterpret_cast<DevBuild*>(p));
    return DDR_OK;
  })
}

ddr_status ddr_graph_fingerprint(const ddr_graph* gh, uint64_t* fp) {
  DDR_GUARD({
    if (!gh || !fp) return fail(DDR_ERR_ARG, "null argument");
    const Graph* g = reinterpret_cast<const Graph*>(gh);
    HostSchedule H;
    if (g->uploaded) {
      ddr_status st = device_schedule_to_host(g, H);
      if (st) return st;
    } else {
      H = g->hs;
    }
    unsigned long long h = schedule_fingerprint(H);
    auto mix = [&](const std::vector<int32_t>& v) {
      for (int32_t x : v) h = (h ^ (unsigned)x) * 1099511628211ull;
    };
    mix(H.pos_of_ref);
    mix(H.block_of_pos);
    mix(H.rs_loc);
    mix(H.rs_ref);
    for (const BlockDesc& B : g->blocks) {
      mix({B.pos0, B.nloc, B.virt0, B.nvirt, B.cout0, B.ncout, B.dmax, B.nxl, (int32_t)B.pre_dn,
           (int32_t)(B.pre_dn >> 32), B.xl0});
    }
    *fp = h;
    return DDR_OK;
  })
}

ddr_status ddr_collate_gauges(int64_t n_conus, int64_t n_gauges, const int64_t* sub_off, const int32_t* rows,
                              const int32_t* cols, const int32_t* gage_idx, int32_t* active, int64_t* n_active,
                              int64_t* crow, int32_t* col, int64_t* nnz, int64_t* out_off, int32_t* out_idx,
                              int64_t out_idx_cap, int32_t* gage_c) {
  DDR_GUARD({
    return collate_gauges(n_conus, n_gauges, sub_off, rows, cols, gage_idx, active, n_active, crow, col, nnz,
                          out_off, out_idx, out_idx_cap, gage_c);
  })
}

ddr_status ddr_collate_gauges_device(int64_t n_conus, int64_t n_gauges, int64_t e, const int32_t* rows,
                                     const int32_t* cols, const int32_t* gage_idx, int32_t* active, int64_t active_cap,
                                     int64_t* n_active, int32_t* rows_c, int32_t* cols_c, int64_t* nnz, int64_t* crow,
                                     int32_t* col, int64_t* out_off, int32_t* out_idx, int64_t out_idx_cap,
                                     int32_t* gage_c, void* stream) {
  DDR_GUARD({
    return collate_gauges_device(n_conus, n_gauges, e, rows, cols, gage_idx, active, active_cap, n_active, rows_c,
                                 cols_c, nnz, crow, col, out_off, out_idx, out_idx_cap, gage_c,
                                 static_cast<hipStream_t>(stream));
  })
}

ddr_status ddr_graph_upload(ddr_graph* g) {
  DDR_GUARD({
    if (!g) return fail(DDR_ERR_ARG, "null graph");
    return upload_schedule(reinterpret_cast<Graph*>(g));
  })
}

ddr_status ddr_graph_upload_async(ddr_graph* g, void* stream) {
  DDR_GUARD({
    if (!g) return fail(DDR_ERR_ARG, "null graph");
    return upload_schedule_async(reinterpret_cast<Graph*>(g), static_cast<hipStream_t>(stream));
  })
}

ddr_status ddr_graph_build_async(int64_t n, int64_t e, const int32_t* rows, const int32_t* cols,
                                 const ddr_build_opts* opts, void* stream, ddr_graph** out) {
  DDR_GUARD({
    if (!out) return fail(DDR_ERR_ARG, "null out");
    ddr_build_opts o;
    std::memset(&o, 0, sizeof(o));
    if (opts) o = *opts;
    const bool host_only = o.flags & DDR_BUILD_HOST_ONLY;
    o.flags |= DDR_BUILD_HOST_ONLY;
    Graph* g = nullptr;
    ddr_status st = build_graph(n, e, rows, cols, &o, &g);
    if (st) return st;
    if (!host_only && (st = upload_schedule_async(g, static_cast<hipStream_t>(stream)))) {
      destroy_graph(g);
      return st;
    }
    *out = reinterpret_cast<ddr_graph*>(g);
    return DDR_OK;
  })
}

ddr_status ddr_graph_destroy(ddr_graph* g) {
  DDR_GUARD({
    Graph* gr = reinterpret_cast<Graph*>(g);
    if (!gr) return DDR_OK;
    // on the graph's own device (the caller may have another one current): its sync, and the null stream
    // the pool-release events are recorded on
    DeviceGuard dg(gr->device);
    if (dg.error != hipSuccess) return fail(DDR_ERR_HIP, hipGetErrorString(dg.error));
    // synchronous, as the header promises: the pooled blocks of a device-built graph go back to the pool
    // only once no launch on any stream can still read them (their release event is recorded on the null
    // stream, which does not order PyTorch's non-blocking streams)
    if (gr->device_built || !gr->async_allocations.empty()) DDR_HIP(hipDeviceSynchronize());
    destroy_graph(gr);
    return DDR_OK;
  })
}

ddr_status ddr_qprime_nan_wait(int32_t* has_nan) {
  DDR_GUARD({
    if (!has_nan) return fail(DDR_ERR_ARG, "null has_nan");
    if (t_nan_dev < 0 || !t_nan[t_nan_dev].armed) return fail(DDR_ERR_ARG, "no DDR_FWD_CHECK_QPRIME forward on this thread");
    NanCheck& c = t_nan[t_nan_dev];
    DDR_HIP(hipEventSynchronize(c.ev));
    *has_nan = *c.host ? 1 : 0;
    c.armed = false;
    return DDR_OK;
  })
}

ddr_status ddr_pool_trim(int64_t* freed_bytes) {
  DDR_GUARD({
    const int64_t f = pool_trim();
    if (freed_bytes) *freed_bytes = f;
    return DDR_OK;
  })
}

ddr_status ddr_graph_destroy_async(ddr_graph* g, void* stream) {
  DDR_GUARD({
    destroy_graph(reinterpret_cast<Graph*>(g), static_cast<hipStream_t>(stream));
    return DDR_OK;
  })
}

ddr_status ddr_xmem_alloc(int64_t bytes, void** ptr, void* handle, int32_t* kind) {
  DDR_GUARD({
    if (bytes <= 0 || !ptr || !handle) return fail(DDR_ERR_ARG, "bad ddr_xmem_alloc arguments");
    // uncached device memory (no stale L2 copy of a peer's stores); fine-grained, then plain device
    // memory where the uncached kind cannot be exported
    for (int k = 0; k < 3; ++k) {
      const unsigned flag = k == 0 ? hipDeviceMallocUncached : (k == 1 ? hipDeviceMallocFinegrained : hipDeviceMallocDefault);
      void* p = nullptr;
      if (hipExtMallocWithFlags(&p, (size_t)bytes, flag) != hipSuccess) {
        (void)hipGetLastError();
        continue;
      }
      hipIpcMemHandle_t h;
      if (hipIpcGetMemHandle(&h, p) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipFree(p);
        continue;
      }
      DDR_HIP(hipMemset(p, 0, (size_t)bytes));
      std::memcpy(handle, &h, sizeof(h));
      *ptr = p;
      if (kind) *kind = k;
      return DDR_OK;
    }
    return fail(DDR_ERR_HIP, "ddr_xmem_alloc: no exportable device allocation");
  })
}

ddr_status ddr_xmem_open(const void* handle, void** ptr) {
  DDR_GUARD({
    if (!handle || !ptr) return fail(DDR_ERR_ARG, "null argument");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle, sizeof(h));
    DDR_HIP(hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess));
    return DDR_OK;
  })
}

ddr_status ddr_xmem_close(void* ptr, int32_t opened) {
  DDR_GUARD({
    if (!ptr) return DDR_OK;
    DDR_HIP(opened ? hipIpcCloseMemHandle(ptr) : hipFree(ptr));
    return DDR_OK;
  })
}

ddr_status ddr_xmem_bytes(int64_t n_x, int64_t T, int64_t* bytes) {
  if (n_x < 0 || T < 1 || !bytes) return fail(DDR_ERR_ARG, "bad ddr_xmem_bytes arguments");
  *bytes = (int64_t)xmem_bytes(n_x, T);
  return DDR_OK;
}

ddr_status ddr_graph_blocks(const ddr_graph* gh, int32_t* nloc, int64_t cap) {
  if (!gh || !nloc) return fail(DDR_ERR_ARG, "null argument");
  const Graph* g = reinterpret_cast<const Graph*>(gh);
  if (cap < (int64_t)g->blocks.size()) return fail(DDR_ERR_ARG, "ddr_graph_blocks: capacity below n_blocks");
  for (size_t b = 0; b < g->blocks.size(); ++b) nloc[b] = g->blocks[b].nloc;
  return DDR_OK;
}

ddr_status ddr_graph_cut_blocks(const ddr_graph* gh, int32_t* prod, int32_t* cons, int64_t cap) {
  DDR_GUARD({
    if (!gh || !prod || !cons) return fail(DDR_ERR_ARG, "null argument");
    const Graph* g = reinterpret_cast<const Graph*>(gh);
    if (cap < g->n_cut) return fail(DDR_ERR_ARG, "ddr_graph_cut_blocks: capacity below n_cut");
    HostSchedule H;
    if (g->uploaded) {
      ddr_status st = device_schedule_to_host(g, H);
      if (st) return st;
    } else {
      H = g->hs;
    }
    for (int64_t e = 0; e < g->n_cut; ++e) prod[e] = cons[e] = -1;
    for (size_t b = 0; b < g->blocks.size(); ++b) {
      const BlockDesc& B = g->blocks[b];
      for (int i = 0; i < B.nloc; ++i) {
        const int32_t e = H.cut[B.pos0 + i];
        if (e >= 0) prod[e] = (int32_t)b;
      }
      for (int v = 0; v < B.nvirt; ++v) cons[H.v_edge[B.virt0 + v]] = (int32_t)b;
    }
    return DDR_OK;
  })
}

ddr_status ddr_graph_set_split(ddr_graph* gh, int32_t rank, int32_t nranks, const int32_t* block_rank, void* local,
                               void* const* peers, int64_t t_cap, int64_t* n_x_out) {
  DDR_GUARD({
    if (!gh || !block_rank || !local || !peers || t_cap < 1) return fail(DDR_ERR_ARG, "bad ddr_graph_set_split arguments");
    if (nranks < 2 || nranks > kMaxSplitRanks || rank < 0 || rank >= nranks)
      return fail(DDR_ERR_ARG, "split basin: 2 <= nranks <= 16, 0 <= rank < nranks");
    Graph* g = reinterpret_cast<Graph*>(gh);
    if (!g->uploaded) return fail(DDR_ERR_ARG, "graph was built host-only: upload it first (ddr_graph_upload)");
    if (g->split.nranks > 0) return fail(DDR_ERR_ARG, "split basin: already set");
    const int64_t nb = (int64_t)g->blocks.size();
    for (int64_t b = 0; b < nb; ++b)
      if (block_rank[b] < 0 || block_rank[b] >= nranks) return fail(DDR_ERR_ARG, "split basin: block rank out of range");
    std::vector<int32_t> prod((size_t)g->n_cut);
    std::vector<int32_t> cons((size_t)g->n_cut);
    ddr_status st = ddr_graph_cut_blocks(gh, prod.data(), cons.data(), g->n_cut);
    if (st) return st;
    std::vector<int32_t> xid((size_t)g->n_cut);
    std::fill(xid.begin(), xid.end(), -1);
    std::vector<int32_t> xcons;
    std::vector<int32_t> xprod;
    std::vector<int64_t> xedge;
    for (int64_t e = 0; e < g->n_cut; ++e) {
      if (prod[e] < 0 || cons[e] < 0) return fail(DDR_ERR_ARG, "split basin: cut edge without both blocks");
      if (block_rank[prod[e]] != block_rank[cons[e]]) {
        xid[e] = (int32_t)xcons.size();
        xcons.push_back(block_rank[cons[e]]);
        xprod.push_back(block_rank[prod[e]]);
        xedge.push_back(e);
      }
    }
    std::vector<uint8_t> owned(nb);
    for (int64_t b = 0; b < nb; ++b) owned[b] = block_rank[b] == rank ? 1 : 0;
    auto up = [&](const void* src, size_t bytes, void** dst) -> hipError_t {
      hipError_t e = hipMalloc(dst, bytes < 16 ? 16 : bytes);
      if (e != hipSuccess) return e;
      g->allocations.push_back(*dst);
      return bytes ? hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice) : hipSuccess;
    };
    SplitState sp;
    DDR_HIP(up(owned.data(), owned.size(), reinterpret_cast<void**>(&sp.owned)));
    DDR_HIP(up(xid.data(), xid.size() * 4, reinterpret_cast<void**>(&sp.xid)));
    DDR_HIP(up(xcons.data(), xcons.size() * 4, reinterpret_cast<void**>(&sp.xcons)));
    DDR_HIP(up(xprod.data(), xprod.size() * 4, reinterpret_cast<void**>(&sp.xprod)));
    DDR_HIP(up(xedge.data(), xedge.size() * 8, reinterpret_cast<void**>(&sp.xedge)));
    sp.rank = rank;
    sp.nranks = nranks;
    sp.n_x = (int32_t)xcons.size();
    sp.t_cap = t_cap;
    sp.local = static_cast<char*>(local);
    for (int p = 0; p < nranks; ++p) sp.peers[p] = static_cast<char*>(peers[p]);
    g->split = sp;
    if (n_x_out) *n_x_out = sp.n_x;
    return DDR_OK;
  })
}

ddr_status ddr_graph_clear_split(ddr_graph* gh) {
  if (!gh) return fail(DDR_ERR_ARG, "null graph");
  Graph* g = reinterpret_cast<Graph*>(gh);
  // the device arrays stay with the graph (freed at destroy); the receive memory is the caller's
  const SplitState none;
  g->split = none;
  return DDR_OK;
}

ddr_status ddr_graph_get_info(const ddr_graph* gh, ddr_graph_info* info) {
  if (!gh || !info) return fail(DDR_ERR_ARG, "null argument");
  const Graph* g = reinterpret_cast<const Graph*>(gh);
  info->n = g->n;
  info->nnz = g->nnz;
  info->n_basins = g->n_basins;
  info->n_pieces = g->n_pieces;
  info->n_blocks = (int64_t)g->blocks.size();
  info->n_cut = g->n_cut;
  info->max_depth = g->max_depth;
  info->max_block_depth = g->max_block_depth;
  info->reaches_per_thread = g->kr;
  info->save_elems_per_t = 2 * g->n;  // x (routing states) | q' gathered into the same layout
  info->save_elems_fixed = 2 * g->sum_dn;
  info->bnd_elems_per_t = g->n_cut;
  info->bwd_elems_per_t = 2 * g->n_cut;
  info->bwd_elems_fixed = 3 * g->n;
  info->generations = g->generations;
  info->status_bytes = kStatusBytes;
  return DDR_OK;
}

ddr_status ddr_graph_csr(const ddr_graph* gh, int64_t* crow, int64_t* col) {
  if (!gh || !crow || (!col && reinterpret_cast<const Graph*>(gh)->nnz > 0)) return fail(DDR_ERR_ARG, "null argument");
  const Graph* g = reinterpret_cast<const Graph*>(gh);
  if (g->device_built) DDR_GUARD({ return device_views_to_host(g, crow, col, nullptr, nullptr, nullptr, nullptr); })
  std::memcpy(crow, g->crow.data(), sizeof(int64_t) * (g->n + 1));
  if (g->nnz) std::memcpy(col, g->col.data(), sizeof(int64_t) * g->nnz);
  return DDR_OK;
}

ddr_status ddr_graph_structure(const ddr_graph* gh, int64_t* down, int64_t* dist, int64_t* basin, int64_t* block) {
  if (!gh) return fail(DDR_ERR_ARG, "null graph");
  const Graph* g = reinterpret_cast<const Graph*>(gh);
  if (g->device_built) DDR_GUARD({ return device_views_to_host(g, nullptr, nullptr, down, dist, basin, block); })
  const size_t b = sizeof(int64_t) * g->n;
  if (down) std::memcpy(down, g->down.data(), b);
  if (dist) std::memcpy(dist, g->dist.data(), b);
  if (basin) std::memcpy(basin, g->basin.data(), b);
  if (block) std::memcpy(block, g->block_of.data(), b);
  return DDR_OK;
}

ddr_status ddr_mc_forward_f32(const ddr_graph* g, const ddr_mc_consts* c, const ddr_mc_reaches* r,
                              const float* qprime, int64_t T, const float* q0, float* runoff, float* x_save,
                              double* bnd, void* status, float* q_last, float* tw, float* ss, int32_t flags,
                              void* stream) {
  DDR_GUARD({ return forward_impl<float>(g, c, r, qprime, T, q0, runoff, x_save, bnd, status, q_last, tw, ss, flags, stream); })
}
ddr_status ddr_mc_forward_f64(const ddr_graph* g, const ddr_mc_consts* c, const ddr_mc_reaches* r,
                              const double* qprime, int64_t T, const double* q0, double* runoff, double* x_save,
                              double* bnd, void* status, double* q_last, double* tw, double* ss, int32_t flags,
                              void* stream) {
  DDR_GUARD({ return forward_impl<double>(g, c, r, qprime, T, q0, runoff, x_save, bnd, status, q_last, tw, ss, flags, stream); })
}
ddr_status ddr_mc_backward_f32(const ddr_graph* g, const ddr_mc_consts* c, const ddr_mc_reaches* r,
                               const float* qprime, int64_t T, const float* x_save, const double* bnd,
                               const float* grad, const ddr_gauges* gauges, double* bwd_bnd, void* status,
                               float* gn, float* gq, float* gp, int32_t flags, void* stream) {
  DDR_GUARD({ return backward_impl<float>(g, c, r, qprime, T, x_save, bnd, grad, gauges, bwd_bnd, status, gn, gq, gp, flags, stream); })
}
ddr_status ddr_mc_backward_f64(const ddr_graph* g, const ddr_mc_consts* c, const ddr_mc_reaches* r,
                               const double* qprime, int64_t T, const double* x_save, const double* bnd,
                               const double* grad, const ddr_gauges* gauges, double* bwd_bnd, void* status,
                               double* gn, double* gq, double* gp, int32_t flags, void* stream) {
  DDR_GUARD({ return backward_impl<double>(g, c, r, qprime, T, x_save, bnd, grad, gauges, bwd_bnd, status, gn, gq, gp, flags, stream); })
}
ddr_status ddr_hotstart_f32(const ddr_graph* gh, const float* q, double discharge_lb, float* out, void* stream) {
  DDR_GUARD({
    if (!gh || !q || !out) return fail(DDR_ERR_ARG, "null hot-start argument");
    const Graph* g = reinterpret_cast<const Graph*>(gh);
    if (!g->uploaded) return fail(DDR_ERR_ARG, "graph was built host-only: upload it first (ddr_graph_upload)");
    hipStream_t s = static_cast<hipStream_t>(stream);
    // one forward step in accumulation mode (every step a hot start, no coefficient physics): its
    // workspace is stream-ordered scratch; the per-reach statics are never read for their values
    const size_t xs = sizeof(float) * 2 * (size_t)(g->n + g->sum_dn);
    void* ws = device_get(xs + sizeof(double) * (size_t)std::max<int64_t>(g->n_cut, 1) + kStatusBytes, s);
    if (!ws) return fail(DDR_ERR_HIP, "hot start: out of device memory");
    ddr_mc_consts c;
    c.dt = 3600.0;
    c.discharge_lb = discharge_lb;
    c.velocity_lb = 0.01;
    c.velocity_ub = 15.0;
    c.depth_lb = 0.01;
    c.bottom_width_lb = 0.01;
    c.side_slope_lb = 0.5;
    c.side_slope_ub = 50.0;
    ddr_mc_reaches r{};
    r.n = r.q_spatial = r.p_spatial = r.length = r.slope = r.x_storage = q;
    r.p_stride = 1;
    unsigned char* base = static_cast<unsigned char*>(ws);
    ddr_status st = forward_impl<float>(gh, &c, &r, q, 1, nullptr, out, reinterpret_cast<float*>(base),
                                        reinterpret_cast<double*>(base + xs), base + xs + sizeof(double) * std::max<int64_t>(g->n_cut, 1),
                                        nullptr, nullptr, nullptr, DDR_FWD_ACCUMULATE, stream);
    device_put(ws, s);
    return st;
  })
}

int64_t ddr_state_work_bytes(const ddr_graph* g, int64_t T, int64_t n_gauges, int32_t real_bytes) {
  if (!g || T < 1 || n_gauges < 0 || (real_bytes != 4 && real_bytes != 8)) return -1;
  return state_work_bytes(reinterpret_cast<const Graph*>(g), T, n_gauges, (size_t)real_bytes);
}
ddr_status ddr_mc_backward_state_f32(const ddr_graph* g, const ddr_mc_consts* c, const ddr_mc_reaches* r,
                                     const float* qprime, int64_t qprime_rows, int64_t T, const float* x_save,
                                     const double* bnd, const float* grad, const ddr_gauges* gauges, double* bwd_bnd,
                                     void* status, float* gn, float* gq, float* gp, float* grad_qprime,
                                     float* grad_q0, void* work, int32_t flags, void* stream) {
  DDR_GUARD({ return backward_impl<float>(g, c, r, qprime, T, x_save, bnd, grad, gauges, bwd_bnd, status, gn, gq, gp, flags, stream, qprime_rows, grad_qprime, grad_q0, work); })
}
ddr_status ddr_mc_backward_state_f64(const ddr_graph* g, const ddr_mc_consts* c, const ddr_mc_reaches* r,
                                     const double* qprime, int64_t qprime_rows, int64_t T, const double* x_save,
                                     const double* bnd, const double* grad, const ddr_gauges* gauges, double* bwd_bnd,
                                     void* status, double* gn, double* gq, double* gp, double* grad_qprime,
                                     double* grad_q0, void* work, int32_t flags, void* stream) {
  DDR_GUARD({ return backward_impl<double>(g, c, r, qprime, T, x_save, bnd, grad, gauges, bwd_bnd, status, gn, gq, gp, flags, stream, qprime_rows, grad_qprime, grad_q0, work); })
}
ddr_status ddr_mc_backward_ex_f32(const ddr_graph* g, const ddr_mc_consts* c, const ddr_mc_reaches* r,
                                  const float* qprime, int64_t qprime_rows, int64_t T, const float* x_save,
                                  const double* bnd, const float* grad, const ddr_gauges* gauges,
                                  const float* state_seed, double* bwd_bnd, void* status, float* gn, float* gq,
                                  float* gp, float* grad_qprime, float* grad_q0, void* work, int32_t flags,
                                  void* stream) {
  DDR_GUARD({ return backward_impl<float>(g, c, r, qprime, T, x_save, bnd, grad, gauges, bwd_bnd, status, gn, gq, gp, flags, stream, qprime_rows, grad_qprime, grad_q0, work, state_seed); })
}
ddr_status ddr_mc_backward_ex_f64(const ddr_graph* g, const ddr_mc_consts* c, const ddr_mc_reaches* r,
                                  const double* qprime, int64_t qprime_rows, int64_t T, const double* x_save,
                                  const double* bnd, const double* grad, const ddr_gauges* gauges,
                                  const double* state_seed, double* bwd_bnd, void* status, double* gn, double* gq,
                                  double* gp, double* grad_qprime, double* grad_q0, void* work, int32_t flags,
                                  void* stream) {
  DDR_GUARD({ return backward_impl<double>(g, c, r, qprime, T, x_save, bnd, grad, gauges, bwd_bnd, status, gn, gq, gp, flags, stream, qprime_rows, grad_qprime, grad_q0, work, state_seed); })
}

int64_t ddr_pnet_param_count(int32_t n_features) {
  if (n_features < 1 || n_features > 12) return -1;
  return pnet_param_count(n_features);
}
int64_t ddr_pnet_work_bytes(int64_t n_rows, int32_t n_features) {
  if (n_rows < 0 || n_features < 1 || n_features > 12) return -1;
  return pnet_work_bytes(n_rows, n_features);
}
ddr_status ddr_pnet_forward_f32(int64_t n_rows, int32_t n_features, const float* x, const float* params,
                                const float* denorm, float* z_save, float* u_save, float* out_n, float* out_q,
                                float* out_p, void* stream) {
  DDR_GUARD({ return pnet_forward_impl(n_rows, n_features, x, params, denorm, z_save, u_save, out_n, out_q, out_p, stream); })
}
ddr_status ddr_pnet_backward_f32(int64_t n_rows, int32_t n_features, const float* x, const float* params,
                                 const float* denorm, const float* z_save, const float* u_save, const float* grad_n,
                                 const float* grad_q, const float* grad_p, float* grad_params, void* work,
                                 void* stream) {
  DDR_GUARD({ return pnet_backward_impl(n_rows, n_features, x, params, denorm, z_save, u_save, grad_n, grad_q, grad_p, grad_params, work, stream); })
}
ddr_status ddr_daily_l1_f32(int64_t n_gauges, int64_t n_days, int64_t warmup, const float* daily, const float* obs,
                            float inv_count, float* loss, float* grad, void* stream) {
  DDR_GUARD({ return daily_l1_impl(n_gauges, n_days, warmup, daily, obs, inv_count, loss, grad, stream); })
}
int64_t ddr_clip_adam_work_bytes(void) { return (int64_t)clip_adam_work_bytes(); }
ddr_status ddr_clip_adam_f32(int64_t n, float* params, const float* grad, float* m, float* v, float lr, float beta1,
                             float beta2, float eps, float* step, float max_norm, float* norm_out, void* work,
                             void* stream) {
  DDR_GUARD({ return clip_adam_impl(n, params, grad, m, v, lr, beta1, beta2, eps, step, max_norm, norm_out, work, stream); })
}
ddr_status ddr_state_f32(const ddr_graph* g, const float* x_save, int64_t T, int64_t t, double discharge_lb,
                         int32_t flags, float* out, void* stream) {
  DDR_GUARD({ return state_impl<float>(g, x_save, T, t, discharge_lb, flags, out, stream); })
}
ddr_status ddr_state_f64(const ddr_graph* g, const double* x_save, int64_t T, int64_t t, double discharge_lb,
                         int32_t flags, double* out, void* stream) {
  DDR_GUARD({ return state_impl<double>(g, x_save, T, t, discharge_lb, flags, out, stream); })
}
ddr_status ddr_gauge_reduce_f32(const ddr_graph* g, const float* x_save, int64_t T, const ddr_gauges* gz,
                                double qlb, int32_t flags, float* out, void* stream) {
  DDR_GUARD({ return gauge_impl<float>(g, x_save, T, gz, qlb, flags, out, stream); })
}
ddr_status ddr_gauge_reduce_f64(const ddr_graph* g, const double* x_save, int64_t T, const ddr_gauges* gz,
                                double qlb, int32_t flags, double* out, void* stream) {
  DDR_GUARD({ return gauge_impl<double>(g, x_save, T, gz, qlb, flags, out, stream); })
}

ddr_status ddr_gauge_daily_f32(const ddr_graph* g, const float* x_save, int64_t T, const ddr_gauges* gz,
                               double qlb, int32_t flags, int64_t t0, int64_t L, int64_t D, float* out,
                               void* stream) {
  DDR_GUARD({ return gauge_daily_impl<float>(g, x_save, T, gz, qlb, flags, t0, L, D, out, stream); })
}
ddr_status ddr_gauge_daily_f64(const ddr_graph* g, const double* x_save, int64_t T, const ddr_gauges* gz,
                               double qlb, int32_t flags, int64_t t0, int64_t L, int64_t D, double* out,
                               void* stream) {
  DDR_GUARD({ return gauge_daily_impl<double>(g, x_save, T, gz, qlb, flags, t0, L, D, out, stream); })
}
ddr_status ddr_gauge_daily_seed_f32(int64_t G, int64_t T, int64_t t0, int64_t L, int64_t D, const float* grad_daily,
                                    float* grad_hourly, void* stream) {
  DDR_GUARD({ return gauge_daily_seed_impl<float>(G, T, t0, L, D, grad_daily, grad_hourly, stream); })
}
ddr_status ddr_gauge_daily_seed_f64(int64_t G, int64_t T, int64_t t0, int64_t L, int64_t D, const double* grad_daily,
                                    double* grad_hourly, void* stream) {
  DDR_GUARD({ return gauge_daily_seed_impl<double>(G, T, t0, L, D, grad_daily, grad_hourly, stream); })
}

ddr_status ddr_geometry_stats_f32(const float* q_daily, int64_t reach_stride, int64_t day_stride, int64_t n,
                                  int64_t days, const float* n_manning, const float* p_spatial, int64_t p_stride,
                                  const float* q_spatial, const float* slope, double depth_lb,
                                  double bottom_width_lb, float* out, void* stream) {
  DDR_GUARD({
    // the long-window kernel sorts one variable of a reach in LDS: 4 B per day, the next power of two
    if (n < 0 || days < 1 || days > kGeoLongMaxDays)
      return fail(DDR_ERR_ARG, "geometry statistics: need 1 <= days <= " + std::to_string(kGeoLongMaxDays));
    if (n > 0 && (!q_daily || !n_manning || !p_spatial || !q_spatial || !slope || !out))
      return fail(DDR_ERR_ARG, "null geometry statistics argument");
    if (p_stride != 0 && p_stride != 1) return fail(DDR_ERR_ARG, "p_stride must be 0 or 1");
    DDR_HIP(launch_geometry_stats(q_daily, reach_stride, day_stride, n, days, n_manning, p_spatial, p_stride,
                                  q_spatial, slope, (float)depth_lb, (float)bottom_width_lb, out,
                                  static_cast<hipStream_t>(stream)));
    return DDR_OK;
  })
}

ddr_status ddr_graph_status(const void* status, void* stream) {
  if (!status) return fail(DDR_ERR_ARG, "null status");
  unsigned h[2] = {0, 0};
  DDR_HIP(hipMemcpyAsync(h, status, sizeof(h), hipMemcpyDeviceToHost, static_cast<hipStream_t>(stream)));
  DDR_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
  if (h[0]) return fail(DDR_ERR_TIMEOUT, std::to_string(h[0]) + " inter-workgroup hand-offs timed out (first block " +
                                             std::to_string((int)h[1] - 1) + ")");
  return DDR_OK;
}

ddr_status ddr_status_check(int32_t wait) {
  DDR_GUARD({ return g_pending.check(wait != 0); })
}

ddr_status ddr_set_debug_flags(int32_t flags) {
  g_debug = ((flags & DDR_DEBUG_FORCE_TIMEOUT) ? kFlagForceTimeout : 0) | ((flags & DDR_DEBUG_NO_STEADY) ? kFlagNoSteady : 0) |
            ((flags & DDR_DEBUG_NO_STORER) ? kFlagNoStorer : 0) | ((flags & DDR_DEBUG_NO_PLAIN) ? kFlagNoPlain : 0);
  return DDR_OK;
}

ddr_status ddr_set_kernel_timing(int32_t enable) {
  g_timing.on = enable != 0;
  return DDR_OK;
}

ddr_status ddr_kernel_ms(int32_t which, float* ms) {
  if ((which != 0 && which != 1) || !ms) return fail(DDR_ERR_ARG, "bad ddr_kernel_ms arguments");
  if (!g_timing.recorded[which]) return fail(DDR_ERR_ARG, "no timed launch recorded");
  DDR_HIP(hipEventSynchronize(g_timing.ev[which][1]));
  DDR_HIP(hipEventElapsedTime(ms, g_timing.ev[which][0], g_timing.ev[which][1]));
  return DDR_OK;
}

ddr_status ddr_set_block_profile(int32_t which, uint64_t* buf) {
  if (which != 0 && which != 1) return fail(DDR_ERR_ARG, "which must be 0 or 1");
  g_prof[which] = reinterpret_cast<unsigned long long*>(buf);
  return DDR_OK;
}

ddr_status ddr_device_info(int32_t* n_cu, int32_t* max_resident) {
  int dev = 0;
  DDR_HIP(hipGetDevice(&dev));
  hipDeviceProp_t prop;
  DDR_HIP(hipGetDeviceProperties(&prop, dev));
  if (n_cu) *n_cu = prop.multiProcessorCount;
  if (max_resident) *max_resident = prop.multiProcessorCount;
  return DDR_OK;
}

const char* ddr_last_error(void) { return ddr::last_error_cstr(); }
#ifndef DDR_SOURCE_HASH
#define DDR_SOURCE_HASH "unknown"
#endif
// src: every library source; kern: the routing kernels' sources only (route.hip and the headers it
// includes) -- the key of the PMC counter files under profiles/counters (bench.py), which describe the
// kernels and stay valid across host-side changes.  The kernel hash is the last word.
#ifndef DDR_KERNEL_HASH
#define DDR_KERNEL_HASH "unknown"
#endif
const char* ddr_version(void) { return "ddr_mc 0.2.0 (gfx950) src " DDR_SOURCE_HASH " kern " DDR_KERNEL_HASH; }

}  // extern "C"
