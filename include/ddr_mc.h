/*
 * ddr_mc.h -- C ABI of the MI355X-native Muskingum-Cunge routing hot path (libddr_mc.so).
 *
 * This is the drop-in boundary for DDR's routing engine (taddyb/ddr, src/ddr/routing).  Every entry
 * point takes plain pointers and sizes; device pointers are caller-allocated (e.g. by the PyTorch
 * caching allocator) and never freed by the library.  All work is enqueued on the caller's stream.
 * No C++ exception crosses this boundary: every call returns a ddr_status (0 = OK, < 0 = error)
 * and ddr_last_error() returns a thread-local message.
 *
 * Reference interfaces each entry point replaces (file:line in /root/reference):
 *   ddr_graph_build     src/ddr/geodatazoo/merit.py:197-223 (COO union -> scipy .tocsr())
 *                       + src/ddr/routing/utils.py:25-163 (PatternMapper / get_network_idx)
 *   ddr_graph_upload    (host build on a loader thread, then upload: the per-batch graph of training)
 *   ddr_graph_build_device  the same build on the device from a device-resident COO (merit.py:197-223,
 *                       builders.py:55-109 per training batch; north star (1))
 *   ddr_graph_csr       scipy.sparse.coo_matrix(...).tocsr() canonical CSR (bit-exact target)
 *   ddr_collate_gauges  src/ddr/io/builders.py:55-109 construct_network_matrix + merit.py:197-238
 *                       (per-batch gauge union, compression, outflow_idx); _device: the same on the device
 *   ddr_mc_forward      src/ddr/routing/mmc.py:365-443 (MuskingumCunge.forward) with
 *                       mmc.py:487-559 (route_timestep), mmc.py:25-66 (compute_hotstart_discharge),
 *                       mmc.py:102-168 + geometry/trapezoidal.py:14-108 (celerity),
 *                       mmc.py:460-485 (coefficients), routing/utils.py:535-627 (solver forward)
 *   ddr_mc_backward     torch autograd of the above + routing/utils.py:629-692 (solver backward,
 *                       _backward_cpu 188-242 / _backward_gpu 245-310, _compute_A_gradients 321-389)
 *   ddr_hotstart_f32    mmc.py:25-66 (compute_hotstart_discharge)
 *   ddr_gauge_reduce    mmc.py:344-363, 405-411, 433-439 (ragged outflow_idx scatter_add)
 *   ddr_tri_solve       routing/utils.py:695 triangular_sparse_solve (general CSR, non-unit diagonal)
 *   ddr_tri_grad_values routing/utils.py:321-389 _compute_A_gradients (gradA = -gradb[row]*x[col])
 */
#ifndef DDR_MC_H
#define DDR_MC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int ddr_status;
enum {
  DDR_OK = 0,
  DDR_ERR_ARG = -1,           /* bad argument / shape                                  */
  DDR_ERR_NOT_LOWER = -2,     /* adjacency not strictly lower triangular (unsorted)     */
  DDR_ERR_NOT_DENDRITIC = -3, /* a reach drains into more than one downstream reach     */
  DDR_ERR_DUPLICATE = -4,     /* duplicate edge (summed value != 1)                     */
  DDR_ERR_HIP = -5,           /* HIP runtime error                                      */
  DDR_ERR_CAPACITY = -6,      /* graph does not fit the co-resident grid of this device */
  DDR_ERR_TIMEOUT = -7,       /* an inter-workgroup hand-off timed out (device status)  */
  DDR_ERR_SINGULAR = -8       /* zero on the diagonal (ddr_tri_solve)                   */
};

/* Opaque river-graph handle: canonical CSR, dendritic down[] pointers, basin/piece partition and the
 * per-workgroup schedule, uploaded to the current device.  Immutable after build: safe to share
 * across host threads and streams on its device. */
typedef struct ddr_graph ddr_graph;

enum { DDR_BUILD_HOST_ONLY = 1 };

typedef struct {
  int32_t flags;              /* DDR_BUILD_HOST_ONLY: validate/partition, no upload  [in]  */
  int32_t max_block_reaches;  /* cap on reaches per workgroup (0 = auto)             [in]  */
  int32_t target_blocks;      /* desired workgroups (0 = auto: CU count)             [in]  */
  int32_t max_resident;       /* co-resident workgroups of the device (0 = query)    [in]  */
  int32_t steps_hint;         /* expected timesteps per launch, for load balancing   [in]  */
                              /* (0 = 8760; any T is correct, this only weighs work)       */
} ddr_build_opts;

typedef struct {
  int64_t n;              /* reaches                                                      */
  int64_t nnz;            /* edges after canonicalisation                                  */
  int64_t n_basins;       /* connected components (outlet basins)                          */
  int64_t n_pieces;       /* schedulable pieces after splitting large basins               */
  int64_t n_blocks;       /* workgroups of one routing launch                              */
  int64_t n_cut;          /* inter-workgroup edges                                         */
  int64_t max_depth;      /* longest reach-to-outlet path (hops + 1)                       */
  int64_t max_block_depth;/* max over workgroups of the in-piece depth                    */
  int64_t reaches_per_thread; /* KR of the routing kernel instantiation                   */
  int64_t save_elems_per_t;   /* x_save elements = save_elems_per_t * T + save_elems_fixed  */
  int64_t save_elems_fixed;
  int64_t bnd_elems_per_t;    /* forward boundary buffer doubles = bnd_elems_per_t * T     */
  int64_t bwd_elems_per_t;    /* backward workspace doubles = bwd_elems_per_t * T + bwd_elems_fixed */
  int64_t bwd_elems_fixed;
  int64_t status_bytes;       /* device status word block (zeroed by the library)          */
  int64_t generations;        /* 1: every workgroup of a launch co-resident (time-pipelined);  */
                              /* g > 1: blocks exceed the device, they run in ~g waves       */
} ddr_graph_info;

/* Build from a host COO (rows = downstream reach, cols = upstream reach, int32, E entries), the
 * ddr-engine zarr contract (engine/src/ddr_engine/core/zarr_io.py:7-76).  Validates lower
 * triangularity and dendritic structure, canonicalises (rows sorted, columns ascending), splits
 * and packs basins into workgroups, and uploads the schedule to the current HIP device.
 * Synchronous (the only host-synchronising call besides ddr_graph_status). */
ddr_status ddr_graph_build(int64_t n, int64_t e, const int32_t* rows, const int32_t* cols,
                           const ddr_build_opts* opts, ddr_graph** out);
/* The same host build with the schedule upload stream-ordered on `stream` (SURVEY §8(b)'s
 * ddr_graph_build(..., hipStream_t, ...)): one pinned staging block, one pooled device block, one copy on
 * `stream`; routing launches on any stream wait for it (no hipMalloc / device-wide synchronisation).
 * The host part (validation, partition) is synchronous and returns the counts, as ddr_graph_build. */
ddr_status ddr_graph_build_async(int64_t n, int64_t e, const int32_t* rows, const int32_t* cols,
                                 const ddr_build_opts* opts, void* stream, ddr_graph** out);
/* The same build from a COO in DEVICE memory (rows / cols: int32 device pointers on the current HIP
 * device), computed on the device on `stream` (north star (1)): validation, canonical CSR, distance
 * to outlet, basins, the stem-preserving split and the whole per-workgroup schedule are device
 * passes; only the packing of the pieces (a few thousand) runs on the host, between two small reads
 * of the device per split pass.  The schedule equals ddr_graph_build's for the same COO, bit for bit
 * (ddr_graph_fingerprint).  Returns once the graph is complete on `stream`; its arrays are
 * device-resident (ddr_graph_csr / ddr_graph_structure copy them to the host on request). */
ddr_status ddr_graph_build_device(int64_t n, int64_t e, const int32_t* rows, const int32_t* cols,
                                  const ddr_build_opts* opts, void* stream, ddr_graph** out);
/* The same build in two halves, for a training loop that builds batch k + d while it trains on batch
 * k, all on its own stream: _begin enqueues every device pass up to the piece table and its copy to
 * pinned host memory and returns at once (no host wait); _finish waits for that copy (long complete
 * when begun a step or more ahead), packs the pieces on the host and enqueues the schedule emission
 * on the same stream.  _finish consumes the pending build (also on error); _cancel drops one unused.
 * rows / cols must stay valid until _finish returns. */
typedef struct ddr_graph_pending ddr_graph_pending;
ddr_status ddr_graph_build_device_begin(int64_t n, int64_t e, const int32_t* rows, const int32_t* cols,
                                        const ddr_build_opts* opts, void* stream, ddr_graph_pending** out);
ddr_status ddr_graph_build_device_finish(ddr_graph_pending* p, ddr_graph** out);
ddr_status ddr_graph_build_device_cancel(ddr_graph_pending* p);
/* FNV-1a hash of a graph's whole schedule (per-reach arrays, block descriptors): equal for a host and
 * a device build of the same COO and options.  Synchronous (copies the device schedule). */
ddr_status ddr_graph_fingerprint(const ddr_graph* g, uint64_t* fp);
/* Per-batch gauge union, replacing construct_network_matrix (src/ddr/io/builders.py:55-109) and the
 * compression steps of Merit._collate_gages (src/ddr/geodatazoo/merit.py:197-238; Lynker twin
 * lynker_hydrofabric.py:198-266).  Host, O(E + n_conus), no device.
 *   in : n_conus; n_gauges subsets as one COO in CONUS numbering, subset g = entries
 *        [sub_off[g], sub_off[g+1]) of rows (downstream) / cols (upstream); gage_idx[g] (CONUS).
 *   out: active[n_active] CONUS ids of the union's reaches, ascending (capacity: min(n_conus,
 *        2 E + n_gauges)); crow[n_active + 1], col[nnz] canonical CSR of the compressed union
 *        (capacity of col: E); out_off[n_gauges + 1], out_idx (out_idx_cap entries; E + n_gauges
 *        suffices for consistent subsets, DDR_ERR_ARG when the lists would exceed it): outflow_idx
 *        of each gauge, the compressed upstream reaches of its reach ascending (itself when it has
 *        none); gage_c[n_gauges] each gauge's compressed index.
 * Rejects non-lower-triangular entries (DDR_ERR_NOT_LOWER) and a union in which a reach drains into
 * two reaches (DDR_ERR_NOT_DENDRITIC). */
ddr_status ddr_collate_gauges(int64_t n_conus, int64_t n_gauges, const int64_t* sub_off, const int32_t* rows,
                              const int32_t* cols, const int32_t* gage_idx, int32_t* active, int64_t* n_active,
                              int64_t* crow, int32_t* col, int64_t* nnz, int64_t* out_off, int32_t* out_idx,
                              int64_t out_idx_cap, int32_t* gage_c);
/* The same union on the device (all arrays device memory on the current HIP device, work on `stream`):
 * the subsets concatenated into one COO of e entries (rows / cols, CONUS numbering; the subset
 * boundaries do not matter to the union).  Outputs: active (active_cap entries) and *n_active (host);
 * the compressed union as a COO rows_c / cols_c (ascending cols; capacity e) with *nnz (host) entries
 * -- the input of ddr_graph_build_device -- and as canonical CSR crow (int64, n_active + 1) / col
 * (capacity e); out_off (int64, n_gauges + 1) / out_idx (out_idx_cap) and gage_c as
 * ddr_collate_gauges.  Bit-identical to ddr_collate_gauges; synchronous (returns the counts). */
ddr_status ddr_collate_gauges_device(int64_t n_conus, int64_t n_gauges, int64_t e, const int32_t* rows,
                                     const int32_t* cols, const int32_t* gage_idx, int32_t* active, int64_t active_cap,
                                     int64_t* n_active, int32_t* rows_c, int32_t* cols_c, int64_t* nnz, int64_t* crow,
                                     int32_t* col, int64_t* out_off, int32_t* out_idx, int64_t out_idx_cap,
                                     int32_t* gage_c, void* stream);
/* Upload the schedule of a graph built with DDR_BUILD_HOST_ONLY to the current HIP device (no-op
 * if already uploaded).  The host build needs no device: it can run on any host thread (e.g. a
 * data-loader worker preparing the next training batch, merit.py:197-223) while the device routes
 * the current one; only this step touches the device.  Synchronous. */
ddr_status ddr_graph_upload(ddr_graph* g);
/* ddr_graph_upload stream-ordered on `stream` (as ddr_graph_build_async): returns without a host wait. */
ddr_status ddr_graph_upload_async(ddr_graph* g, void* stream);
/* Any graph size builds: workgroups take ticket-ordered logical blocks, so a schedule with more
 * blocks than co-resident workgroups still completes (ddr_graph_info.generations > 1).
 * ddr_graph_destroy is synchronous: a graph with pooled (stream-ordered) memory waits for the device. */
ddr_status ddr_graph_destroy(ddr_graph* g);
/* Destroy a graph whose last use is queued on `stream`: a device-built graph's memory is released
 * stream-ordered (no device-wide synchronisation -- the per-batch graphs of a training loop); a
 * host-built one's as ddr_graph_destroy. */
ddr_status ddr_graph_destroy_async(ddr_graph* g, void* stream);
/* Release every idle block of the library's memory pools (device blocks of device-built graphs and
 * async uploads, pinned staging blocks) whose last user's queued work has finished; *freed_bytes
 * (may be NULL) receives the bytes returned to HIP.  Blocks handed out or still in use stay. */
ddr_status ddr_pool_trim(int64_t* freed_bytes);
ddr_status ddr_graph_get_info(const ddr_graph* g, ddr_graph_info* info);
/* Canonical CSR of the adjacency into host buffers: crow (n+1), col (nnz), int64. */
ddr_status ddr_graph_csr(const ddr_graph* g, int64_t* crow, int64_t* col);
/* Host copies of the dendritic structure: down (n, -1 = outlet), dist (n, hops to outlet),
 * basin (n, outlet reach id), block (n, workgroup id), each int64; any pointer may be NULL. */
ddr_status ddr_graph_structure(const ddr_graph* g, int64_t* down, int64_t* dist, int64_t* basin,
                               int64_t* block);

/* Physical constants of the routing step (mmc.py:192-208, trapezoidal.py:79, mmc.py:166). */
typedef struct {
  double dt;             /* seconds per step (3600; BMI may override, ddr_bmi.py:208) */
  double discharge_lb;   /* q_lb */
  double velocity_lb;
  double velocity_ub;    /* 15 */
  double depth_lb;
  double bottom_width_lb;
  double side_slope_lb;  /* 0.5 */
  double side_slope_ub;  /* 50 */
} ddr_mc_consts;

/* Per-reach inputs in the reference reach order.  Element type is float for the *_f32 entry
 * points and double for the *_f64 ones.  p_spatial may be a single value (p_stride = 0). */
typedef struct {
  const void* n;           /* Manning n, denormalised                 (N)   */
  const void* q_spatial;   /* Leopold & Maddock exponent, denormalised  (N)   */
  const void* p_spatial;   /* Leopold & Maddock coefficient        (N) or (1) */
  int64_t p_stride;        /* 1 (per reach) or 0 (scalar)                     */
  const void* length;      /* m                                         (N)   */
  const void* slope;       /* already clamped at the slope minimum     (N)   */
  const void* x_storage;   /* Muskingum X                               (N)   */
  const void* flow_scale;  /* optional per-reach q' multiplier (N) or NULL    */
  int64_t qprime_hours;    /* hours per stored q' row: 0/1 hourly (T, N); 24 a daily */
                           /* store (ceil(T / 24), N), indexed q'[t / 24] in-kernel, */
                           /* the reader's repeat(24) (readers.py:513-519)           */
  const uint8_t* qprime_valid; /* optional (N): 0 = divide missing from the store, */
                           /* its q' is 0.001 (readers.py:523-530); NULL = all valid */
} ddr_mc_reaches;

/* Gauge mode: out[g, t] = sum_{k in [off[g], off[g+1])} Q_t[idx[k]] (device int64 arrays,
 * indices already normalised to [0, N)); reach_offsets/reach_gauges list, per reach, the gauges
 * (with multiplicity) whose outflow set contains it. */
typedef struct {
  int64_t n_gauges;
  const int64_t* offsets;        /* (G+1)                                         */
  const int64_t* index;          /* (offsets[G]) reach ids                         */
  const int64_t* reach_offsets;  /* (N+1) inverse map used by the backward        */
  const int64_t* reach_gauges;   /* (offsets[G]) gauge id of each membership      */
} ddr_gauges;

/* DDR_FWD_SAVE_X is accepted for compatibility: x_save is always written.
 * DDR_FWD_ACCUMULATE: every step is a hot start, Q_t = max((I - N)^-1 q'_t, q_lb) with step t
 * reading q' row t -- the per-day discharge accumulation of scripts/geometry_predictor.py:193-212
 * (compute_hotstart_discharge, mmc.py:25-66) for all days in one launch. */
/* Forward coefficient arithmetic (fp32 only; default: the reference's operation order with IEEE
 * division and a correctly rounded pow -- bit-identical to the oracle):
 * DDR_FWD_FAITHFUL_MATH: the same operation order and IEEE divisions, pow in fp32 faithful-class
 *   arithmetic (like the reference's own Sleef powf; no fp64 on the chain);
 * DDR_FWD_FAST_MATH: hardware v_rcp / v_log / v_exp throughout (~1e-6 relative per coefficient). */
enum { DDR_FWD_SAVE_X = 1, DDR_FWD_CARRY = 2, DDR_FWD_NO_RUNOFF = 4, DDR_FWD_ACCUMULATE = 8, DDR_FWD_FAST_MATH = 16,
       DDR_FWD_FAITHFUL_MATH = 32, DDR_FWD_CHECK_QPRIME = 64, DDR_BWD_EXACT_ADJOINT = 128 };
/* DDR_BWD_EXACT_ADJOINT (backward flag, fp32; ignored by the forward): the adjoint of the fp32 trajectory the
 * forward computed to ~1e-6 on any depth.  dL/dk (the Muskingum K) is a sum of O(Q) terms that cancels to the
 * step's discharge change; by default the fp32 adjoint takes that change as Q(t-1) - x(t) from the stored
 * fp32 state (no q' re-read), which carries x's rounding into it: ~1e-3 of the gradient on a 2215-deep
 * basin, ~1e-7 on shallow ones.  With the flag it forms the step's mass imbalances Q(t-1) - q'c - sum x_j(t)
 * and Q(t-1) - q'c - I(t) exactly (fp64 upstream sums, q' re-read): 1.8e-7 there, +30 % backward time. */
/* DDR_FWD_CHECK_QPRIME: the forward also tests the flow-scaled q' of the window for NaN (the reference's
 * cold-start assertion, mmc.py:335) inside its q' gather -- no extra pass over q'.  The verdict of the
 * calling thread's last such launch: ddr_qprime_nan_wait, which waits for the gather only (an event
 * recorded behind it), not for the routing kernel queued after it. */
ddr_status ddr_qprime_nan_wait(int32_t* has_nan);

/* Fused forward over T steps (hot start at t = 0 unless DDR_FWD_CARRY, then q0 is Q_0).
 * Returns DDR_ERR_TIMEOUT instead of launching when an earlier launch's hand-off timed out
 * (ddr_status_check). 
 *   qprime     (T, N) lateral inflow, time-major, reference order
 *   q0         (N) carried discharge (DDR_FWD_CARRY) or NULL
 *   runoff     (N, T), or NULL / DDR_FWD_NO_RUNOFF (e.g. gauges: ddr_gauge_reduce afterwards)
 *   x_save     required workspace (save_elems_per_t * T + save_elems_fixed reals): the routed
 *              states, then q' * flow_scale, both in the schedule layout (runoff is written
 *              by the routing kernel itself); keep it unchanged for ddr_mc_backward
 *   bnd        forward boundary buffer (bnd_elems_per_t * T doubles; may be NULL if n_cut == 0);
 *              must be kept unchanged for ddr_mc_backward
 *   status     device status block (status_bytes)
 *   q_last, top_width_last, side_slope_last (N), any may be NULL */
ddr_status ddr_mc_forward_f32(const ddr_graph* g, const ddr_mc_consts* c, const ddr_mc_reaches* r,
                              const float* qprime, int64_t T, const float* q0, float* runoff,
                              float* x_save, double* bnd, void* status, float* q_last,
                              float* top_width_last, float* side_slope_last, int32_t flags,
                              void* stream);
ddr_status ddr_mc_forward_f64(const ddr_graph* g, const ddr_mc_consts* c, const ddr_mc_reaches* r,
                              const double* qprime, int64_t T, const double* q0, double* runoff,
                              double* x_save, double* bnd, void* status, double* q_last,
                              double* top_width_last, double* side_slope_last, int32_t flags,
                              void* stream);

/* Hot start (src/ddr/routing/mmc.py:25-66 compute_hotstart_discharge): out = max((I - N)^-1 q, lb) for
 * q (N) in reference order -- the accumulation solve of the routing graph in one launch, fp64 sums as
 * the reference's SciPy solve; device pointers, enqueued on `stream` (its workspace is stream-ordered
 * scratch).  The same sweep is step 0 of every ddr_mc_forward_f32 without DDR_FWD_CARRY. */
ddr_status ddr_hotstart_f32(const ddr_graph* g, const float* q, double discharge_lb, float* out, void* stream);

/* Reverse-time, reverse-topological adjoint.  grad_runoff is (N, T), or (G, T) with gauges != NULL.
 * bwd_bnd is the backward workspace (size in ddr_graph_info).
 * Writes per-reach dL/dn, dL/dq_spatial, dL/dp_spatial (N each; for a scalar p the caller sums). */
ddr_status ddr_mc_backward_f32(const ddr_graph* g, const ddr_mc_consts* c, const ddr_mc_reaches* r,
                               const float* qprime, int64_t T, const float* x_save,
                               const double* bnd, const float* grad_runoff, const ddr_gauges* gauges,
                               double* bwd_bnd, void* status, float* grad_n, float* grad_q,
                               float* grad_p, int32_t flags, void* stream);
ddr_status ddr_mc_backward_f64(const ddr_graph* g, const ddr_mc_consts* c, const ddr_mc_reaches* r,
                               const double* qprime, int64_t T, const double* x_save,
                               const double* bnd, const double* grad_runoff, const ddr_gauges* gauges,
                               double* bwd_bnd, void* status, double* grad_n, double* grad_q,
                               double* grad_p, int32_t flags, void* stream);

/* State-gradient adjoint: ddr_mc_backward plus the gradients the reference's autograd delivers to
 * the lateral inflow and the discharge state (routing/mmc.py:487-559 route_timestep is
 * differentiable w.r.t. q_prime_clamp and _discharge_t; the hot start mmc.py:25-66 w.r.t. q'[0]):
 *   grad_qprime (qprime_rows, N) dL/dq' in the caller's store layout (rows of qprime_hours steps;
 *               flow_scale applied, 0 for a divide filled by qprime_valid), or NULL
 *   grad_q0     (N) dL/dQ0 of a carried state (forward run with DDR_FWD_CARRY), or NULL
 *   work        device workspace of ddr_state_work_bytes(g, T, n_gauges, sizeof(real)) bytes
 * Replaces: torch autograd through mmc.py:421-424 (q' clamp), 535-538 (c4 q'), 25-66 (hot start)
 * and the carried _discharge_t (mmc.py:330-342). */
int64_t ddr_state_work_bytes(const ddr_graph* g, int64_t T, int64_t n_gauges, int32_t real_bytes);
ddr_status ddr_mc_backward_state_f32(const ddr_graph* g, const ddr_mc_consts* c, const ddr_mc_reaches* r,
                                     const float* qprime, int64_t qprime_rows, int64_t T, const float* x_save,
                                     const double* bnd, const float* grad_runoff, const ddr_gauges* gauges,
                                     double* bwd_bnd, void* status, float* grad_n, float* grad_q,
                                     float* grad_p, float* grad_qprime, float* grad_q0, void* work,
                                     int32_t flags, void* stream);
ddr_status ddr_mc_backward_state_f64(const ddr_graph* g, const ddr_mc_consts* c, const ddr_mc_reaches* r,
                                     const double* qprime, int64_t qprime_rows, int64_t T, const double* x_save,
                                     const double* bnd, const double* grad_runoff, const ddr_gauges* gauges,
                                     double* bwd_bnd, void* status, double* grad_n, double* grad_q,
                                     double* grad_p, double* grad_qprime, double* grad_q0, void* work,
                                     int32_t flags, void* stream);

/* The general adjoint: ddr_mc_backward_state (grad_qprime, grad_q0 and work may be NULL: with both NULL
 * this is ddr_mc_backward) plus per-reach gradients into the discharge state itself:
 *   state_seed  (2, N) reference order, or NULL: row 0 dL/dQ_{T-1} -- the final state `_discharge_t`
 *               (mmc.py:441, retained by dmc, torch_mc.py:196-216; an ordinary autograd tensor in gauge
 *               mode too, mmc.py:433-441) -- and row 1 dL/dQ_{T-2}, the state the reported top width /
 *               side slope of the last step were computed from (mmc.py:161-162; the caller forms it by
 *               differentiating that geometry, e.g. from ddr_state_f32's Q_{T-2})
 * Replaces: torch autograd through `_discharge_t` and `top_width` / `side_slope` after a forward. */
ddr_status ddr_mc_backward_ex_f32(const ddr_graph* g, const ddr_mc_consts* c, const ddr_mc_reaches* r,
                                  const float* qprime, int64_t qprime_rows, int64_t T, const float* x_save,
                                  const double* bnd, const float* grad_runoff, const ddr_gauges* gauges,
                                  const float* state_seed, double* bwd_bnd, void* status, float* grad_n,
                                  float* grad_q, float* grad_p, float* grad_qprime, float* grad_q0, void* work,
                                  int32_t flags, void* stream);
ddr_status ddr_mc_backward_ex_f64(const ddr_graph* g, const ddr_mc_consts* c, const ddr_mc_reaches* r,
                                  const double* qprime, int64_t qprime_rows, int64_t T, const double* x_save,
                                  const double* bnd, const double* grad_runoff, const ddr_gauges* gauges,
                                  const double* state_seed, double* bwd_bnd, void* status, double* grad_n,
                                  double* grad_q, double* grad_p, double* grad_qprime, double* grad_q0,
                                  void* work, int32_t flags, void* stream);

/* Q_t (N, reference order) from a forward's saved states: max(x(t), discharge_lb), or x(0) unclamped for a
 * carried state (flags & DDR_FWD_CARRY) -- the routed discharge the reference holds as `_discharge_t`
 * after step t (mmc.py:441, 557).  Enqueued on `stream`; 0 <= t < T.
 * Replaces: reading MuskingumCunge._discharge_t / output[:, t] mid-window (mmc.py:428-441). */
ddr_status ddr_state_f32(const ddr_graph* g, const float* x_save, int64_t T, int64_t t, double discharge_lb,
                         int32_t flags, float* out, void* stream);
ddr_status ddr_state_f64(const ddr_graph* g, const double* x_save, int64_t T, int64_t t, double discharge_lb,
                         int32_t flags, double* out, void* stream);

/* Fused parameter network of the C3 training step (the bench's stand-in for the reference's KAN,
 * src/ddr/nn/kan.py:11-62, whose pykan dependency is not installed): attributes x (n_rows, n_features <= 12)
 * -> Linear(F, 128) -> SiLU -> Linear(128, 128) -> SiLU -> Linear(128, 128) -> SiLU -> Linear(128, 3) -> sigmoid
 * -> denormalize (routing/utils.py:166-185: y = u scale + offset, exp(y) for a log-space parameter) ->
 * out_n, out_q, out_p (n_rows each), on the fp32 matrix cores.
 *   params  flat fp32, ddr_pnet_param_count(F) values: W1 (128, F) | b1 (128) | W2 (128, 128) | b2 | W3 | b3 |
 *           W4 (3, 128) | b4 (3), torch.nn.Linear's (out, in) weight layout
 *   denorm  HOST array [3][3]: per output (scale, offset, log-space flag)
 *   z_save  (3, n_rows, 128) pre-activations, u_save (n_rows, 3) sigmoid outputs: kept for the backward
 *   grad_params (same layout as params) = dL/dparams given dL/d(out_n, out_q, out_p); work: device scratch of
 *           ddr_pnet_work_bytes bytes.  Deterministic (fixed-order reduction of per-workgroup partials).
 * Replaces: the network's forward (kan.py:50-62) and its torch autograd in scripts/train.py:54-104. */
int64_t ddr_pnet_param_count(int32_t n_features);
int64_t ddr_pnet_work_bytes(int64_t n_rows, int32_t n_features);
ddr_status ddr_pnet_forward_f32(int64_t n_rows, int32_t n_features, const float* x, const float* params,
                                const float* denorm, float* z_save, float* u_save, float* out_n, float* out_q,
                                float* out_p, void* stream);
ddr_status ddr_pnet_backward_f32(int64_t n_rows, int32_t n_features, const float* x, const float* params,
                                 const float* denorm, const float* z_save, const float* u_save, const float* grad_n,
                                 const float* grad_q, const float* grad_p, float* grad_params, void* work,
                                 void* stream);

/* The tail of a training step (scripts/train.py:91-100), one launch each, device pointers on `stream`:
 * ddr_daily_l1_f32: loss[0] = inv_count * sum_{g, d >= warmup} |daily[g, d] - obs[g, d]| over (G, D) row-major
 *   series, and (grad != NULL) grad[g, d] = inv_count * sign(daily - obs), 0 for d < warmup -- l1_loss
 *   (train.py:91-94; inv_count = 1 / (G (D - warmup)) is its mean) and its backward in one pass.
 * ddr_clip_adam_f32: clip_grad_norm_(max_norm) (train.py:99; max_norm <= 0: none) then one Adam step
 *   (torch.optim.Adam, no weight decay / amsgrad; train.py:100) on a flat parameter vector of n values with
 *   its moments m, v; step is a device fp32 counter (0 before the first step) that the launch increments and
 *   takes the bias corrections from, as torch's capturable Adam does -- no host value, so the launch can be
 *   captured into a graph and replayed.
 *   norm_out (or NULL) receives the gradient's norm before clipping.  grad is not modified.  work: device
 *   scratch of ddr_clip_adam_work_bytes() bytes.
 * Both deterministic (fixed slices and reduction order).
 * Replaces: the ~15 PyTorch launches of l1_loss + backward, clip_grad_norm_ and Adam.step per step. */
ddr_status ddr_daily_l1_f32(int64_t n_gauges, int64_t n_days, int64_t warmup, const float* daily, const float* obs,
                            float inv_count, float* loss, float* grad, void* stream);
int64_t ddr_clip_adam_work_bytes(void);
ddr_status ddr_clip_adam_f32(int64_t n, float* params, const float* grad, float* m, float* v, float lr, float beta1,
                             float beta2, float eps, float* step, float max_norm, float* norm_out, void* work,
                             void* stream);

/* Gauge reduction of a forward's saved states x_save: runoff (G, T). */
ddr_status ddr_gauge_reduce_f32(const ddr_graph* g, const float* x_save, int64_t T,
                                const ddr_gauges* gauges, double discharge_lb, int32_t flags,
                                float* runoff, void* stream);
ddr_status ddr_gauge_reduce_f64(const ddr_graph* g, const double* x_save, int64_t T,
                                const ddr_gauges* gauges, double discharge_lb, int32_t flags,
                                double* runoff, void* stream);

/* Gauge-mode training objective, fused (scripts/train.py:78-82 + io/functions.py:7-23): daily area
 * means of the gauge sums over the trimmed window [t0, t0 + L) of the routed states x_save,
 * out (G, D): day d averages hours t0 + [floor(d L / D), ceil((d + 1) L / D)) like
 * F.interpolate(mode="area").  The reference trims runoff[:, 13 : -11 + tau] and pools to
 * D = L // 24 days: t0 = 13, L = T - 24 + tau. */
ddr_status ddr_gauge_daily_f32(const ddr_graph* g, const float* x_save, int64_t T, const ddr_gauges* gauges,
                               double discharge_lb, int32_t flags, int64_t t0, int64_t L, int64_t D,
                               float* daily, void* stream);
ddr_status ddr_gauge_daily_f64(const ddr_graph* g, const double* x_save, int64_t T, const ddr_gauges* gauges,
                               double discharge_lb, int32_t flags, int64_t t0, int64_t L, int64_t D,
                               double* daily, void* stream);
/* Its adjoint: dL/d(hourly gauge series) (G, T) from dL/d(daily) (G, D), the seed of the gauge-mode
 * ddr_mc_backward (zero outside the trimmed window). */
ddr_status ddr_gauge_daily_seed_f32(int64_t G, int64_t T, int64_t t0, int64_t L, int64_t D,
                                    const float* grad_daily, float* grad_hourly, void* stream);
ddr_status ddr_gauge_daily_seed_f64(int64_t G, int64_t T, int64_t t0, int64_t L, int64_t D,
                                    const double* grad_daily, double* grad_hourly, void* stream);

/* Per-reach temporal statistics of the trapezoid geometry (src/ddr/geometry/statistics.py:20-83):
 * q_daily holds the daily accumulated discharge, element (reach, day) at
 * reach * reach_stride + day * day_stride (1 <= days <= 32768); out is (24, n): for the variables
 * depth, top_width, bottom_width, side_slope, hydraulic_radius, discharge (in this order) the rows
 * min, max, median, mean (NaN skipped as numpy's nan* reductions).  Device pointers, float32. */
ddr_status ddr_geometry_stats_f32(const float* q_daily, int64_t reach_stride, int64_t day_stride, int64_t n,
                                  int64_t days, const float* n_manning, const float* p_spatial,
                                  int64_t p_stride, const float* q_spatial, const float* slope,
                                  double depth_lb, double bottom_width_lb, float* out, void* stream);

/* Synchronise `stream` and read the device status block written by the last launches:
 * returns DDR_OK or DDR_ERR_TIMEOUT. */
ddr_status ddr_graph_status(const void* status, void* stream);
/* Hand-off failures without a host sync: every routing launch queues an async copy of its status
 * words; every entry point returns DDR_ERR_TIMEOUT once a queued copy reports a timed-out hand-off
 * (whose outputs hold NaN).  wait = 1 blocks until every queued copy has landed.  No reference
 * counterpart (the reference solver raises ValueError on failure, routing/utils.py:598-600). */
ddr_status ddr_status_check(int32_t wait);
/* ---- One basin split across GPUs (no reference counterpart: the reference routes a basin on one
 * device; north star item (5)) ----------------------------------------------------
 * Every rank of a split builds the SAME graph of the basin (same COO and options: the builders are
 * deterministic), then ddr_graph_set_split tells it which logical blocks it runs (block_rank[b] ==
 * rank; the others are skipped).  A cut edge between blocks of two ranks carries its fp64 granules
 * through the receive memory of the rank that reads them: the consumer's in the forward, the
 * producer's in the backward, written with system-scope stores over xGMI.  Each rank allocates its
 * receive memory with ddr_xmem_alloc (uncached device memory, exported as an IPC handle of
 * DDR_XMEM_HANDLE_BYTES bytes), the ranks exchange handles (torch.distributed) and open the peers'
 * with ddr_xmem_open.  Before each routing launch the ranks reset their receive rows and hand-shake
 * on the device (an epoch word per peer), so no host synchronisation is needed; all ranks of a split
 * must call forward / backward the same number of times with the same T.  Gauge mode and state
 * gradients are not supported on a split graph. */
enum { DDR_XMEM_HANDLE_BYTES = 64 };
/* bytes of one rank's receive memory for n_x cross-rank cut edges and windows of up to T steps */
ddr_status ddr_xmem_bytes(int64_t n_x, int64_t T, int64_t* bytes);
/* kind: 0 uncached, 1 fine-grained, 2 plain device memory (the first kind that exports) */
ddr_status ddr_xmem_alloc(int64_t bytes, void** ptr, void* handle, int32_t* kind);
ddr_status ddr_xmem_open(const void* handle, void** ptr);
ddr_status ddr_xmem_close(void* ptr, int32_t opened);
/* reaches of every logical block (n_blocks entries, ticket order) */
ddr_status ddr_graph_blocks(const ddr_graph* g, int32_t* nloc, int64_t cap);
/* producer (upstream) and consumer (downstream) logical block of every cut edge (n_cut entries) */
ddr_status ddr_graph_cut_blocks(const ddr_graph* g, int32_t* prod, int32_t* cons, int64_t cap);
/* block_rank: n_blocks entries in [0, nranks); peers: every rank's receive memory (peers[rank] ==
 * local), each ddr_xmem_bytes(n_x, t_cap) bytes, n_x = the cut edges whose blocks differ in rank
 * (returned in *n_x) */
ddr_status ddr_graph_set_split(ddr_graph* g, int32_t rank, int32_t nranks, const int32_t* block_rank, void* local,
                               void* const* peers, int64_t t_cap, int64_t* n_x);
/* detach the split (before its receive memory is released): later launches run every block again.
 * One stream per split graph: its launch epochs are counted per graph. */
ddr_status ddr_graph_clear_split(ddr_graph* g);

/* Debug knobs.  DDR_DEBUG_FORCE_TIMEOUT: every inter-workgroup wait of the following launches
 * times out (tests the failure path).  DDR_DEBUG_NO_STEADY: the routing kernels run every tick
 * through their general path instead of the specialised steady-tick path (bitwise A/B; also set by
 * the environment variable DDR_NO_STEADY=1).  DDR_DEBUG_NO_STORER: light forward blocks store the
 * routing state and runoff from their compute waves instead of their idle waves (DDR_NO_STORER=1).
 * DDR_DEBUG_NO_PLAIN: launches without the rare options (split basin, profile, state seeds, daily
 * accumulation) run the general kernel instances instead of the plain ones compiled without those options
 * (bitwise A/B; DDR_NO_PLAIN=1). */
enum { DDR_DEBUG_FORCE_TIMEOUT = 1, DDR_DEBUG_NO_STEADY = 2, DDR_DEBUG_NO_STORER = 4, DDR_DEBUG_NO_PLAIN = 8 };
ddr_status ddr_set_debug_flags(int32_t flags);

/* General sparse triangular solve A x = b (lower) or A^T x = b (transpose = 1), CSR A with a
 * non-unit diagonal, fp32 values accumulated in fp64 (SciPy semantics, utils.py:587-600).
 * crow/col are HOST int64 arrays (the pattern); values, b, x are device float arrays.
 * Synchronous w.r.t. the pattern upload only. */
ddr_status ddr_tri_solve(int64_t n, int64_t nnz, const int64_t* crow_host, const int64_t* col_host,
                         const float* values, const float* b, float* x, int32_t lower,
                         int32_t transpose, void* stream);
/* ddr_tri_solve with SciPy's / CuPy's unit_diagonal (routing/utils.py:596, 611 forward; 239, 307
 * backward): unit_diagonal != 0 takes every diagonal entry as 1 without reading it (a missing one
 * included) and skips the diag^-1 scaling and the singular check (no host round trip). */
ddr_status ddr_tri_solve_ex(int64_t n, int64_t nnz, const int64_t* crow_host, const int64_t* col_host,
                            const float* values, const float* b, float* x, int32_t lower,
                            int32_t transpose, int32_t unit_diagonal, void* stream);
/* gradA[k] = -gradb[row(k)] * x[col(k)] for CSR (device int64 crow/col). */
ddr_status ddr_tri_grad_values(int64_t n, int64_t nnz, const int64_t* crow, const int64_t* col,
                               const float* gradb, const float* x, float* grad_values, void* stream);

/* Kernel timing (measurement hook, no reference counterpart).  While enabled, every routing
 * launch brackets its main kernel (route_forward_kernel / route_backward_kernel) with HIP events
 * on the launch stream.  ddr_kernel_ms(0 = forward, 1 = backward) synchronises on the last such
 * pair and returns its duration in milliseconds. */
ddr_status ddr_set_kernel_timing(int32_t enable);
ddr_status ddr_kernel_ms(int32_t which, float* ms);

/* Per-workgroup launch profile (debug).  When `buf` is non-null, the next routing launches write
 * 16 uint64 per workgroup: start and end (s_memrealtime, 100 MHz), time spent waiting on
 * inter-workgroup imports, the hardware id (HW_ID | XCC_ID << 32), then the time at every 1024th
 * tick.  `buf` is a zeroed device array of at least 16 * n_blocks uint64; which = 0 (forward) or
 * 1 (backward). */
ddr_status ddr_set_block_profile(int32_t which, uint64_t* buf);

/* Device capacity helpers. */
ddr_status ddr_device_info(int32_t* n_cu, int32_t* max_resident_blocks);
const char* ddr_last_error(void);
const char* ddr_version(void);

#ifdef __cplusplus
}
#endif
#endif /* DDR_MC_H */
