// Internal definitions shared by the host graph builder (graph.cpp), the routing kernels
// (route.hip) and the C ABI (capi.cpp).  Not part of the public interface (include/ddr_mc.h).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/ddr_mc.h"

namespace ddr {

// Routing workgroups: 1024 threads (16 waves, 4 per SIMD), one per CU, up to kMaxKR reaches per
// thread.  The per-reach statics live in LDS, not registers, so the 128-VGPR budget of 4 waves per
// SIMD holds KR = 4.  One workgroup per CU (not two of 512): co-resident workgroups are served by
// age priority, so the younger one of a pair progresses at less than half the older one's tick
// rate, and every multi-workgroup basin is throttled to its slowest member (measured).
#ifndef DDR_BLOCK_THREADS
#define DDR_BLOCK_THREADS 1024
#endif
constexpr int kBlockThreads = DDR_BLOCK_THREADS;
constexpr int kMaxKR = 4;
constexpr int kBlocksPerCU = 1024 / kBlockThreads;
// Default workgroup capacity (reaches): KR = 4 reaches per thread.  The LDS check of the builder
// lowers it when a block's slots and import rings would not fit.
constexpr int kDefaultBlockReaches = kBlockThreads * kMaxKR;
// Smallest workgroup capacity the packer aims for when the network is small (graph.cpp).
#ifndef DDR_MIN_BLOCK_CAP
#define DDR_MIN_BLOCK_CAP 256
#endif
constexpr int kMinBlockCap = DDR_MIN_BLOCK_CAP;
// LDS budget per workgroup (160 KiB per CU).
constexpr size_t kLdsBudget = 160 * 1024 / kBlocksPerCU - 512;
// Chunk of ticks between two inter-workgroup imports (SURVEY §7 "time-pipelined").  Every
// block-DAG hop adds about one chunk of lag, so the chunk is short.
// Forward and backward chunks differ (A/B, profiles/r02/ab_defer_early.txt: forward 4 beats 8 and 16;
// the backward's import is a workgroup-wide step, 8 kept).  The forward's must be a multiple of the
// import batch (4).
#ifndef DDR_CHUNK_FWD
#define DDR_CHUNK_FWD 4
#endif
#ifndef DDR_CHUNK_BWD
#define DDR_CHUNK_BWD 8
#endif
constexpr int kChunkFwd = DDR_CHUNK_FWD;
constexpr int kChunkBwd = DDR_CHUNK_BWD;
// the packer's lag estimate per block-DAG hop (graph.cpp)
constexpr int kChunk = 8;
// Parameter-gradient partial sums are flushed to the fp64 accumulators every kGradFlush steps
// (aligned to the step index, so the summation grouping does not depend on the partition).
constexpr int kGradFlush = 128;
__host__ __device__ inline size_t align16(size_t x) { return (x + 15) / 16 * 16; }
// LDS slots per buffer of the routing kernels: every block's nloc + nvirt slots, one zero slot
// (missing upstreams of the forward read it), rounded up to even (16-B aligned statics rows).
__host__ __device__ inline int route_slot_stride(int max_slots) { return (max_slots + 2) & ~1; }
// Forward x slots double-buffered by tick parity at KR <= 2 (one workgroup barrier per tick instead of
// two: a tick's results go straight into the other buffer; the LDS is there at one or two reaches per
// thread, not at four)
__host__ __device__ constexpr int fwd_xbuf(int kr) { return kr <= 2 ? 2 : 1; }
// The backward's three slot arrays (c1 gb, c2 gb, published x) likewise: each tick reads the values its
// neighbours wrote the tick before and writes the next tick's, one barrier per tick (KR <= 2)
__host__ __device__ constexpr int bwd_xbuf(int kr) { return kr <= 2 ? 2 : 1; }
// reaches per thread of the routing kernels for a largest block of `max_load` reaches
inline int kr_of_load(int64_t max_load) {
  int kr = 1;
  while (int64_t(kr) * kBlockThreads < max_load) kr *= 2;
  return kr;
}
// Dynamic LDS of the routing kernels (route.hip), for `slots` = nloc + nvirt slots and `nring`
// import rings (virtual inflows forward, cut-outs backward), reals of `rsize` bytes:
//   forward : x slots (f64, xbuf buffers) | 6 statics (R) | ring [nvirt][kChunkFwd] f64
//   backward: A slots (R) | B slots (R) | published x slots (R) (each xbuf buffers) | 6 statics (R)
//             | ring [ncout][kChunkBwd][2] (R)
//             | owner words
// and then the block's confluence lists (after the math tables of fastmath.h, which occupy the first
// kMathTabBytes)
constexpr size_t kMathTabBytes = 3072;
// Confluence lists (reaches with more than two inflows) of a block, in LDS after the ring: at most
// kMaxConfluenceList int32 entries per block (13-bit offsets in the packed upstream word).
constexpr int kMaxConfluenceList = 8191;
__host__ __device__ inline size_t route_lds_bytes(size_t slots, size_t nvirt, size_t ncout, size_t nxl, bool backward,
                                                  size_t rsize, int kr = 4, int xb = 0) {
  // xb: the slot buffers when not the KR rule's (the forward's double-buffered KR = 4 variant; the
  // backward's single-buffered fp64 KR = 2 variant, whose double buffer does not fit)
  const size_t base = backward ? slots * (3 * (size_t)(xb > 0 ? xb : bwd_xbuf(kr)) + 6) * rsize
                               : slots * (8 * (size_t)(xb > 0 ? xb : fwd_xbuf(kr)) + 6 * rsize);
  const size_t ring = backward ? ncout * kChunkBwd * 2 * rsize : nvirt * kChunkFwd * 8;
  // backward: per hand-off owner thread (tid < max(nvirt, ncout)) its virtual's downstream slot and
  // its cut-out's tick offset
  const size_t own = backward ? align16(4 * (nvirt > ncout ? nvirt : ncout)) : 0;
  return kMathTabBytes + align16(base) + align16(ring) + own + nxl * 4;
}

// One workgroup's slice of the schedule.  Reaches of a block occupy internal positions
// [pos0, pos0 + nloc); virtual inflows (edges from other blocks) [virt0, virt0 + nvirt).
struct BlockDesc {
  int32_t pos0;
  int32_t nloc;
  int32_t virt0;
  int32_t nvirt;
  int32_t cout0;   // index into cout_loc (reaches whose downstream lives in another block)
  int32_t ncout;
  int32_t dmax;    // ticks = T + dmax
  int32_t nxl;     // confluence-list entries (LDS copy of xlist[xl0, xl0 + nxl))
  int64_t pre_dn;  // sum over earlier blocks of dmax * nloc (x_save base = T*pos0 + pre_dn)
  int32_t xl0;
  int32_t pad;
};

// Device-side schedule (structure of arrays, indexed by internal position unless noted).
struct DevSchedule {
  BlockDesc* blocks = nullptr;
  int32_t* ref = nullptr;      // reference reach index
  int32_t* off = nullptr;      // tick offset: step t of this reach runs at tick t + off
  int32_t* upb = nullptr;      // first upstream entry in uplist
  int32_t* upc = nullptr;      // number of upstream entries
  int32_t* dloc = nullptr;     // downstream local index in the same block, -1 otherwise
  int32_t* cut = nullptr;      // cut-edge id if the downstream is in another block, -1 otherwise
  int32_t* uplist = nullptr;   // local index (< nloc) or nloc + virtual index
  int32_t* xoff = nullptr;     // block-local confluence-list offset (upc > 2), else -1
  int32_t* xlist = nullptr;    // per block: for each confluence [c, u1, ..., u_{c-1}]
  int32_t* v_edge = nullptr;   // per virtual: cut-edge id
  int32_t* v_off = nullptr;    // per virtual: tick offset (= off(consumer) - 1)
  int32_t* v_dloc = nullptr;   // per virtual: consumer local index
  int32_t* cout_loc = nullptr; // per block list: local indices of reaches with cut >= 0
  int32_t* pos_of_ref = nullptr;   // (N) internal position of each reference reach
  int32_t* block_of_pos = nullptr; // (N) block of each internal position
  int32_t* rs_loc = nullptr;       // (N) per block, local indices in ascending reference order
  int32_t* rs_ref = nullptr;       // (N) the matching reference indices
};

// The same schedule on the host (built by build_graph; released once uploaded).
struct HostSchedule {
  std::vector<int32_t> ref, off, upb, upc, dloc, cut, uplist, xoff, xlist, v_edge, v_off, v_dloc, cout_loc;
  std::vector<int32_t> pos_of_ref, block_of_pos, rs_loc, rs_ref;
};

// CSR and structure of a device-built graph (int32, device memory; host copies on request).
struct DeviceViews {
  int32_t* crow = nullptr;   // (n + 1)
  int32_t* col = nullptr;    // (nnz)
  int32_t* down = nullptr;   // (n)
  int32_t* dist = nullptr;
  int32_t* basin = nullptr;
  int32_t* block = nullptr;
};

// One basin's schedule shared by several ranks (ddr_graph_set_split): every rank builds the same
// graph, runs the blocks it owns and skips the others; a cut edge between blocks of two ranks carries
// its granules through the receive block of the rank that reads them (forward: the consumer block's
// rank, backward: the producer's), written there with system-scope stores (ddr_xmem_alloc: uncached
// device memory shared by IPC handles).  A receive block: [2][kMaxSplitRanks] u64 launch epochs
// (forward, backward; set by each peer before its launch) | forward rows [n_x][T] f64 | backward rows
// [n_x][T][2] f64.
constexpr int kMaxSplitRanks = 16;
struct SplitState {
  int32_t rank = 0, nranks = 0, n_x = 0;
  int64_t t_cap = 0;
  uint8_t* owned = nullptr;  // device (n_blocks): 1 = this rank runs the logical block
  int32_t* xid = nullptr;    // device (n_cut): index among the cross-rank cut edges, -1 = local
  int32_t* xcons = nullptr;  // device (n_x): rank of the consumer (downstream) block
  int32_t* xprod = nullptr;  // device (n_x): rank of the producer (upstream) block
  int64_t* xedge = nullptr;  // device (n_x): the cut edge of each cross-rank index
  char* local = nullptr;     // this rank's receive block
  char* peers[kMaxSplitRanks] = {};
  unsigned long long epoch[2] = {0, 0};
};
inline size_t xmem_flags_bytes() { return 2 * kMaxSplitRanks * sizeof(unsigned long long); }
inline size_t xmem_bytes(int64_t n_x, int64_t T) { return xmem_flags_bytes() + (size_t)(n_x * T) * 24; }

struct Graph {
  int64_t n = 0, nnz = 0;
  std::vector<int64_t> crow, col;
  std::vector<int64_t> down, dist, basin, block_of;
  int64_t n_basins = 0, n_pieces = 0, n_cut = 0, max_depth = 0, max_block_depth = 0;
  int bs = kBlockThreads, kr = 1;
  int max_slots = 0;     // max over blocks of nloc + nvirt
  int max_virt = 0, max_cout = 0;
  int max_xl = 0;        // max over blocks of nxl
  int device = 0;
  std::vector<BlockDesc> blocks;
  int64_t sum_dn = 0;    // sum over blocks of dmax * nloc
  int64_t n_xlist = 0;   // confluence-list entries over all blocks
  int max_nloc = 0;      // largest block
  int64_t generations = 1;  // ceil(blocks / resident) the packer aimed for (1: all blocks co-resident)
  int64_t resident = 0;     // co-resident workgroups assumed by the packer
  HostSchedule hs;
  DevSchedule dev;
  bool uploaded = false;
  bool device_built = false;  // built by build_graph_device: crow/col/down/... live in dviews only
  DeviceViews dviews;
  hipEvent_t ready = nullptr;  // device builds: recorded on the build stream once the schedule is complete
  mutable std::atomic<bool> ready_waited{false};  // a launch outside a stream capture has waited for `ready`
  void* staging = nullptr;     // pinned host sources of the device build's last uploads
  std::vector<void*> allocations;        // hipMalloc (host builds)
  std::vector<void*> async_allocations;  // device_get blocks (device builds): returned stream-ordered
  SplitState split;                      // ddr_graph_set_split (nranks == 0: not split)
};

// ---- piece-level packing, shared by the host builder (graph.cpp) and the device builder ---------
// (devgraph.hip).  Pieces are numbered by descending root index, so a child piece (upstream) comes
// after its parent.
struct PieceTable {
  std::vector<int64_t> root;       // root reach (the piece's most downstream reach)
  std::vector<int64_t> size;       // reaches
  std::vector<int64_t> dmax;       // max in-piece distance of a member to the root
  std::vector<int64_t> xl;         // confluence-list entries (members with more than two inflows)
  std::vector<int64_t> parent;     // piece of down[root], -1 for an outlet piece
  std::vector<int64_t> dloc_down;  // in-piece distance of down[root] (0 for an outlet piece)
  std::vector<int64_t> ht_root;    // longest path from the root up to a source
  std::vector<int64_t> dist_root;  // hops from the root to its outlet
  size_t count() const { return root.size(); }
};
// The packer's state across re-splits (capacity, weighting, generations).
struct PackPlan {
  int64_t n = 0, cap = 0, hard_cap = 0, cap_start = 0, min_cap = 0, target = 0, resident = 0, gen = 1;
  int64_t scap_pct = 80, pack_quant = 1;
  bool weighted = true, dbg = false;
  double steps = 8760.0, fac_pow = 1.0;
  int device = 0;
  int64_t scap() const { return cap * scap_pct / 100; }  // split threshold of this pass
};
struct PackResult {
  int64_t nblocks = 0, ncut = 0;
  std::vector<int64_t> block_of_piece, load, bdmax, bv, bc, bx;  // per block: reaches, dmax, virt, cut-outs, xl
};
enum { kPackDone = 0, kPackResplit = 1 };
// bmax: the largest basin (selects the split threshold)
ddr_status plan_init(int64_t n, int64_t bmax, const ddr_build_opts* opts, PackPlan& plan);
// Pack the pieces of one split; *outcome = kPackResplit when the plan changed (split again).
ddr_status pack_pieces(PackPlan& plan, const PieceTable& pt, PackResult& res, int* outcome);
// Block descriptors and the graph-wide sizes (max slots, KR, ...) of a finished packing.
ddr_status finalize_blocks(Graph* g, const PackPlan& plan, const PackResult& res);
unsigned long long schedule_fingerprint(const HostSchedule& H);
double now_ms();

// error plumbing (capi.cpp)
void set_error(const std::string& msg);
ddr_status fail(ddr_status code, const std::string& msg);
ddr_status hip_fail(hipError_t e, const char* where);
const char* last_error_cstr();

#define DDR_HIP(call)                                        \
  do {                                                       \
    hipError_t _e = (call);                                  \
    if (_e != hipSuccess) return ::ddr::hip_fail(_e, #call); \
  } while (0)

// Pinned host blocks reused across builds (graph.cpp).  hipHostFree waits for every queued device
// operation, so releasing a batch's staging memory that way stalled a training loop's host behind the
// previous step's routing launches (the C3 stream's 28-74 ms graph waits).  pinned_put(p, s) returns a
// block once the work queued on `s` so far is done (an event recorded on `s`); pinned_get reuses a
// returned block of at least `bytes` whose event has fired, or allocates.  Blocks live until exit.
void* pinned_get(size_t bytes);
void pinned_put(void* p, hipStream_t s);
// Device blocks reused the same way (graph.cpp), for the per-batch build scratch and graph arrays:
// hipFreeAsync blocked the host 5-44 ms per call in the training stream (profiles/r03), leaving the
// device idle while the host caught up.  device_get(bytes, s) hands out a free block of the current
// device and makes `s` wait (hipStreamWaitEvent, no host wait) for the work queued when it was
// returned; device_put(p, s) returns it after the work queued on `s` so far.  hipMalloc only grows.
void* device_get(size_t bytes, hipStream_t s);
void device_put(void* p, hipStream_t s);
// Releases every pooled block (pinned and device) that is not handed out and whose last user's work has
// finished; returns the bytes freed (ddr_pool_trim)
int64_t pool_trim();

// graph.cpp
ddr_status build_graph(int64_t n, int64_t e, const int32_t* rows, const int32_t* cols,
                       const ddr_build_opts* opts, Graph** out);
void destroy_graph(Graph* g, hipStream_t stream = nullptr);
// Order `stream` after the device build of `g` (no-op for host builds): every launch that reads the
// schedule calls this first.
inline hipError_t graph_ready(const Graph* g, hipStream_t stream) {
  return g->ready ? hipStreamWaitEvent(stream, g->ready, 0) : hipSuccess;
}
// collate.cpp: per-batch gauge union (ddr_collate_gauges)
ddr_status collate_gauges(int64_t n_conus, int64_t n_gauges, const int64_t* sub_off, const int32_t* rows,
                          const int32_t* cols, const int32_t* gage_idx, int32_t* active, int64_t* n_active,
                          int64_t* crow, int32_t* col, int64_t* nnz, int64_t* out_off, int32_t* out_idx,
                          int64_t out_idx_cap, int32_t* gage_c);
// devgraph.hip: the on-device builder (COO in device memory, work on `stream`) and host copies of
// what it keeps on the device
ddr_status build_graph_device(int64_t n, int64_t e, const int32_t* rows, const int32_t* cols,
                              const ddr_build_opts* opts, hipStream_t stream, Graph** out);
struct DevBuild;  // a device build between its two halves
ddr_status build_graph_device_begin(int64_t n, int64_t e, const int32_t* rows, const int32_t* cols,
                                    const ddr_build_opts* opts, hipStream_t stream, DevBuild** out);
ddr_status build_graph_device_finish(DevBuild* b, Graph** out);  // consumes b
void build_graph_device_cancel(DevBuild* b);
ddr_status collate_gauges_device(int64_t n_conus, int64_t n_gauges, int64_t e, const int32_t* rows,
                                 const int32_t* cols, const int32_t* gage_idx, int32_t* active, int64_t active_cap,
                                 int64_t* n_active, int32_t* rows_c, int32_t* cols_c, int64_t* nnz, int64_t* crow,
                                 int32_t* col, int64_t* out_off, int32_t* out_idx, int64_t out_idx_cap,
                                 int32_t* gage_c, hipStream_t stream);
ddr_status device_views_to_host(const Graph* g, int64_t* crow, int64_t* col, int64_t* down, int64_t* dist,
                                int64_t* basin, int64_t* block);
ddr_status device_schedule_to_host(const Graph* g, HostSchedule& H);
// Upload a host-built schedule (DDR_BUILD_HOST_ONLY) to the current device; no-op once uploaded.
ddr_status upload_schedule(Graph* g);
ddr_status upload_schedule_async(Graph* g, hipStream_t stream);

// Status block layout (device, zeroed before every launch): word 0 = timed-out hand-offs, word 1 =
// first failing block + 1, word 2 = forward ticket counter, word 3 = backward ticket counter.
// Workgroups take their logical block from the ticket counter (route.hip: take_ticket), so a
// running workgroup's producers are always running or finished: any grid size is deadlock-free.
constexpr int64_t kStatusBytes = 256;
constexpr int kStatusTicketFwd = 2;
constexpr int kStatusTicketBwd = 3;
constexpr int kStatusNaN = 4;  // DDR_FWD_CHECK_QPRIME: a NaN in the flow-scaled q' the window reads
// RouteArgs.flags bits beyond the public DDR_FWD_* flags
constexpr int32_t kFlagForceTimeout = 1 << 16;  // debug: every inter-workgroup wait times out
constexpr int32_t kFlagNoSteady = 1 << 17;      // debug / A/B: every tick through the general path
constexpr int32_t kFlagNoStorer = 1 << 18;      // debug / A/B: light blocks store from their compute waves
constexpr int32_t kFlagNoPlain = 1 << 19;       // debug / A/B: the general kernel instances, never the plain ones

}  // namespace ddr
