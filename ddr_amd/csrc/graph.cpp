// Host-side river-graph builder: validation, canonical CSR, dendritic structure, basin splitting,
// workgroup packing and the per-workgroup tick schedule; uploads the schedule to the device.
//
// Reference behaviour reproduced here:
//   * COO -> canonical CSR exactly as scipy.sparse.coo_matrix(...).tocsr() (rows sorted, columns
//     ascending) -- src/ddr/geodatazoo/merit.py:197-223, lynker_hydrofabric.py:198-224.
//   * lower-triangular / dendritic contract of the engine -- engine/src/ddr_engine/merit/build.py:94,105.
//   * the solve order of the reference triangular solve (utils.py:587-600): a reach's upstream
//     terms are accumulated in ascending column order (uplist is kept in that order).
//
// Schedule: every reach gets a tick offset off(i) = dmax(block) - dist_in_piece(i), so
// step t of reach i runs at tick t + off(i) and every edge inside a workgroup has a slack of exactly
// one tick ("as late as possible" wavefront).  Large basins are split into connected pieces whose
// inter-piece edges become cut edges exchanged through global memory.
//
// The piece-level half (pack_pieces, finalize_blocks) is shared with the on-device builder
// (devgraph.hip): both split the basins into the same pieces, number them the same way and hand the
// same piece table to the same packer, so a device build emits the host build's schedule bit for bit.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <memory>
#include <mutex>
#include <numeric>

#include "internal.h"

namespace ddr {

namespace {

template <typename T>
ddr_status upload(Graph* g, T** dst, const std::vector<T>& src) {
  size_t bytes = std::max<size_t>(src.size(), 1) * sizeof(T);
  void* p = nullptr;
  DDR_HIP(hipMalloc(&p, bytes));
  g->allocations.push_back(p);
  if (!src.empty()) DDR_HIP(hipMemcpy(p, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
  *dst = static_cast<T*>(p);
  return DDR_OK;
}

}  // namespace

// Stream-ordered upload (ddr_graph_build_async / ddr_graph_upload_async): every schedule array is packed
// into one pinned staging block and one pooled device block, one copy on `stream`, and the graph's ready
// event recorded behind it -- routing launches on any stream wait for that event (graph_ready); no
// device-wide synchronisation (hipMalloc / hipMemcpy of pageable memory have one each).
ddr_status upload_schedule_async(Graph* g, hipStream_t stream) {
  if (g->uploaded) return DDR_OK;
  HostSchedule& H = g->hs;
  DevSchedule& D = g->dev;
  size_t total = 0;
  auto room = [&](size_t n, size_t elem) { total = align16(total) + std::max<size_t>(n, 1) * elem; };
  room(g->blocks.size(), sizeof(BlockDesc));
  for (const std::vector<int32_t>* v : {&H.ref, &H.off, &H.upb, &H.upc, &H.dloc, &H.cut, &H.uplist, &H.xoff,
                                        &H.xlist, &H.v_edge, &H.v_off, &H.v_dloc, &H.cout_loc, &H.pos_of_ref,
                                        &H.block_of_pos, &H.rs_loc, &H.rs_ref})
    room(v->size(), sizeof(int32_t));
  total = align16(total);
  unsigned char* host = static_cast<unsigned char*>(pinned_get(total));
  if (!host) return fail(DDR_ERR_HIP, "graph upload: pinned host memory");
  unsigned char* dev = static_cast<unsigned char*>(device_get(total, stream));
  if (!dev) {
    pinned_put(host, stream);
    return fail(DDR_ERR_HIP, "graph upload: out of device memory");
  }
  g->async_allocations.push_back(dev);
  size_t o = 0;
  auto place = [&](const void* src, size_t n, size_t elem) {
    o = align16(o);
    if (n) std::memcpy(host + o, src, n * elem);
    void* d = dev + o;
    o += std::max<size_t>(n, 1) * elem;
    return d;
  };
  D.blocks = static_cast<BlockDesc*>(place(g->blocks.data(), g->blocks.size(), sizeof(BlockDesc)));
  auto put = [&](int32_t** dst, const std::vector<int32_t>& v) { *dst = static_cast<int32_t*>(place(v.data(), v.size(), 4)); };
  put(&D.ref, H.ref);
  put(&D.off, H.off);
  put(&D.upb, H.upb);
  put(&D.upc, H.upc);
  put(&D.dloc, H.dloc);
  put(&D.cut, H.cut);
  put(&D.uplist, H.uplist);
  put(&D.xoff, H.xoff);
  put(&D.xlist, H.xlist);
  put(&D.v_edge, H.v_edge);
  put(&D.v_off, H.v_off);
  put(&D.v_dloc, H.v_dloc);
  put(&D.cout_loc, H.cout_loc);
  put(&D.pos_of_ref, H.pos_of_ref);
  put(&D.block_of_pos, H.block_of_pos);
  put(&D.rs_loc, H.rs_loc);
  put(&D.rs_ref, H.rs_ref);
  const hipError_t ce = hipMemcpyAsync(dev, host, total, hipMemcpyHostToDevice, stream);
  // the staging block goes back to the pool at once: its event (recorded on `stream` behind the copy)
  // keeps it from reuse until the copy has read it -- a prefetcher holding many built graphs pins no host
  // memory per graph
  pinned_put(host, stream);
  DDR_HIP(ce);
  if (!g->ready) DDR_HIP(hipEventCreateWithFlags(&g->ready, hipEventDisableTiming));
  DDR_HIP(hipEventRecord(g->ready, stream));
  DDR_HIP(hipGetDevice(&g->device));
  g->uploaded = true;
  g->hs = HostSchedule{};
  return DDR_OK;
}

ddr_status upload_schedule(Graph* g) {
  if (g->uploaded) return DDR_OK;
  HostSchedule& H = g->hs;
  DevSchedule& D = g->dev;
  ddr_status st;
  if ((st = upload(g, &D.blocks, g->blocks))) return st;
  if ((st = upload(g, &D.ref, H.ref))) return st;
  if ((st = upload(g, &D.off, H.off))) return st;
  if ((st = upload(g, &D.upb, H.upb))) return st;
  if ((st = upload(g, &D.upc, H.upc))) return st;
  if ((st = upload(g, &D.dloc, H.dloc))) return st;
  if ((st = upload(g, &D.cut, H.cut))) return st;
  if ((st = upload(g, &D.uplist, H.uplist))) return st;
  if ((st = upload(g, &D.xoff, H.xoff))) return st;
  if ((st = upload(g, &D.xlist, H.xlist))) return st;
  if ((st = upload(g, &D.v_edge, H.v_edge))) return st;
  if ((st = upload(g, &D.v_off, H.v_off))) return st;
  if ((st = upload(g, &D.v_dloc, H.v_dloc))) return st;
  if ((st = upload(g, &D.cout_loc, H.cout_loc))) return st;
  if ((st = upload(g, &D.pos_of_ref, H.pos_of_ref))) return st;
  if ((st = upload(g, &D.block_of_pos, H.block_of_pos))) return st;
  if ((st = upload(g, &D.rs_loc, H.rs_loc))) return st;
  if ((st = upload(g, &D.rs_ref, H.rs_ref))) return st;
  DDR_HIP(hipGetDevice(&g->device));
  g->uploaded = true;
  g->hs = HostSchedule{};  // the device copy is the schedule from here on
  return DDR_OK;
}

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ---- the packer's plan (capacity, generations) ------------------------------------------------
ddr_status plan_init(int64_t n, int64_t bmax, const ddr_build_opts* opts, PackPlan& P) {
  int dev = 0, n_cu = 0;
  if (hipGetDevice(&dev) == hipSuccess) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess) n_cu = prop.multiProcessorCount;
  }
  P.device = dev;
  if (n_cu <= 0) n_cu = 256;
  const int bs = kBlockThreads;
  P.n = n;
  P.hard_cap = std::min<int64_t>(int64_t(bs) * kMaxKR, kDefaultBlockReaches);
  if (opts && opts->max_block_reaches > 0) P.hard_cap = std::min<int64_t>(int64_t(bs) * kMaxKR, opts->max_block_reaches);
  P.target = (opts && opts->target_blocks > 0) ? opts->target_blocks : int64_t(n_cu) * kBlocksPerCU;
  P.resident = (opts && opts->max_resident > 0) ? opts->max_resident : n_cu * kBlocksPerCU;
  // Capacity floor: one wave-slice per SIMD (4 x 64 reaches).  A tick costs ~0.66 us + 0.49 us per
  // slice on the busiest SIMD, so a light load (n well below 256 x 1024) is
  // cheapest spread thin over many workgroups, not packed into a few full ones.
  P.min_cap = std::min<int64_t>(kMinBlockCap, bs);
  P.cap = std::min<int64_t>(P.hard_cap, std::max<int64_t>(P.min_cap, (n + P.target - 1) / P.target));
  // ... rounded up to whole slices per SIMD (4 x 64 reaches) at light and medium loads: a tick costs
  // per slice on the busiest SIMD, so the rounding keeps that cost and makes fewer, larger pieces --
  // fewer cut edges and shorter block chains (routing of a C3 8-way shard 8.1 -> 7.2 ms, of C5's
  // giant-basin shard 57.6 -> 54.3 ms); at full load (C3, C5 on one GPU) it measured slower
  // (profiles/r02/ab_defer_early.txt)
#ifndef DDR_CAP_QUANT
#define DDR_CAP_QUANT 256
#endif
#ifndef DDR_CAP_QUANT_MAX
#define DDR_CAP_QUANT_MAX 2048
#endif
  if (DDR_CAP_QUANT > 1 && P.cap <= DDR_CAP_QUANT_MAX)
    P.cap = std::min<int64_t>(P.hard_cap, (P.cap + DDR_CAP_QUANT - 1) / DDR_CAP_QUANT * DDR_CAP_QUANT);
  P.cap_start = P.cap;
  P.steps = (opts && opts->steps_hint > 0) ? (double)opts->steps_hint : 8760.0;
  // exponent of the chain-pacing weight (T + L) / T (experiments: DDR_PACK_FAC_POW)
  P.fac_pow = getenv("DDR_PACK_FAC_POW") ? atof(getenv("DDR_PACK_FAC_POW")) : 1.0;
  // block capacity rounded down to a multiple of this many reaches: a tick costs per 256-reach
  // slice-per-SIMD unit, so at light loads (one reach per thread) a block of 513..523 reaches ticks at the
  // rate of 768 and loses the storer waves (<= 512) -- C3 8-way shard forward 3.15 -> 2.88 ms; at full
  // load (C3, C5 on one GPU) no gain, off (profiles/r04/ab_r04.txt; DDR_PACK_QUANT overrides)
  P.pack_quant = getenv("DDR_PACK_QUANT") ? atol(getenv("DDR_PACK_QUANT")) : (P.cap <= kBlockThreads ? 256 : 1);
  // Split threshold (pieces up to scap_pct % of the capacity): with a dominant basin (C4/C5: 0.35 N)
  // its chain of pieces is the critical path, and pieces at 80 % leave the packer room to give chain
  // blocks fewer reaches; without one (C3: 256 basins of at most 2 % of N) pieces at the full
  // capacity mean fewer cut edges (C3 38.7 -> 36.5 ms per step; C5 at 100 %: 138 -> 149 ms;
  // profiles/r02/ab_defer_early.txt)
  P.scap_pct = bmax * 10 < n ? 100 : 80;
#ifdef DDR_SCAP_PCT
  P.scap_pct = DDR_SCAP_PCT;
#endif
  P.weighted = true;
  P.gen = 1;
  // A network beyond ~97 % of one resident generation (resident x hard_cap reaches: packing never fills
  // every block) starts at the generation count it needs, instead of reaching it through the failed
  // one-generation variants (a ~1.07M-reach C3 batch: 1 split pass instead of 4 -- each a device
  // round trip in the on-device builder)
  const int64_t per_gen_cap = P.resident * P.hard_cap * 97 / 100;
  if (n > per_gen_cap) {
    P.gen = (n + per_gen_cap - 1) / per_gen_cap;
    const int64_t per_gen = std::min<int64_t>(P.target, P.resident) * P.gen;
    P.cap = std::min<int64_t>(P.hard_cap, std::max<int64_t>(P.min_cap, (n + per_gen - 1) / per_gen));
  }
  P.dbg = getenv("DDR_DEBUG_PART") != nullptr;
  return DDR_OK;
}

// ---- packing of the pieces into workgroups ----------------------------------------------------
// Workgroups take their logical block index from a ticket counter in block order (route.hip:
// take_ticket), and blocks are numbered by piece height, so a running workgroup's producers are
// running or done: a schedule with more blocks than resident workgroups is still deadlock-free.
// The packer first tries to fit one resident generation (all blocks co-resident, fully time-
// pipelined): path-weighted packing, then unweighted; failing both it packs gen x resident
// smaller blocks (every extra generation costs about T more ticks of the blocks it holds).
ddr_status pack_pieces(PackPlan& P, const PieceTable& pt, PackResult& R, int* outcome) {
  const size_t np = pt.count();
  // virtual inflows deepen the consuming piece by one tick; piece heights (children first: a child
  // piece is numbered after its parent)
  std::vector<int64_t> dmax(pt.dmax), height(np, 0);
  for (int64_t p = (int64_t)np - 1; p >= 0; --p) {
    const int64_t q = pt.parent[p];
    if (q >= 0) {
      dmax[q] = std::max<int64_t>(dmax[q], pt.dloc_down[p] + 1);
      height[q] = std::max(height[q], height[p] + 1);
    }
  }
  int64_t ncut = 0;
  for (size_t p = 0; p < np; ++p) ncut += (pt.parent[p] >= 0);
  // Packing: pieces of equal height share blocks (so the block dependency graph is a DAG),
  // worst-fit by weight.  The blocks of a split basin progress at the pace of their slowest
  // member (a consumer waits for its producers, forward and backward alike), so every block
  // holding a piece of a long path needs T + (path length) ticks, not T + dmax: a piece is
  // weighted by (T + L) / T with L the longest source-to-outlet path through its root, plus one
  // chunk per inter-block hop on it.  Chain blocks get fewer reaches and tick faster (a tick
  // costs in proportion to the reaches of a workgroup).
  std::vector<int64_t> hops_down(np, 0);
  for (size_t p = 0; p < np; ++p)  // parents before children (numbering order)
    if (pt.parent[p] >= 0) hops_down[p] = hops_down[pt.parent[p]] + 1;
  std::vector<double> fac(np);
  double wsum = 0.0;
  for (size_t p = 0; p < np; ++p) {
    const double L = (double)(pt.ht_root[p] + pt.dist_root[p] + kChunk * (hops_down[p] + height[p]));
    fac[p] = P.weighted ? std::pow((P.steps + L) / P.steps, P.fac_pow) : 1.0;
  }
  for (size_t p = 0; p < np; ++p) wsum += (double)pt.size[p] * fac[p];
  // A block's tick budget is set by its most constrained piece: capacity capw / max factor.
  // Pieces are taken by factor (descending) so blocks gather pieces of similar factor; capw is
  // the smallest (1 % steps) that packs into the target number of workgroups.
  std::vector<int64_t> order(np), block_of_piece(np), load;
  std::vector<double> bcap;
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
    if (height[a] != height[b]) return height[a] < height[b];
    if (fac[a] != fac[b]) return fac[a] > fac[b];
    return pt.size[a] > pt.size[b];
  });
  const int64_t limit = ncut > 0 ? std::min<int64_t>(P.target, P.resident) * P.gen : P.target;
  // capw_k = capw_0 * 1.01^k; beyond k_sat (capw / fac >= hard_cap for every piece) the packing no
  // longer changes.  The block count falls with k, so the smallest k that fits is binary-searched
  // (a handful of packing passes instead of one per 1 % step).
  double maxfac = 1.0;
  for (double f : fac) maxfac = std::max(maxfac, f);
  const double capw0 = wsum / (double)limit;
  // light loads (capacity <= half a workgroup, one reach per thread): no block above half a workgroup while
  // the capacity stays there -- a block of 513+ reaches has no idle upper waves (storer / import / x-helper
  // waves, route.hip) and three routing waves per SIMD, and sets the kernel's pace (a C3 8-way shard's
  // five 700-reach blocks: 8.15 ms against 6.9-7.5 for the shards without); the capacity growth below
  // lifts the clamp when the blocks do not fit otherwise
  const bool light_clamp = !getenv("DDR_PACK_NO_LIGHT_CLAMP") && P.cap <= kBlockThreads / 2;
  const double bc_max = light_clamp ? (double)(kBlockThreads / 2) : (double)P.hard_cap;
  auto pack = [&](int k) {
    const double capw = capw0 * std::pow(1.01, (double)k);
    load.clear();
    bcap.clear();
    size_t hstart = 0;  // first block of the current height class
    int64_t curh = -1;
    for (int64_t p : order) {
      if (height[p] != curh) {
        curh = height[p];
        hstart = load.size();
      }
      int64_t best = -1;
      const int64_t sz = pt.size[p];
      for (size_t b = hstart; b < load.size(); ++b)
        if ((double)(load[b] + sz) <= bcap[b] && (best < 0 || load[b] < load[best])) best = (int64_t)b;
      if (best < 0) {
        best = (int64_t)load.size();
        load.push_back(0);
        double bc = std::min<double>(bc_max, std::max<double>((double)sz, capw / fac[p]));
        if (P.pack_quant > 1 && bc >= (double)P.pack_quant)
          bc = std::max<double>((double)sz, std::floor(bc / (double)P.pack_quant) * (double)P.pack_quant);
        bcap.push_back(bc);
      }
      load[best] += sz;
      block_of_piece[p] = best;
    }
    return (int64_t)load.size();
  };
  const int k_sat = std::max(0, (int)std::ceil(std::log((double)P.hard_cap * maxfac / capw0) / std::log(1.01)));
  int npass = 1;
  if (pack(0) > limit) {
    int lo = 0, hi = k_sat;  // pack(lo) > limit; find the smallest k in (lo, hi] with pack(k) <= limit
    ++npass;
    if (pack(hi) <= limit) {
      while (hi - lo > 1) {
        const int mid = (lo + hi) / 2;
        ++npass;
        if (pack(mid) <= limit) hi = mid;
        else lo = mid;
      }
      ++npass;
      pack(hi);
    }
  }
  const int64_t nblocks = (int64_t)load.size();
  if (P.dbg) {
    fprintf(stderr, "[part] pack passes %d\n", npass);
    fprintf(stderr, "[part] cap %ld hard %ld gen %ld weighted %d pieces %zu blocks %ld cut %ld\n", (long)P.cap,
            (long)P.hard_cap, (long)P.gen, (int)P.weighted, np, (long)nblocks, (long)ncut);
  }
  // LDS of the fp32 kernels at the resulting slot / ring sizes; shrink the capacity if a workgroup
  // would no longer fit on a CU
  std::vector<int64_t> bv(nblocks, 0), bc(nblocks, 0), bx(nblocks, 0);
  for (size_t p = 0; p < np; ++p) {
    bx[block_of_piece[p]] += pt.xl[p];
    if (pt.parent[p] >= 0) {
      bv[block_of_piece[pt.parent[p]]]++;
      bc[block_of_piece[p]]++;
    }
  }
  int64_t ms = 0, mv = 0, mc = 0, mx = 0;
  for (int64_t b = 0; b < nblocks; ++b) {
    ms = std::max(ms, load[b] + bv[b]);
    mv = std::max(mv, bv[b]);
    mc = std::max(mc, bc[b]);
    mx = std::max(mx, bx[b]);
  }
  int64_t maxl = 0;
  for (int64_t b = 0; b < nblocks; ++b) maxl = std::max(maxl, load[b]);
  const size_t need = std::max(route_lds_bytes(route_slot_stride((int)ms), mv, mc, mx, false, 4, kr_of_load(maxl)),
                               route_lds_bytes(route_slot_stride((int)ms), mv, mc, mx, true, 4, kr_of_load(maxl)));
  if (P.dbg) fprintf(stderr, "[part]   slots %ld virt %ld cout %ld xl %ld lds %zu\n", (long)ms, (long)mv, (long)mc, (long)mx, need);
  // (a count failure at the capacity ceiling of the unweighted packing goes to more generations:
  // shrinking the capacity for LDS would only add blocks)
  const bool count_dead = ncut > 0 && nblocks > limit && P.cap >= P.hard_cap && !P.weighted;
  if (!count_dead && (need > kLdsBudget || mx >= kMaxConfluenceList)) {
    if (P.hard_cap <= 64) return fail(DDR_ERR_CAPACITY, "workgroup LDS budget exceeded");
    P.hard_cap -= std::max<int64_t>(1, P.hard_cap / 32);
    P.cap = std::min(P.cap, P.hard_cap);
    *outcome = kPackResplit;
    return DDR_OK;
  }
  if (ncut > 0 && nblocks > limit) {
    *outcome = kPackResplit;
    if (P.cap < P.hard_cap) {
      const int64_t grown = std::min<int64_t>(P.hard_cap, P.cap + P.cap / 32 + 1);
      // light loads: before the capacity leaves half a workgroup (blocks of 513+ reaches lose their idle
      // waves, see light_clamp), the unweighted packing at this capacity (C3 8-way shard 3: 7.72 ms with
      // one 530-reach block, 7.35 ms unweighted at 512, 8.16 ms before the clamp; profiles/r04/ab_r04.txt)
      if (light_clamp && P.weighted && grown > kBlockThreads / 2) {
        P.weighted = false;
        return DDR_OK;
      }
      P.cap = grown;
      return DDR_OK;
    }
    if (P.weighted) {
      P.weighted = false;
      P.cap = P.cap_start;
      return DDR_OK;
    }
    if (++P.gen > 64) return fail(DDR_ERR_CAPACITY, "graph cannot be packed into workgroups");
    P.weighted = true;
    const int64_t per_gen = std::min<int64_t>(P.target, P.resident) * P.gen;
    P.cap = std::min<int64_t>(P.hard_cap, std::max<int64_t>(P.min_cap, (P.n + per_gen - 1) / per_gen));
    return DDR_OK;
  }
  *outcome = kPackDone;
  R.nblocks = nblocks;
  R.ncut = ncut;
  R.block_of_piece = std::move(block_of_piece);
  R.load = std::move(load);
  R.bv = std::move(bv);
  R.bc = std::move(bc);
  R.bx = std::move(bx);
  R.bdmax.assign(nblocks, 0);
  for (size_t p = 0; p < np; ++p) R.bdmax[R.block_of_piece[p]] = std::max(R.bdmax[R.block_of_piece[p]], dmax[p]);
  return DDR_OK;
}

// Block descriptors and the graph-wide sizes from the packing (counts only: the per-reach arrays are
// emitted by the host or the device builder in the same order -- blocks contiguous, inside a block by
// (tick offset, reference index); a block's cut edges, virtual inflows and confluence lists in that
// position order).
ddr_status finalize_blocks(Graph* g, const PackPlan& P, const PackResult& R) {
  const int64_t nb = R.nblocks;
  g->generations = P.gen;
  g->resident = P.resident;
  g->n_cut = R.ncut;
  g->blocks.assign(nb, BlockDesc{});
  int64_t p0 = 0, pre_dn = 0, v0 = 0, c0 = 0, x0 = 0, max_load = 0;
  g->max_slots = g->max_virt = g->max_cout = g->max_xl = 0;
  g->max_block_depth = 0;
  for (int64_t b = 0; b < nb; ++b) {
    BlockDesc& B = g->blocks[b];
    B.pos0 = (int32_t)p0;
    B.nloc = (int32_t)R.load[b];
    B.virt0 = (int32_t)v0;
    B.nvirt = (int32_t)R.bv[b];
    B.cout0 = (int32_t)c0;
    B.ncout = (int32_t)R.bc[b];
    B.dmax = (int32_t)R.bdmax[b];
    B.nxl = (int32_t)R.bx[b];
    B.pre_dn = pre_dn;
    B.xl0 = (int32_t)x0;
    B.pad = 0;
    g->max_xl = std::max<int>(g->max_xl, B.nxl);
    g->max_slots = std::max<int>(g->max_slots, B.nloc + B.nvirt);
    g->max_virt = std::max<int>(g->max_virt, B.nvirt);
    g->max_cout = std::max<int>(g->max_cout, B.ncout);
    g->max_block_depth = std::max<int64_t>(g->max_block_depth, B.dmax + 1);
    max_load = std::max<int64_t>(max_load, R.load[b]);
    pre_dn += R.bdmax[b] * R.load[b];
    p0 += R.load[b];
    v0 += R.bv[b];
    c0 += R.bc[b];
    x0 += R.bx[b];
  }
  g->sum_dn = pre_dn;
  g->max_nloc = (int)max_load;
  g->n_xlist = x0;
  g->kr = kr_of_load(max_load);
  if (g->max_virt > kBlockThreads || g->max_cout > kBlockThreads)
    return fail(DDR_ERR_CAPACITY, "too many inter-workgroup edges in one workgroup");
  return DDR_OK;
}

// FNV-1a over the schedule arrays (DDR_DEBUG_PART): the host and device builds print it.
unsigned long long schedule_fingerprint(const HostSchedule& H) {
  unsigned long long h = 1469598103934665603ull;
  auto mix = [&](const std::vector<int32_t>& v) {
    for (int32_t x : v) h = (h ^ (unsigned)x) * 1099511628211ull;
  };
  mix(H.ref); mix(H.off); mix(H.upb); mix(H.upc); mix(H.dloc); mix(H.cut); mix(H.xoff); mix(H.uplist); mix(H.xlist);
  mix(H.v_edge); mix(H.v_off); mix(H.v_dloc); mix(H.cout_loc);
  return h;
}

ddr_status build_graph(int64_t n, int64_t e, const int32_t* rows, const int32_t* cols,
                       const ddr_build_opts* opts, Graph** out) {
  if (n <= 0) return fail(DDR_ERR_ARG, "graph must have at least one reach");
  if (n >= (int64_t(1) << 31) - 1) return fail(DDR_ERR_ARG, "graph too large for int32 reach ids");
  if (e < 0 || (e > 0 && (!rows || !cols))) return fail(DDR_ERR_ARG, "bad COO arrays");
  auto g = std::make_unique<Graph>();
  g->n = n;
  const bool dbg = getenv("DDR_DEBUG_PART") != nullptr;
  double tp = now_ms();
  auto phase = [&](const char* what) {
    if (!dbg) return;
    const double t = now_ms();
    fprintf(stderr, "[part] %-10s %8.2f ms\n", what, t - tp);
    tp = t;
  };
  // ---- validation + canonical CSR (counting sort by row, then ascending columns) ----------
  std::vector<int64_t> cnt(n + 1, 0);
  for (int64_t k = 0; k < e; ++k) {
    int64_t r = rows[k], c = cols[k];
    if (r < 0 || r >= n || c < 0 || c >= n) return fail(DDR_ERR_ARG, "COO index out of range");
    if (c >= r)
      return fail(DDR_ERR_NOT_LOWER, "adjacency entry (" + std::to_string(r) + "," + std::to_string(c) +
                                         ") is not strictly lower triangular (network not topologically sorted)");
    cnt[r + 1]++;
  }
  for (int64_t i = 0; i < n; ++i) cnt[i + 1] += cnt[i];
  std::vector<int64_t> col(e), fill(cnt.begin(), cnt.end() - 1);
  for (int64_t k = 0; k < e; ++k) col[fill[rows[k]]++] = cols[k];
  for (int64_t i = 0; i < n; ++i) {  // rows hold a few entries: insertion sort
    for (int64_t k = cnt[i] + 1; k < cnt[i + 1]; ++k) {
      const int64_t v = col[k];
      int64_t j = k;
      for (; j > cnt[i] && col[j - 1] > v; --j) col[j] = col[j - 1];
      col[j] = v;
    }
  }
  for (int64_t i = 0; i < n; ++i)
    for (int64_t k = cnt[i] + 1; k < cnt[i + 1]; ++k)
      if (col[k] == col[k - 1])
        return fail(DDR_ERR_DUPLICATE, "duplicate edge (" + std::to_string(i) + "," + std::to_string(col[k]) + ")");
  g->nnz = e;
  // ---- dendritic structure ---------------------------------------------------------------
  g->down.assign(n, -1);
  for (int64_t i = 0; i < n; ++i)
    for (int64_t k = cnt[i]; k < cnt[i + 1]; ++k) {
      int64_t j = col[k];
      if (g->down[j] >= 0)
        return fail(DDR_ERR_NOT_DENDRITIC, "reach " + std::to_string(j) + " drains into two reaches");
      g->down[j] = i;
    }
  g->dist.assign(n, 0);
  g->basin.assign(n, 0);
  for (int64_t i = n - 1; i >= 0; --i) {
    int64_t d = g->down[i];
    g->dist[i] = d < 0 ? 0 : g->dist[d] + 1;
    g->basin[i] = d < 0 ? i : g->basin[d];
  }
  g->max_depth = n ? *std::max_element(g->dist.begin(), g->dist.end()) + 1 : 0;
  for (int64_t i = 0; i < n; ++i) g->n_basins += (g->down[i] < 0);
  phase("csr+tree");

  // Splitting works on full-subtree sizes and heights: sub(i) = reaches draining through i,
  // ht(i) = longest path from i up to a source.
  std::vector<int32_t> sub(n, 1), ht(n, 0);
  for (int64_t i = 0; i < n; ++i)
    for (int64_t k = cnt[i]; k < cnt[i + 1]; ++k) {
      sub[i] += sub[col[k]];
      ht[i] = std::max(ht[i], ht[col[k]] + 1);
    }
  int64_t bmax = 0;
  {
    std::vector<int32_t> bsz(n, 0);
    for (int64_t i = 0; i < n; ++i) bmax = std::max<int64_t>(bmax, ++bsz[g->basin[i]]);
  }
  PackPlan plan;
  ddr_status st = plan_init(n, bmax, opts, plan);
  if (st) return st;
  g->device = plan.device;
  std::vector<int32_t> piece(n), resid(n), stem(n), dloc_piece(n);
  std::vector<char> is_root(n);
  std::vector<int64_t> others;
  PieceTable pt;
  PackResult pr;
  for (;;) {
    // Stem-preserving split (bottom-up).  A reach whose subtree exceeds the capacity keeps its
    // deepest child (the main stem: every block boundary crossed along the longest flow path adds
    // a hand-off to the critical path) and absorbs other children, smallest first, while the
    // piece's tributary mass stays within cap - lseg, so every piece carries a stem stretch of at
    // least lseg reaches.  The stem child is cut only when the piece is full.
    // Pieces of split basins are kept below the block capacity: they land in blocks on long
    // chains, whose packing weight is up to ~(T + depth) / T times their size.
    const int64_t scap = plan.scap();
    const int64_t lseg = scap / 8;
    std::fill(is_root.begin(), is_root.end(), 0);
    for (int64_t i = 0; i < n; ++i) {
      const int64_t k0 = cnt[i], k1 = cnt[i + 1];
      if (sub[i] <= scap || k0 == k1) {
        resid[i] = sub[i];
        stem[i] = ht[i] + 1;
        continue;
      }
      int64_t dc = col[k0];
      for (int64_t k = k0 + 1; k < k1; ++k) {
        const int64_t c = col[k];
        if (ht[c] > ht[dc] || (ht[c] == ht[dc] && sub[c] > sub[dc])) dc = c;
      }
      int64_t base = 1 + resid[dc], trib = resid[dc] - stem[dc];
      const bool keep = base <= scap;
      if (!keep) {
        is_root[dc] = 1;
        base = 1;
        trib = 0;
      }
      others.clear();
      for (int64_t k = k0; k < k1; ++k)
        if (col[k] != dc) others.push_back(col[k]);
      std::stable_sort(others.begin(), others.end(), [&](int64_t a, int64_t b) { return resid[a] < resid[b]; });
      int64_t acc = 0;
      for (int64_t c : others) {
        if (trib + acc + resid[c] <= scap - lseg && base + acc + resid[c] <= scap) acc += resid[c];
        else is_root[c] = 1;
      }
      resid[i] = base + acc;
      stem[i] = keep ? 1 + stem[dc] : 1;
    }
    // pieces numbered by descending root index (a child piece after its parent)
    pt = PieceTable{};
    for (int64_t i = n - 1; i >= 0; --i) {
      int64_t d = g->down[i];
      if (d < 0 || is_root[i]) {
        is_root[i] = 1;
        piece[i] = (int32_t)pt.count();
        pt.root.push_back(i);
        pt.size.push_back(0);
        pt.dmax.push_back(0);
        pt.xl.push_back(0);
        pt.parent.push_back(d < 0 ? -1 : piece[d]);
        pt.dloc_down.push_back(d < 0 ? 0 : dloc_piece[d]);
        pt.ht_root.push_back(ht[i]);
        pt.dist_root.push_back(g->dist[i]);
        dloc_piece[i] = 0;
      } else {
        piece[i] = piece[d];
        dloc_piece[i] = dloc_piece[d] + 1;
      }
      const int64_t p = piece[i];
      pt.size[p]++;
      if (cnt[i + 1] - cnt[i] > 2) pt.xl[p] += cnt[i + 1] - cnt[i];
      pt.dmax[p] = std::max<int64_t>(pt.dmax[p], dloc_piece[i]);
    }
    phase("split");
    int outcome = kPackDone;
    if ((st = pack_pieces(plan, pt, pr, &outcome))) return st;
    phase("pack");
    if (outcome == kPackResplit) continue;
    break;
  }
  g->n_pieces = (int64_t)pt.count();
  if ((st = finalize_blocks(g.get(), plan, pr))) return st;
  const int64_t nblocks = pr.nblocks;
  // ---- emit the schedule -----------------------------------------------------------------
  g->block_of.assign(n, 0);
  for (int64_t i = 0; i < n; ++i) g->block_of[i] = pr.block_of_piece[piece[i]];
  const std::vector<int64_t>& bdmax = pr.bdmax;
  std::vector<int32_t> offv(n);
  for (int64_t i = 0; i < n; ++i) offv[i] = bdmax[g->block_of[i]] - dloc_piece[i];
  // internal order (block, tick offset, reference index): two stable counting sorts over the
  // ascending reach ids, by offset and then by block (O(n), no comparison sort)
  std::vector<int64_t> bstart(nblocks + 1, 0);
  std::vector<int32_t> order_all(n);
  {
    int64_t omax = 0;
    for (int64_t b = 0; b < nblocks; ++b) omax = std::max(omax, bdmax[b]);
    std::vector<int64_t> oc(omax + 2, 0);
    for (int64_t i = 0; i < n; ++i) oc[offv[i] + 1]++;
    for (int64_t o = 0; o <= omax; ++o) oc[o + 1] += oc[o];
    std::vector<int32_t> by_off(n);
    for (int64_t i = 0; i < n; ++i) by_off[oc[offv[i]]++] = (int32_t)i;
    for (int64_t i = 0; i < n; ++i) bstart[g->block_of[i] + 1]++;
    for (int64_t b = 0; b < nblocks; ++b) bstart[b + 1] += bstart[b];
    std::vector<int64_t> fillb(bstart.begin(), bstart.end() - 1);
    for (int64_t j = 0; j < n; ++j) {
      const int32_t i = by_off[j];
      order_all[fillb[g->block_of[i]]++] = i;
    }
  }
  phase("members");
  std::vector<int32_t> pos(n), local(n);
  HostSchedule& H = g->hs;
  H = HostSchedule{};
  std::vector<int32_t>&ref = H.ref, &offs = H.off, &upb = H.upb, &upc = H.upc, &dl = H.dloc, &cut = H.cut,
                      &xoff = H.xoff, &uplist = H.uplist, &xlist = H.xlist, &v_edge = H.v_edge, &v_off = H.v_off,
                      &v_dloc = H.v_dloc, &cout_loc = H.cout_loc;
  ref.resize(n);
  offs.resize(n);
  upb.resize(n);
  upc.resize(n);
  dl.resize(n);
  cut.assign(n, -1);
  xoff.assign(n, -1);
  std::vector<int32_t> edge_id(n, -1);
  for (int64_t P = 0; P < n; ++P) {
    pos[order_all[P]] = (int32_t)P;
    local[order_all[P]] = (int32_t)(P - bstart[g->block_of[order_all[P]]]);
  }
  // Cut edges are numbered in (block, local position) order, i.e. by their index in cout_loc: the
  // forward kernel derives a cut reach's granule row from B.cout0 + its rank among the block's
  // cut reaches (route.hip), with no table load in the tick.
  int64_t eid = 0;
  for (int64_t P = 0; P < n; ++P) {
    const int32_t i = order_all[P];
    if (g->down[i] >= 0 && g->block_of[g->down[i]] != g->block_of[i]) edge_id[i] = (int32_t)eid++;
  }
  for (int64_t b = 0; b < nblocks; ++b) {
    const BlockDesc& B = g->blocks[b];
    for (int64_t r = 0; r < B.nloc; ++r) {
      const int64_t P = B.pos0 + r;
      const int64_t i = order_all[P];
      ref[P] = (int32_t)i;
      offs[P] = offv[i];
      upb[P] = (int32_t)uplist.size();
      upc[P] = (int32_t)(cnt[i + 1] - cnt[i]);
      for (int64_t k = cnt[i]; k < cnt[i + 1]; ++k) {
        int64_t j = col[k];
        if (g->block_of[j] == b) {
          uplist.push_back(local[j]);
        } else {
          // virtual inflow of cut edge j -> i
          uplist.push_back((int32_t)(B.nloc + (v_edge.size() - B.virt0)));
          v_edge.push_back(edge_id[j]);
          v_off.push_back(offv[i] - 1);
          v_dloc.push_back((int32_t)r);
        }
      }
      if (upc[P] > 2) {
        // confluence list: [c, u1, ..., u_{c-1}] at xoff (block-local), see route.hip pack_up
        xoff[P] = (int32_t)(xlist.size() - B.xl0);
        xlist.push_back(upc[P]);
        for (int32_t k = 1; k < upc[P]; ++k) xlist.push_back(uplist[upb[P] + k]);
      }
      const int64_t d = g->down[i];
      dl[P] = (d >= 0 && g->block_of[d] == b) ? local[d] : -1;
      if (d >= 0 && g->block_of[d] != b) {
        cut[P] = edge_id[i];
        cout_loc.push_back((int32_t)r);
      }
    }
  }
  phase("emit");
  if (dbg) fprintf(stderr, "[part] schedule fingerprint %016llx\n", schedule_fingerprint(H));
  // reference-order views for the q' gather: pos_of_ref, block_of_pos, and per block its local
  // indices in ascending reference order (a stable counting sort of the reach ids by block)
  H.pos_of_ref.resize(n);
  H.block_of_pos.resize(n);
  H.rs_loc.resize(n);
  H.rs_ref.resize(n);
  {
    std::vector<int64_t> fillb(bstart.begin(), bstart.end() - 1);
    for (int64_t i = 0; i < n; ++i) {
      H.pos_of_ref[i] = pos[i];
      H.block_of_pos[pos[i]] = (int32_t)g->block_of[i];
      const int64_t k = fillb[g->block_of[i]]++;
      H.rs_ref[k] = (int32_t)i;
      H.rs_loc[k] = local[i];
    }
  }
  phase("views");
  g->crow = std::move(cnt);
  g->col = std::move(col);
  if (!(opts && (opts->flags & DDR_BUILD_HOST_ONLY))) {
    if ((st = upload_schedule(g.get()))) return st;
    phase("upload");
  }
  *out = g.release();
  return DDR_OK;
}

// The device builder's memory is freed stream-ordered on `stream` (after the work queued there, e.g. the
// routing launches that used the graph): no device-wide synchronisation per training batch.  The host
// builder's arrays (hipMalloc) go through hipFree, which waits for the device.
void destroy_graph(Graph* g, hipStream_t stream) {
  if (!g) return;
  for (void* p : g->allocations) (void)hipFree(p);
  if (g->ready) (void)hipStreamWaitEvent(stream, g->ready, 0);  // the build's last work precedes the free
  for (void* p : g->async_allocations) device_put(p, stream);
  // the build's uploads read the staging block: reusable once `stream` has passed the build
  if (g->staging) pinned_put(g->staging, stream);
  if (g->ready) (void)hipEventDestroy(g->ready);
  delete g;
}

namespace {
// One pool for pinned host blocks (device = -1) and device blocks (device id).  Blocks are kept for reuse
// (hipHostFree and hipFree synchronise with the device) until ddr_pool_trim releases the idle ones; sizes
// are rounded up to classes of 8 steps per power of two (at most 1/8 over the request past 2 KiB).
struct PoolBlock {
  void* p = nullptr;
  size_t bytes = 0;
  int device = -1;
  hipEvent_t ev = nullptr;  // recorded at return
  bool out = false;         // handed out
};
std::mutex g_pool_mu;
std::vector<PoolBlock> g_pool;

size_t size_class(size_t bytes) {
  if (bytes <= 2048) {
    size_t cls = 256;
    while (cls < bytes) cls <<= 1;
    return cls;
  }
  size_t top = 2048;
  while (top * 2 < bytes) top <<= 1;  // top < bytes <= 2 top
  const size_t step = top / 8;
  return (bytes + step - 1) / step * step;
}

void pool_put(void* p, hipStream_t s) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (PoolBlock& b : g_pool) {
    if (b.p != p) continue;
    if (!b.ev) (void)hipEventCreateWithFlags(&b.ev, hipEventDisableTiming);
    if (b.ev && hipEventRecord(b.ev, s) != hipSuccess) {
      (void)hipEventDestroy(b.ev);  // not recordable: wait here rather than hand out a block in use
      b.ev = nullptr;
      (void)hipStreamSynchronize(s);
    }
    b.out = false;
    return;
  }
}
}  // namespace

void* pinned_get(size_t bytes) {
  const size_t cls = size_class(bytes);
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (PoolBlock& b : g_pool) {
    if (b.out || b.device != -1 || b.bytes != cls) continue;
    if (b.ev && hipEventQuery(b.ev) != hipSuccess) continue;  // still read by queued copies
    b.out = true;
    return b.p;
  }
  void* p = nullptr;
  if (hipHostMalloc(&p, cls, hipHostMallocDefault) != hipSuccess) return nullptr;
  PoolBlock b;
  b.p = p;
  b.bytes = cls;
  b.out = true;
  g_pool.push_back(b);
  return p;
}
void pinned_put(void* p, hipStream_t s) { pool_put(p, s); }

void* device_get(size_t bytes, hipStream_t s) {
  const size_t cls = size_class(bytes);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (PoolBlock& b : g_pool) {
    if (b.out || b.device != dev || b.bytes != cls) continue;
    // the last user's work (queued on its stream) precedes this one's, without a host wait
    if (b.ev && hipStreamWaitEvent(s, b.ev, 0) != hipSuccess) continue;
    b.out = true;
    return b.p;
  }
  void* p = nullptr;
  if (hipMalloc(&p, cls) != hipSuccess) return nullptr;
  PoolBlock b;
  b.p = p;
  b.bytes = cls;
  b.device = dev;
  b.out = true;
  g_pool.push_back(b);
  return p;
}
void device_put(void* p, hipStream_t s) { pool_put(p, s); }

int64_t pool_trim() {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  int64_t freed = 0;
  std::vector<PoolBlock> keep;
  for (PoolBlock& b : g_pool) {
    // a block handed out, or one whose last user's queued work has not finished, stays
    if (b.out || (b.ev && hipEventQuery(b.ev) != hipSuccess)) {
      keep.push_back(b);
      continue;
    }
    if (b.ev) (void)hipEventDestroy(b.ev);
    if (b.device < 0) (void)hipHostFree(b.p);
    else (void)hipFree(b.p);
    freed += (int64_t)b.bytes;
  }
  g_pool.swap(keep);
  return freed;
}

}  // namespace ddr
