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
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <memory>
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

struct Piece {
  int64_t root;
  int64_t size = 0;
  int64_t height = 0;
  int64_t dmax = 0;  // max in-piece dist including virtual inflows
  int64_t xl = 0;    // confluence-list entries (reaches with more than two inflows, route.hip)
};

}  // namespace

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

ddr_status build_graph(int64_t n, int64_t e, const int32_t* rows, const int32_t* cols,
                       const ddr_build_opts* opts, Graph** out) {
  if (n <= 0) return fail(DDR_ERR_ARG, "graph must have at least one reach");
  if (n >= (int64_t(1) << 31) - 1) return fail(DDR_ERR_ARG, "graph too large for int32 reach ids");
  if (e < 0 || (e > 0 && (!rows || !cols))) return fail(DDR_ERR_ARG, "bad COO arrays");
  auto g = std::make_unique<Graph>();
  g->n = n;
  const bool dbg = getenv("DDR_DEBUG_PART") != nullptr;
  auto tnow = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  double tp = tnow();
  auto phase = [&](const char* what) {
    if (!dbg) return;
    const double t = tnow();
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

  // ---- partition: split basins larger than cap into connected pieces ---------------------
  int dev = 0, n_cu = 0, resident = 0;
  if (hipGetDevice(&dev) == hipSuccess) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess) n_cu = prop.multiProcessorCount;
  }
  g->device = dev;
  if (n_cu <= 0) n_cu = 256;
  const int bs = kBlockThreads;
  int64_t hard_cap = std::min<int64_t>(int64_t(bs) * kMaxKR, kDefaultBlockReaches);
  if (opts && opts->max_block_reaches > 0) hard_cap = std::min<int64_t>(int64_t(bs) * kMaxKR, opts->max_block_reaches);
  int64_t target = (opts && opts->target_blocks > 0) ? opts->target_blocks : int64_t(n_cu) * kBlocksPerCU;
  resident = (opts && opts->max_resident > 0) ? opts->max_resident : n_cu * kBlocksPerCU;
  // Capacity floor: one wave-slice per SIMD (4 x 64 reaches).  A tick costs ~0.66 us + 0.49 us per
  // slice on the busiest SIMD, so a light load (n well below 256 x 1024) is
  // cheapest spread thin over many workgroups, not packed into a few full ones.
  const int64_t min_cap = std::min<int64_t>(kMinBlockCap, bs);
  int64_t cap = std::min<int64_t>(hard_cap, std::max<int64_t>(min_cap, (n + target - 1) / target));
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
  if (DDR_CAP_QUANT > 1 && cap <= DDR_CAP_QUANT_MAX)
    cap = std::min<int64_t>(hard_cap, (cap + DDR_CAP_QUANT - 1) / DDR_CAP_QUANT * DDR_CAP_QUANT);
  const double steps = (opts && opts->steps_hint > 0) ? (double)opts->steps_hint : 8760.0;
  // exponent of the chain-pacing weight (T + L) / T (experiments: DDR_PACK_FAC_POW)
  const double fac_pow = getenv("DDR_PACK_FAC_POW") ? atof(getenv("DDR_PACK_FAC_POW")) : 1.0;
  // block capacity rounded down to a multiple of this many reaches (a tick costs per 256-reach
  // slice-per-SIMD unit; experiments: DDR_PACK_QUANT)
  const int64_t pack_quant = getenv("DDR_PACK_QUANT") ? atol(getenv("DDR_PACK_QUANT")) : 1;

  // Splitting works on full-subtree sizes and heights: sub(i) = reaches draining through i,
  // ht(i) = longest path from i up to a source.
  std::vector<int32_t> sub(n, 1), ht(n, 0);
  for (int64_t i = 0; i < n; ++i)
    for (int64_t k = cnt[i]; k < cnt[i + 1]; ++k) {
      sub[i] += sub[col[k]];
      ht[i] = std::max(ht[i], ht[col[k]] + 1);
    }
  std::vector<int32_t> piece(n), resid(n), stem(n), dloc_piece(n);
  std::vector<char> is_root(n);
  std::vector<Piece> pieces;
  std::vector<int64_t> others;
  // Workgroups take their logical block index from a ticket counter in block order (route.hip:
  // take_ticket), and blocks are numbered by piece height, so a running workgroup's producers are
  // running or done: a schedule with more blocks than resident workgroups is still deadlock-free.
  // The packer first tries to fit one resident generation (all blocks co-resident, fully time-
  // pipelined): path-weighted packing, then unweighted; failing both it packs gen x resident
  // smaller blocks (every extra generation costs about T more ticks of the blocks it holds).
  // Split threshold (pieces up to scap_pct % of the capacity): with a dominant basin (C4/C5: 0.35 N)
  // its chain of pieces is the critical path, and pieces at 80 % leave the packer room to give chain
  // blocks fewer reaches; without one (C3: 256 basins of at most 2 % of N) pieces at the full
  // capacity mean fewer cut edges (C3 38.7 -> 36.5 ms per step; C5 at 100 %: 138 -> 149 ms;
  // profiles/r02/ab_defer_early.txt)
  int64_t scap_pct = 80;
  {
    std::vector<int32_t> bsz(n, 0);
    int64_t bmax = 0;
    for (int64_t i = 0; i < n; ++i) bmax = std::max<int64_t>(bmax, ++bsz[g->basin[i]]);
    if (bmax * 10 < n) scap_pct = 100;
#ifdef DDR_SCAP_PCT
    scap_pct = DDR_SCAP_PCT;
#endif
  }
  bool weighted = true;
  int64_t gen = 1;
  const int64_t cap_start = cap;
  for (;;) {
    // Stem-preserving split (bottom-up).  A reach whose subtree exceeds the capacity keeps its
    // deepest child (the main stem: every block boundary crossed along the longest flow path adds
    // a hand-off to the critical path) and absorbs other children, smallest first, while the
    // piece's tributary mass stays within cap - lseg, so every piece carries a stem stretch of at
    // least lseg reaches.  The stem child is cut only when the piece is full.
    // Pieces of split basins are kept below the block capacity: they land in blocks on long
    // chains, whose packing weight is up to ~(T + depth) / T times their size.
    const int64_t scap = cap * scap_pct / 100;
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
    pieces.clear();
    for (int64_t i = n - 1; i >= 0; --i) {
      int64_t d = g->down[i];
      if (d < 0 || is_root[i]) {
        is_root[i] = 1;
        piece[i] = (int64_t)pieces.size();
        pieces.push_back(Piece{i});
        dloc_piece[i] = 0;
      } else {
        piece[i] = piece[d];
        dloc_piece[i] = dloc_piece[d] + 1;
      }
      Piece& P = pieces[piece[i]];
      P.size++;
      if (cnt[i + 1] - cnt[i] > 2) P.xl += cnt[i + 1] - cnt[i];
      P.dmax = std::max<int64_t>(P.dmax, dloc_piece[i]);
    }
    // virtual inflows deepen the consuming piece by one tick; piece heights (children first:
    // a child piece is created after its parent in the loop above)
    for (int64_t p = (int64_t)pieces.size() - 1; p >= 0; --p) {
      int64_t r = pieces[p].root, d = g->down[r];
      if (d >= 0) {
        Piece& Q = pieces[piece[d]];
        Q.dmax = std::max<int64_t>(Q.dmax, dloc_piece[d] + 1);
        Q.height = std::max(Q.height, pieces[p].height + 1);
      }
    }
    phase("split");
    int64_t ncut = 0;
    for (auto& P : pieces) ncut += (g->down[P.root] >= 0);
    // Packing: pieces of equal height share blocks (so the block dependency graph is a DAG),
    // worst-fit by weight.  The blocks of a split basin progress at the pace of their slowest
    // member (a consumer waits for its producers, forward and backward alike), so every block
    // holding a piece of a long path needs T + (path length) ticks, not T + dmax: a piece is
    // weighted by (T + L) / T with L the longest source-to-outlet path through its root, plus one
    // chunk per inter-block hop on it.  Chain blocks get fewer reaches and tick faster (a tick
    // costs in proportion to the reaches of a workgroup).
    std::vector<int64_t> hops_down(pieces.size(), 0);
    for (size_t p = 0; p < pieces.size(); ++p) {  // parents before children (creation order)
      const int64_t d = g->down[pieces[p].root];
      if (d >= 0) hops_down[p] = hops_down[piece[d]] + 1;
    }
    std::vector<double> fac(pieces.size());
    double wsum = 0.0;
    for (size_t p = 0; p < pieces.size(); ++p) {
      const int64_t r = pieces[p].root;
      const double L = (double)(ht[r] + g->dist[r] + kChunk * (hops_down[p] + pieces[p].height));
      fac[p] = weighted ? std::pow((steps + L) / steps, fac_pow) : 1.0;
    }
    for (size_t p = 0; p < pieces.size(); ++p) wsum += (double)pieces[p].size * fac[p];
    // A block's tick budget is set by its most constrained piece: capacity capw / max factor.
    // Pieces are taken by factor (descending) so blocks gather pieces of similar factor; capw is
    // the smallest (1 % steps) that packs into the target number of workgroups.
    std::vector<int64_t> order(pieces.size()), block_of_piece(pieces.size()), load;
    std::vector<double> bcap;
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
      if (pieces[a].height != pieces[b].height) return pieces[a].height < pieces[b].height;
      if (fac[a] != fac[b]) return fac[a] > fac[b];
      return pieces[a].size > pieces[b].size;
    });
    int64_t ncut0 = 0;
    for (auto& P : pieces) ncut0 += (g->down[P.root] >= 0);
    const int64_t limit = ncut0 > 0 ? std::min<int64_t>(target, resident) * gen : target;
    // capw_k = capw_0 * 1.01^k; beyond k_sat (capw / fac >= hard_cap for every piece) the packing no
    // longer changes.  The block count falls with k, so the smallest k that fits is binary-searched
    // (a handful of packing passes instead of one per 1 % step).
    double maxfac = 1.0;
    for (double f : fac) maxfac = std::max(maxfac, f);
    const double capw0 = wsum / (double)limit;
    auto pack = [&](int k) {
      const double capw = capw0 * std::pow(1.01, (double)k);
      load.clear();
      bcap.clear();
      size_t hstart = 0;  // first block of the current height class
      int64_t curh = -1;
      for (int64_t p : order) {
        if (pieces[p].height != curh) {
          curh = pieces[p].height;
          hstart = load.size();
        }
        int64_t best = -1;
        const int64_t sz = pieces[p].size;
        for (size_t b = hstart; b < load.size(); ++b)
          if ((double)(load[b] + sz) <= bcap[b] && (best < 0 || load[b] < load[best])) best = (int64_t)b;
        if (best < 0) {
          best = (int64_t)load.size();
          load.push_back(0);
          double bc = std::min<double>((double)hard_cap, std::max<double>((double)sz, capw / fac[p]));
          if (pack_quant > 1 && bc >= (double)pack_quant)
            bc = std::max<double>((double)sz, std::floor(bc / (double)pack_quant) * (double)pack_quant);
          bcap.push_back(bc);
        }
        load[best] += sz;
        block_of_piece[p] = best;
      }
      return (int64_t)load.size();
    };
    const int k_sat = std::max(0, (int)std::ceil(std::log((double)hard_cap * maxfac / capw0) / std::log(1.01)));
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
    if (dbg) fprintf(stderr, "[part] pack passes %d\n", npass);
    phase("pack");
    if (getenv("DDR_DEBUG_PART"))
      fprintf(stderr, "[part] cap %ld hard %ld gen %ld weighted %d pieces %zu blocks %ld cut %ld\n", (long)cap,
              (long)hard_cap, (long)gen, (int)weighted, pieces.size(), (long)nblocks, (long)ncut);
    {
      // LDS of the fp32 kernels at the resulting slot / ring sizes; shrink the capacity if two
      // workgroups would no longer fit on a CU
      std::vector<int64_t> bv(nblocks, 0), bc(nblocks, 0), bx(nblocks, 0);
      for (size_t p = 0; p < pieces.size(); ++p) {
        bx[block_of_piece[p]] += pieces[p].xl;
        const int64_t d = g->down[pieces[p].root];
        if (d >= 0) {
          bv[block_of_piece[piece[d]]]++;
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
      const size_t need = std::max(route_lds_bytes(route_slot_stride((int)ms), mv, mc, mx, false, 4),
                                   route_lds_bytes(route_slot_stride((int)ms), mv, mc, mx, true, 4));
      if (getenv("DDR_DEBUG_PART"))
        fprintf(stderr, "[part]   slots %ld virt %ld cout %ld xl %ld lds %zu\n", (long)ms, (long)mv, (long)mc, (long)mx, need);
      // (a count failure at the capacity ceiling of the unweighted packing goes to more generations:
      // shrinking the capacity for LDS would only add blocks)
      const bool count_dead = ncut > 0 && nblocks > limit && cap >= hard_cap && !weighted;
      if (!count_dead && (need > kLdsBudget || mx >= kMaxConfluenceList)) {
        if (hard_cap <= 64) return fail(DDR_ERR_CAPACITY, "workgroup LDS budget exceeded");
        hard_cap -= std::max<int64_t>(1, hard_cap / 32);
        cap = std::min(cap, hard_cap);
        continue;
      }
    }
    if (ncut > 0 && nblocks > limit) {
      if (cap < hard_cap) {
        cap = std::min<int64_t>(hard_cap, cap + cap / 32 + 1);
        continue;
      }
      if (weighted) {
        weighted = false;
        cap = cap_start;
        continue;
      }
      if (++gen > 64) return fail(DDR_ERR_CAPACITY, "graph cannot be packed into workgroups");
      weighted = true;
      const int64_t per_gen = std::min<int64_t>(target, resident) * gen;
      cap = std::min<int64_t>(hard_cap, std::max<int64_t>(min_cap, (n + per_gen - 1) / per_gen));
      continue;
    }
    phase("lds");
    g->generations = gen;
    g->resident = resident;
    // ---- emit the schedule ---------------------------------------------------------------
    g->n_pieces = (int64_t)pieces.size();
    g->n_cut = ncut;
    g->block_of.assign(n, 0);
    for (int64_t i = 0; i < n; ++i) g->block_of[i] = block_of_piece[piece[i]];
    std::vector<int64_t> bdmax(nblocks, 0);
    for (size_t p = 0; p < pieces.size(); ++p)
      bdmax[block_of_piece[p]] = std::max(bdmax[block_of_piece[p]], pieces[p].dmax);
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
    struct Span {
      const int32_t* b;
      const int32_t* e;
      const int32_t* begin() const { return b; }
      const int32_t* end() const { return e; }
      size_t size() const { return (size_t)(e - b); }
      int64_t operator[](size_t k) const { return b[k]; }
    };
    auto members_of = [&](int64_t b) { return Span{order_all.data() + bstart[b], order_all.data() + bstart[b + 1]}; };
    phase("members");
    // internal order: blocks contiguous; inside a block by (tick offset, reference index)
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
    // Cut edges are numbered in (block, local position) order, i.e. by their index in cout_loc: the
    // forward kernel derives a cut reach's granule row from B.cout0 + its rank among the block's
    // cut reaches (route.hip), with no table load in the tick.
    phase("sort");
    int64_t eid = 0;
    for (int64_t b = 0; b < nblocks; ++b)
      for (int64_t i : members_of(b))
        if (g->down[i] >= 0 && g->block_of[g->down[i]] != b) edge_id[i] = eid++;
    g->n_cut = eid;  // inter-workgroup edges (pieces packed into one block hand off in LDS)
    g->blocks.assign(nblocks, BlockDesc{});
    int64_t p0 = 0, pre_dn = 0;
    g->max_slots = g->max_virt = g->max_cout = g->max_xl = 0;
    g->max_block_depth = 0;
    int64_t max_load = 0;
    for (int64_t b = 0; b < nblocks; ++b) {
      const Span m = members_of(b);
      for (size_t r = 0; r < m.size(); ++r) {
        pos[m[r]] = p0 + (int64_t)r;
        local[m[r]] = (int64_t)r;
      }
      BlockDesc& B = g->blocks[b];
      B.pos0 = (int32_t)p0;
      B.nloc = (int32_t)m.size();
      B.virt0 = (int32_t)v_edge.size();
      B.cout0 = (int32_t)cout_loc.size();
      B.dmax = (int32_t)bdmax[b];
      B.pre_dn = pre_dn;
      B.xl0 = (int32_t)xlist.size();
      max_load = std::max<int64_t>(max_load, (int64_t)m.size());
      for (size_t r = 0; r < m.size(); ++r) {
        int64_t i = m[r];
        int64_t P = p0 + (int64_t)r;
        ref[P] = (int32_t)i;
        offs[P] = (int32_t)offv[i];
        upb[P] = (int32_t)uplist.size();
        upc[P] = (int32_t)(cnt[i + 1] - cnt[i]);
        for (int64_t k = cnt[i]; k < cnt[i + 1]; ++k) {
          int64_t j = col[k];
          if (g->block_of[j] == b) {
            uplist.push_back((int32_t)local[j]);
          } else {
            // virtual inflow of cut edge j -> i
            uplist.push_back((int32_t)(m.size() + (v_edge.size() - B.virt0)));
            v_edge.push_back((int32_t)edge_id[j]);
            v_off.push_back((int32_t)(offv[i] - 1));
            v_dloc.push_back((int32_t)r);
          }
        }
        if (upc[P] > 2) {
          // confluence list: [c, u1, ..., u_{c-1}] at xoff (block-local), see route.hip pack_up
          xoff[P] = (int32_t)(xlist.size() - B.xl0);
          xlist.push_back(upc[P]);
          for (int32_t k = 1; k < upc[P]; ++k) xlist.push_back(uplist[upb[P] + k]);
        }
        int64_t d = g->down[i];
        dl[P] = (d >= 0 && g->block_of[d] == b) ? -2 : -1;  // resolved below (local of d)
        if (d >= 0 && g->block_of[d] != b) {
          cut[P] = (int32_t)edge_id[i];
          cout_loc.push_back((int32_t)r);
        }
      }
      B.nvirt = (int32_t)(v_edge.size() - B.virt0);
      B.ncout = (int32_t)(cout_loc.size() - B.cout0);
      B.nxl = (int32_t)(xlist.size() - B.xl0);
      g->max_xl = std::max<int>(g->max_xl, B.nxl);
      g->max_slots = std::max<int>(g->max_slots, B.nloc + B.nvirt);
      g->max_virt = std::max<int>(g->max_virt, B.nvirt);
      g->max_cout = std::max<int>(g->max_cout, B.ncout);
      g->max_block_depth = std::max<int64_t>(g->max_block_depth, B.dmax + 1);
      pre_dn += bdmax[b] * (int64_t)m.size();
      p0 += (int64_t)m.size();
    }
    phase("emit");
    for (int64_t i = 0; i < n; ++i) {
      int64_t P = pos[i];
      if (dl[P] == -2) dl[P] = (int32_t)local[g->down[i]];
    }
    g->sum_dn = pre_dn;
    g->max_nloc = (int)max_load;
    int kr = 1;
    while (int64_t(kr) * bs < max_load) kr *= 2;
    g->kr = kr;
    if (g->max_virt > bs || g->max_cout > bs)
      return fail(DDR_ERR_CAPACITY, "too many inter-workgroup edges in one workgroup");
    phase("schedule");
    if (dbg) {  // schedule fingerprint (FNV-1a over the emitted arrays)
      unsigned long long h = 1469598103934665603ull;
      auto mix = [&](const std::vector<int32_t>& v) {
        for (int32_t x : v) h = (h ^ (unsigned)x) * 1099511628211ull;
      };
      mix(ref); mix(offs); mix(upb); mix(upc); mix(dl); mix(cut); mix(xoff); mix(uplist); mix(xlist);
      mix(v_edge); mix(v_off); mix(v_dloc); mix(cout_loc);
      fprintf(stderr, "[part] schedule fingerprint %016llx\n", h);
    }
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
    if (opts && (opts->flags & DDR_BUILD_HOST_ONLY)) break;
    ddr_status st = upload_schedule(g.get());
    if (st) return st;
    phase("upload");
    break;
  }
  g->crow = std::move(cnt);
  g->col = std::move(col);
  *out = g.release();
  return DDR_OK;
}

void destroy_graph(Graph* g) {
  if (!g) return;
  for (void* p : g->allocations) (void)hipFree(p);
  delete g;
}

}  // namespace ddr
