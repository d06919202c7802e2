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

ddr_status build_graph(int64_t n, int64_t e, const int32_t* rows, const int32_t* cols,
                       const ddr_build_opts* opts, Graph** out) {
  if (n <= 0) return fail(DDR_ERR_ARG, "graph must have at least one reach");
  if (n >= (int64_t(1) << 31) - 1) return fail(DDR_ERR_ARG, "graph too large for int32 reach ids");
  if (e < 0 || (e > 0 && (!rows || !cols))) return fail(DDR_ERR_ARG, "bad COO arrays");
  auto g = std::make_unique<Graph>();
  g->n = n;
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
  for (int64_t i = 0; i < n; ++i) std::sort(col.begin() + cnt[i], col.begin() + cnt[i + 1]);
  for (int64_t i = 0; i < n; ++i)
    for (int64_t k = cnt[i] + 1; k < cnt[i + 1]; ++k)
      if (col[k] == col[k - 1])
        return fail(DDR_ERR_DUPLICATE, "duplicate edge (" + std::to_string(i) + "," + std::to_string(col[k]) + ")");
  g->crow = cnt;
  g->col = col;
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
  std::vector<int64_t> bsize(n, 0);
  for (int64_t i = 0; i < n; ++i) bsize[g->basin[i]]++;
  for (int64_t i = 0; i < n; ++i) g->n_basins += (g->down[i] < 0);

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
  int64_t cap = std::min<int64_t>(hard_cap, std::max<int64_t>(bs, (n + target - 1) / target));
  const double steps = (opts && opts->steps_hint > 0) ? (double)opts->steps_hint : 8760.0;

  // Splitting works on full-subtree sizes and heights: sub(i) = reaches draining through i,
  // ht(i) = longest path from i up to a source.
  std::vector<int64_t> sub(n, 1), ht(n, 0);
  for (int64_t i = 0; i < n; ++i)
    for (int64_t k = cnt[i]; k < cnt[i + 1]; ++k) {
      sub[i] += sub[col[k]];
      ht[i] = std::max(ht[i], ht[col[k]] + 1);
    }
  std::vector<int64_t> piece(n), resid(n), stem(n), dloc_piece(n);
  std::vector<char> is_root(n);
  std::vector<Piece> pieces;
  std::vector<int64_t> others;
  // Workgroups take their logical block index from a ticket counter in block order (route.hip:
  // take_ticket), and blocks are numbered by piece height, so a running workgroup's producers are
  // running or done: a schedule with more blocks than resident workgroups is still deadlock-free.
  // The packer first tries to fit one resident generation (all blocks co-resident, fully time-
  // pipelined): path-weighted packing, then unweighted; failing both it packs gen x resident
  // smaller blocks (every extra generation costs about T more ticks of the blocks it holds).
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
    const int64_t scap = cap * 4 / 5;
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
      P.dmax = std::max(P.dmax, dloc_piece[i]);
    }
    // virtual inflows deepen the consuming piece by one tick; piece heights (children first:
    // a child piece is created after its parent in the loop above)
    for (int64_t p = (int64_t)pieces.size() - 1; p >= 0; --p) {
      int64_t r = pieces[p].root, d = g->down[r];
      if (d >= 0) {
        Piece& Q = pieces[piece[d]];
        Q.dmax = std::max(Q.dmax, dloc_piece[d] + 1);
        Q.height = std::max(Q.height, pieces[p].height + 1);
      }
    }
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
      fac[p] = weighted ? (steps + L) / steps : 1.0;
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
    for (double capw = wsum / (double)limit;; capw *= 1.01) {
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
        for (size_t b = hstart; b < load.size(); ++b)
          if ((double)(load[b] + pieces[p].size) <= bcap[b] && (best < 0 || load[b] < load[best])) best = (int64_t)b;
        if (best < 0) {
          best = (int64_t)load.size();
          load.push_back(0);
          bcap.push_back(std::min<double>((double)hard_cap, std::max<double>((double)pieces[p].size, capw / fac[p])));
        }
        load[best] += pieces[p].size;
        block_of_piece[p] = best;
      }
      if ((int64_t)load.size() <= limit || capw / 1.3 > (double)hard_cap) break;
    }
    const int64_t nblocks = (int64_t)load.size();
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
      if (need > kLdsBudget || mx >= kMaxConfluenceList) {
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
      cap = std::min<int64_t>(hard_cap, std::max<int64_t>(bs, (n + per_gen - 1) / per_gen));
      continue;
    }
    g->generations = gen;
    g->resident = resident;
    // ---- emit the schedule ---------------------------------------------------------------
    g->n_pieces = (int64_t)pieces.size();
    g->n_cut = ncut;
    g->block_of.assign(n, 0);
    for (int64_t i = 0; i < n; ++i) g->block_of[i] = block_of_piece[piece[i]];
    std::vector<std::vector<int64_t>> members(nblocks);
    for (int64_t i = 0; i < n; ++i) members[g->block_of[i]].push_back(i);
    std::vector<int64_t> bdmax(nblocks, 0);
    for (size_t p = 0; p < pieces.size(); ++p)
      bdmax[block_of_piece[p]] = std::max(bdmax[block_of_piece[p]], pieces[p].dmax);
    std::vector<int64_t> offv(n);
    for (int64_t i = 0; i < n; ++i) offv[i] = bdmax[g->block_of[i]] - dloc_piece[i];
    // internal order: blocks contiguous; inside a block by (tick offset, reference index)
    std::vector<int64_t> pos(n), local(n);
    std::vector<int32_t> ref(n), offs(n), upb(n), upc(n), dl(n), cut(n, -1), xoff(n, -1), uplist;
    std::vector<int32_t> v_edge, v_off, v_dloc, cout_loc;
    std::vector<int64_t> edge_id(n, -1);
    // Cut edges are numbered in (block, local position) order, i.e. by their index in cout_loc: the
    // forward kernel derives a cut reach's granule row from B.cout0 + its rank among the block's
    // cut reaches (route.hip), with no table load in the tick.
    for (int64_t b = 0; b < nblocks; ++b)
      std::stable_sort(members[b].begin(), members[b].end(), [&](int64_t a, int64_t c) {
        if (offv[a] != offv[c]) return offv[a] < offv[c];
        return a < c;
      });
    int64_t eid = 0;
    for (int64_t b = 0; b < nblocks; ++b)
      for (int64_t i : members[b])
        if (g->down[i] >= 0 && g->block_of[g->down[i]] != b) edge_id[i] = eid++;
    g->n_cut = eid;  // inter-workgroup edges (pieces packed into one block hand off in LDS)
    std::vector<int32_t> xlist;
    g->blocks.assign(nblocks, BlockDesc{});
    int64_t p0 = 0, pre_dn = 0;
    g->max_slots = g->max_virt = g->max_cout = g->max_xl = 0;
    g->max_block_depth = 0;
    int64_t max_load = 0;
    for (int64_t b = 0; b < nblocks; ++b) {
      auto& m = members[b];
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
    // ---- upload ----------------------------------------------------------------------------
    if (opts && (opts->flags & DDR_BUILD_HOST_ONLY)) break;
    DevSchedule& D = g->dev;
    ddr_status st;
    if ((st = upload(g.get(), &D.blocks, g->blocks))) return st;
    if ((st = upload(g.get(), &D.ref, ref))) return st;
    if ((st = upload(g.get(), &D.off, offs))) return st;
    if ((st = upload(g.get(), &D.upb, upb))) return st;
    if ((st = upload(g.get(), &D.upc, upc))) return st;
    if ((st = upload(g.get(), &D.dloc, dl))) return st;
    if ((st = upload(g.get(), &D.cut, cut))) return st;
    if ((st = upload(g.get(), &D.uplist, uplist))) return st;
    if ((st = upload(g.get(), &D.xoff, xoff))) return st;
    if ((st = upload(g.get(), &D.xlist, xlist))) return st;
    if ((st = upload(g.get(), &D.v_edge, v_edge))) return st;
    if ((st = upload(g.get(), &D.v_off, v_off))) return st;
    if ((st = upload(g.get(), &D.v_dloc, v_dloc))) return st;
    if ((st = upload(g.get(), &D.cout_loc, cout_loc))) return st;
    std::vector<int32_t> pos_of_ref(n), block_of_pos(n);
    for (int64_t i = 0; i < n; ++i) {
      pos_of_ref[i] = (int32_t)pos[i];
      block_of_pos[pos[i]] = (int32_t)g->block_of[i];
    }
    if ((st = upload(g.get(), &D.pos_of_ref, pos_of_ref))) return st;
    if ((st = upload(g.get(), &D.block_of_pos, block_of_pos))) return st;
    // per block: local indices in ascending reference order (coalesced reads of q' rows)
    std::vector<int32_t> rs_loc(n), rs_ref(n);
    for (int64_t b = 0; b < nblocks; ++b) {
      const BlockDesc& B = g->blocks[b];
      std::vector<std::pair<int32_t, int32_t>> v(B.nloc);
      for (int32_t r = 0; r < B.nloc; ++r) v[r] = {ref[B.pos0 + r], r};
      std::sort(v.begin(), v.end());
      for (int32_t k = 0; k < B.nloc; ++k) {
        rs_ref[B.pos0 + k] = v[k].first;
        rs_loc[B.pos0 + k] = v[k].second;
      }
    }
    if ((st = upload(g.get(), &D.rs_loc, rs_loc))) return st;
    if ((st = upload(g.get(), &D.rs_ref, rs_ref))) return st;
    break;
  }
  *out = g.release();
  return DDR_OK;
}

void destroy_graph(Graph* g) {
  if (!g) return;
  for (void* p : g->allocations) (void)hipFree(p);
  delete g;
}

}  // namespace ddr
