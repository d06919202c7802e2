// On-device river-graph builder (BASELINE north star (1): "a CSR/level-set converter builds on device
// from the zarr COO").  Input: the COO adjacency in device memory (row = downstream reach, col =
// upstream reach, the ddr-engine contract, engine/src/ddr_engine/core/zarr_io.py:7-76).  Output: the
// same Graph as the host builder (graph.cpp) -- validation, canonical CSR (scipy .tocsr(),
// merit.py:197-223), dendritic structure, stem-preserving basin split, and the per-workgroup tick
// schedule -- bit for bit, with every O(n) pass on the device:
//
//   validate + down[] (atomicCAS: a reach with two downstream reaches, a duplicate edge) -> CSR (one
//   stable radix sort of the reaches by their downstream reach: the children of each row come out
//   ascending) -> distance to outlet and basin (pointer jumping, log2(depth) rounds) -> subtree size
//   and height, then the split (per basin one workgroup walks its reaches level by level, deepest
//   first: a reach's children are final when its level runs) -> pieces (nearest piece root by
//   pointer jumping; pieces numbered by descending root index as on the host) -> piece table ->
//   HOST: pack_pieces (the packer works on the few thousand pieces, graph.cpp) -> schedule emission
//   (sort by (block, tick offset, reach); prefix sums number the cut edges, virtual inflows,
//   upstream lists and confluence lists in position order).
//
// The host reads the device twice per split pass (a count, then the piece table); everything per
// reach stays on the device.  Temporaries are pooled device blocks (device_get) ordered on the build stream.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <memory>
#include <vector>

#include "internal.h"

namespace ddr {

namespace {

constexpr int kTB = 256;  // threads per workgroup of the flat kernels
inline unsigned nblk(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + kTB - 1) / kTB); }
inline int bits_for(uint64_t maxval) {  // radix-sort key bits covering [0, maxval]
  int b = 1;
  while (b < 64 && (maxval >> b) != 0) ++b;
  return b;
}

// error words (min over offending entries): edge out of range, edge not below the diagonal, duplicate
// edge, reach with two downstream reaches
enum { kErrRange = 0, kErrLower = 1, kErrDup = 2, kErrDend = 3, kErrWords = 4 };

__global__ void k_iota(int32_t* v, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = (int32_t)i;
}

// down[c] = r for every edge (r, c); deg[r] = number of upstream reaches
__global__ void k_coo(int64_t n, int64_t e, const int32_t* rows, const int32_t* cols, int32_t* down, int32_t* deg,
                      unsigned long long* err) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= e) return;
  const int32_t r = rows[k], c = cols[k];
  if (r < 0 || r >= n || c < 0 || c >= n) {
    atomicMin(err + kErrRange, (unsigned long long)k);
    return;
  }
  if (c >= r) {
    atomicMin(err + kErrLower, (unsigned long long)k);
    return;
  }
  const int32_t old = atomicCAS(down + c, -1, r);
  if (old == -1) atomicAdd(deg + r, 1);
  else if (old == r) atomicMin(err + kErrDup, (unsigned long long)k);
  else atomicMin(err + kErrDend, (unsigned long long)c);
}

// sort key of reach c for the CSR: its downstream reach (outlets last)
__global__ void k_down_key(int64_t n, const int32_t* down, uint32_t* key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) key[i] = down[i] < 0 ? (uint32_t)n : (uint32_t)down[i];
}

// pointer jumping: p = parent (a root points to itself), d = hops to p
__global__ void k_jump_init(int64_t n, const int32_t* down, const uint8_t* stop, int32_t* p, int32_t* d) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool r = down[i] < 0 || (stop && stop[i]);
  p[i] = r ? (int32_t)i : down[i];
  d[i] = r ? 0 : 1;
}
__global__ void k_jump(int64_t n, const int32_t* p, const int32_t* d, int32_t* p2, int32_t* d2) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t q = p[i];
  p2[i] = p[q];
  d2[i] = d[i] + d[q];
}

// Wave-aggregated atomics on keyed counters: the lanes sharing the first active lane's key combine their
// values (one wave reduction) and that lane issues one atomic; repeated for up to kAggRounds distinct keys,
// the rest atomically per lane.  Reaches of one basin / piece are mostly numbered together, so a wave
// holds one or two keys: ~1M same-address atomics per build (0.4-0.5 ms each for basin sizes and the
// piece table at C3) become a few per wave.
constexpr int kAggRounds = 4;
__device__ __forceinline__ int wave_sum_i(int v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}
// op 0: add, 1: max
template <int OP>
__device__ __forceinline__ void wave_atomic(int32_t* base, int32_t key, int32_t val, bool active) {
  const int lane = threadIdx.x & 63;
  for (int r = 0; r < kAggRounds; ++r) {
    const unsigned long long m = __builtin_amdgcn_ballot_w64(active);
    if (m == 0) return;
    const int leader = __builtin_ffsll((long long)m) - 1;
    const int32_t k = __builtin_amdgcn_readlane(key, leader);
    const bool mine = active && key == k;
    const int32_t agg = OP == 0 ? wave_sum_i(mine ? val : 0) : wave_max_i(mine ? val : INT32_MIN);
    if (lane == leader) {
      if (OP == 0) atomicAdd(base + k, agg);
      else atomicMax(base + k, agg);
    }
    active = active && !mine;
  }
  if (active) {
    if (OP == 0) atomicAdd(base + key, val);
    else atomicMax(base + key, val);
  }
}

// basin sizes, deepest reach, outlet count
__global__ void k_stats(int64_t n, const int32_t* down, const int32_t* basin, const int32_t* dist, int32_t* bsize,
                        int32_t* agg) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = i < n;
  wave_atomic<0>(bsize, in ? basin[i] : 0, 1, in);
  // the graph-wide maximum depth and outlet count: one atomic per wave, not per reach (a million
  // same-address atomics serialised to ~0.5 ms per build)
  int dmax = in ? dist[i] : 0;
  int outl = (in && down[i] < 0) ? 1 : 0;
  for (int o = 32; o > 0; o >>= 1) {
    dmax = max(dmax, __shfl_xor(dmax, o));
    outl += __shfl_xor(outl, o);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(agg + 0, dmax);
    if (outl) atomicAdd(agg + 1, outl);
  }
}
__global__ void k_bmax(int64_t n, const int32_t* down, const int32_t* bsize, int32_t* agg) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && down[i] < 0) atomicMax(agg + 2, bsize[i]);
}

// level-order key: basin-major, deepest level first
__global__ void k_level_key(int64_t n, const int32_t* basin, const int32_t* dist, int64_t D, uint64_t* key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) key[i] = (uint64_t)basin[i] * (uint64_t)(D + 1) + (uint64_t)(D - dist[i]);
}
// level starts (for the max-scan), basin segments
__global__ void k_level_marks(int64_t n, const uint64_t* key, const int32_t* ord, const int32_t* basin,
                              int32_t* start_of, int32_t* seg_lo, int32_t* seg_hi) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  start_of[p] = (p == 0 || key[p] != key[p - 1]) ? (int32_t)p : 0;
  const int32_t b = basin[ord[p]];
  if (p == 0 || basin[ord[p - 1]] != b) seg_lo[b] = (int32_t)p;
  if (p == n - 1 || basin[ord[p + 1]] != b) seg_hi[b] = (int32_t)(p + 1);
}
// level links: lvl_next[start] = end, lvl_first[end - 1] = start
__global__ void k_level_links(int64_t n, const uint64_t* key, const int32_t* smax, int32_t* lvl_next) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n) return;
  if (q == n - 1 || key[q + 1] != key[q]) lvl_next[smax[q]] = (int32_t)(q + 1);
}
// outlets in ascending order (one workgroup per basin in the level walks)
__global__ void k_roots(int64_t n, const int32_t* down, const int32_t* rank, int32_t* roots) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && down[i] < 0) roots[rank[i]] = (int32_t)i;
}
__global__ void k_is_outlet(int64_t n, const int32_t* down, int32_t* f) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) f[i] = down[i] < 0 ? 1 : 0;
}

// Subtree size and height (graph.cpp: sub, ht), one workgroup per basin, deepest level first.
__global__ void __launch_bounds__(256) k_sub_ht(const int32_t* roots, const int32_t* nroots, const int32_t* seg_lo,
                                                const int32_t* seg_hi, const int32_t* lvl_next, const int32_t* ord,
                                                const int32_t* crow, const int32_t* col, int32_t* sub, int32_t* ht) {
  for (int32_t b = blockIdx.x; b < *nroots; b += gridDim.x) {
  const int32_t root = roots[b];
  const int32_t lo = seg_lo[root], hi = seg_hi[root];
  for (int32_t s = lo; s < hi;) {
    const int32_t e = lvl_next[s];
    for (int32_t p = s + threadIdx.x; p < e; p += blockDim.x) {
      const int32_t i = ord[p];
      int32_t su = 1, h = 0;
      for (int32_t k = crow[i]; k < crow[i + 1]; ++k) {
        const int32_t c = col[k];
        su += sub[c];
        h = max(h, ht[c] + 1);
      }
      sub[i] = su;
      ht[i] = h;
    }
    __threadfence_block();
    __syncthreads();
    s = e;
  }
  }
}

// Level order position of every reach, and the child table in level order: cnt[p] children of reach
// ord[p], cpos[p] the level positions of its first four (column order; -1 past the count)
__global__ void k_inv(int64_t n, const int32_t* ord, int32_t* inv) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n) inv[ord[p]] = (int32_t)p;
}
__global__ void k_child_tab(int64_t n, const int32_t* ord, const int32_t* crow, const int32_t* col, const int32_t* inv,
                            int32_t* cnt, int4* cpos) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const int32_t i = ord[p], k0 = crow[i], k1 = crow[i + 1];
  cnt[p] = k1 - k0;
  int4 q;
  q.x = k0 + 0 < k1 ? inv[col[k0 + 0]] : -1;
  q.y = k0 + 1 < k1 ? inv[col[k0 + 1]] : -1;
  q.z = k0 + 2 < k1 ? inv[col[k0 + 2]] : -1;
  q.w = k0 + 3 < k1 ? inv[col[k0 + 3]] : -1;
  cpos[p] = q;
}

__device__ __forceinline__ void lds_barrier_dg() {
  // LDS hand-off only: global loads issued ahead stay in flight across the barrier
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// k_sub_ht with the basin's subtree sizes and heights in LDS (segments of at most kLevelLds reaches;
// larger basins take the global walk of k_sub_ht): a level reads its children's values from LDS at
// positions from the child table, whose rows (and the level bounds) are requested a level ahead -- a
// level costs an LDS round trip and a barrier instead of a chain of four dependent global loads
constexpr int kLevelLds = 20480;  // reaches: 4 B size + 2 B height each, 120 KB
__global__ void __launch_bounds__(256) k_sub_ht_lds(const int32_t* roots, const int32_t* nroots, const int32_t* seg_lo,
                                                    const int32_t* seg_hi, const int32_t* lvl_next, const int32_t* ord,
                                                    const int32_t* crow, const int32_t* col, const int32_t* inv,
                                                    const int32_t* cnt, const int4* cpos, int32_t* sub, int32_t* ht) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lsm[];
  int32_t* sub_l = reinterpret_cast<int32_t*>(lsm);
  uint16_t* ht_l = reinterpret_cast<uint16_t*>(lsm + 4 * kLevelLds);
  const int tid = threadIdx.x;
  for (int32_t b = blockIdx.x; b < *nroots; b += gridDim.x) {
    const int32_t root = roots[b];
    const int32_t lo = seg_lo[root], hi = seg_hi[root];
    if (hi - lo > kLevelLds) {
      // the global walk (k_sub_ht's body)
      for (int32_t s = lo; s < hi;) {
        const int32_t e = lvl_next[s];
        for (int32_t p = s + tid; p < e; p += blockDim.x) {
          const int32_t i = ord[p];
          int32_t su = 1, h = 0;
          for (int32_t k = crow[i]; k < crow[i + 1]; ++k) {
            const int32_t c = col[k];
            su += sub[c];
            h = max(h, ht[c] + 1);
          }
          sub[i] = su;
          ht[i] = h;
        }
        __threadfence_block();
        __syncthreads();
        s = e;
      }
      continue;
    }
    int32_t s = lo, e = lvl_next[lo];
    int32_t e2 = e < hi ? lvl_next[e] : hi;
    int32_t pc = 0;
    int4 pq = make_int4(-1, -1, -1, -1);
    if (s + tid < e) {
      pc = cnt[s + tid];
      pq = cpos[s + tid];
    }
    while (s < hi) {
      // the next level's first row and the level after's bound, requested before this level's work
      int32_t nc = 0;
      int4 nq = make_int4(-1, -1, -1, -1);
      if (e + tid < e2) {
        nc = cnt[e + tid];
        nq = cpos[e + tid];
      }
      const int32_t e3 = e2 < hi ? lvl_next[e2] : hi;
      for (int32_t p = s + tid; p < e; p += blockDim.x) {
        int32_t c4 = pc;
        int4 q = pq;
        if (p != s + tid) {
          c4 = cnt[p];
          q = cpos[p];
        }
        int32_t su = 1, h = 0;
        auto add = [&](int32_t cp) {
          su += sub_l[cp - lo];
          h = max(h, (int32_t)ht_l[cp - lo] + 1);
        };
        if (c4 > 0) add(q.x);
        if (c4 > 1) add(q.y);
        if (c4 > 2) add(q.z);
        if (c4 > 3) add(q.w);
        if (c4 > 4) {
          const int32_t i = ord[p], k0 = crow[i];
          for (int32_t k = k0 + 4; k < k0 + c4; ++k) add(inv[col[k]]);
        }
        sub_l[p - lo] = su;
        ht_l[p - lo] = (uint16_t)h;
      }
      lds_barrier_dg();
      s = e;
      e = e2;
      e2 = e3;
      pc = nc;
      pq = nq;
    }
    for (int32_t p = lo + tid; p < hi; p += blockDim.x) {
      const int32_t i = ord[p];
      sub[i] = sub_l[p - lo];
      ht[i] = ht_l[p - lo];
    }
    __syncthreads();  // (the next basin reuses the LDS)
  }
}

// Stem-preserving split of the basins larger than scap (graph.cpp build_graph, same rule and the
// same tie-breaks: the deepest child by (height, size), first in column order; the others by
// ascending residual size, ties in column order).  Smaller basins stay one piece.
// scap < 0: the first pass, whose threshold the device chose from the largest basin (k_scap)
__global__ void __launch_bounds__(256) k_split(const int32_t* roots, const int32_t* nroots, const int32_t* seg_lo,
                                               const int32_t* seg_hi, const int32_t* lvl_next, const int32_t* ord,
                                               const int32_t* crow, const int32_t* col, const int32_t* sub,
                                               const int32_t* ht, int32_t* resid, int32_t* stem, uint8_t* is_root,
                                               int64_t scap_arg, const int32_t* agg) {
  const int64_t scap = scap_arg >= 0 ? scap_arg : (int64_t)agg[3];
  const int64_t lseg = scap / 8;
  for (int32_t bb = blockIdx.x; bb < *nroots; bb += gridDim.x) {
  const int32_t root = roots[bb];
  if (sub[root] <= scap) continue;
  const int32_t lo = seg_lo[root], hi = seg_hi[root];
  for (int32_t s = lo; s < hi;) {
    const int32_t e = lvl_next[s];
    for (int32_t p = s + threadIdx.x; p < e; p += blockDim.x) {
      const int32_t i = ord[p];
      const int32_t k0 = crow[i], k1 = crow[i + 1];
      if (sub[i] <= scap || k0 == k1) {
        resid[i] = sub[i];
        stem[i] = ht[i] + 1;
        continue;
      }
      int32_t dc = col[k0];
      for (int32_t k = k0 + 1; k < k1; ++k) {
        const int32_t c = col[k];
        if (ht[c] > ht[dc] || (ht[c] == ht[dc] && sub[c] > sub[dc])) dc = c;
      }
      int64_t base = 1 + (int64_t)resid[dc], trib = (int64_t)resid[dc] - stem[dc];
      const bool keep = base <= scap;
      if (!keep) {
        is_root[dc] = 1;
        base = 1;
        trib = 0;
      }
      int64_t acc = 0;
      // the other children in (resid, column position) order: a selection per step (few children)
      int64_t pr = -1, pk = -1;
      for (int32_t step = 0; step < k1 - k0 - 1; ++step) {
        int64_t br = 0x7fffffffffffffffll, bk = -1;
        for (int32_t k = k0; k < k1; ++k) {
          const int32_t c = col[k];
          if (c == dc) continue;
          const int64_t r = resid[c];
          const bool after = r > pr || (r == pr && k > pk);
          if (after && (r < br || (r == br && k < bk))) {
            br = r;
            bk = k;
          }
        }
        const int32_t c = col[bk];
        if (trib + acc + br <= scap - lseg && base + acc + br <= scap) acc += br;
        else is_root[c] = 1;
        pr = br;
        pk = bk;
      }
      resid[i] = (int32_t)(base + acc);
      stem[i] = keep ? 1 + stem[dc] : 1;
    }
    __threadfence_block();
    __syncthreads();
    s = e;
  }
  }
}
// Per level position, everything the split reads that no level writes (k_sub_ht's sizes and heights):
// a = (own size, own height, child count, 0), and per child j < 4 (column order) its level position,
// reach, size and height -- one coalesced row per position for k_split_lds
struct SplitRow {
  int4 a, pos, id, sz, h;
};
__global__ void k_split_tab(int64_t n, const int32_t* ord, const int32_t* cnt, const int4* cpos, const int32_t* sub,
                            const int32_t* ht, SplitRow* tab) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const int32_t i = ord[p], c = cnt[p];
  SplitRow r;
  r.a = make_int4(sub[i], ht[i], c, 0);
  r.pos = cpos[p];
  const int32_t q[4] = {r.pos.x, r.pos.y, r.pos.z, r.pos.w};
  int32_t id[4], sz[4], hh[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    id[j] = j < c ? ord[q[j]] : -1;
    sz[j] = j < c ? sub[id[j]] : 0;
    hh[j] = j < c ? ht[id[j]] : 0;
  }
  r.id = make_int4(id[0], id[1], id[2], id[3]);
  r.sz = make_int4(sz[0], sz[1], sz[2], sz[3]);
  r.h = make_int4(hh[0], hh[1], hh[2], hh[3]);
  tab[p] = r;
}

// k_split with the residual sizes and stem lengths of a basin in LDS (segments of at most kLevelLds
// reaches; larger basins take k_split's global walk) and every static input from the split table,
// requested a level ahead: the same decisions in the same order (deepest child by (height, size),
// first in column order; the others by ascending (residual, column position))
__global__ void __launch_bounds__(256) k_split_lds(const int32_t* roots, const int32_t* nroots, const int32_t* seg_lo,
                                                   const int32_t* seg_hi, const int32_t* lvl_next, const int32_t* ord,
                                                   const int32_t* crow, const int32_t* col, const int32_t* inv,
                                                   const SplitRow* tab, const int32_t* sub, const int32_t* ht,
                                                   int32_t* resid, int32_t* stem, uint8_t* is_root, int64_t scap_arg,
                                                   const int32_t* agg) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lsm[];
  int32_t* res_l = reinterpret_cast<int32_t*>(lsm);
  uint16_t* stem_l = reinterpret_cast<uint16_t*>(lsm + 4 * kLevelLds);
  const int64_t scap = scap_arg >= 0 ? scap_arg : (int64_t)agg[3];
  const int64_t lseg = scap / 8;
  const int tid = threadIdx.x;
  for (int32_t bb = blockIdx.x; bb < *nroots; bb += gridDim.x) {
    const int32_t root = roots[bb];
    if (sub[root] <= scap) continue;
    const int32_t lo = seg_lo[root], hi = seg_hi[root];
    const bool in_lds = hi - lo <= kLevelLds;
    // a reach's residual / stem: LDS (by level position) or global (by reach)
    auto get_res = [&](int32_t pos, int32_t id) { return in_lds ? res_l[pos - lo] : resid[id]; };
    auto get_stem = [&](int32_t pos, int32_t id) { return in_lds ? (int32_t)stem_l[pos - lo] : stem[id]; };
    auto put = [&](int32_t p, int32_t i, int32_t r, int32_t st) {
      if (in_lds) {
        res_l[p - lo] = r;
        stem_l[p - lo] = (uint16_t)st;
      } else {
        resid[i] = r;
        stem[i] = st;
      }
    };
    // one position: the split rule of k_split
    auto step = [&](int32_t p, const SplitRow& R) {
      const int32_t i = ord[p];
      const int32_t nc = R.a.z;
      if ((int64_t)R.a.x <= scap || nc == 0) {
        put(p, i, R.a.x, R.a.y + 1);
        return;
      }
      // children j < nc: (position, reach, size, height); beyond 4 from the CSR
      auto child = [&](int32_t j, int32_t& pos, int32_t& id, int32_t& sz, int32_t& h) {
        if (j < 4) {
          pos = j == 0 ? R.pos.x : j == 1 ? R.pos.y : j == 2 ? R.pos.z : R.pos.w;
          id = j == 0 ? R.id.x : j == 1 ? R.id.y : j == 2 ? R.id.z : R.id.w;
          sz = j == 0 ? R.sz.x : j == 1 ? R.sz.y : j == 2 ? R.sz.z : R.sz.w;
          h = j == 0 ? R.h.x : j == 1 ? R.h.y : j == 2 ? R.h.z : R.h.w;
        } else {
          id = col[crow[i] + j];
          pos = inv[id];
          sz = sub[id];
          h = ht[id];
        }
      };
      int32_t dj = 0, dpos, did, dsz, dh;
      child(0, dpos, did, dsz, dh);
      for (int32_t j = 1; j < nc; ++j) {
        int32_t cp, ci, cs, ch;
        child(j, cp, ci, cs, ch);
        if (ch > dh || (ch == dh && cs > dsz)) {
          dj = j; dpos = cp; did = ci; dsz = cs; dh = ch;
        }
      }
      const int32_t dres = get_res(dpos, did), dstem = get_stem(dpos, did);
      int64_t base = 1 + (int64_t)dres, trib = (int64_t)dres - dstem;
      const bool keep = base <= scap;
      if (!keep) {
        is_root[did] = 1;
        base = 1;
        trib = 0;
      }
      int64_t acc = 0;
      // the other children in (resid, column position) order: a selection per step (few children)
      int64_t pr = -1, pk = -1;
      for (int32_t stp = 0; stp < nc - 1; ++stp) {
        int64_t br = 0x7fffffffffffffffll, bk = -1;
        int32_t bid = -1;
        for (int32_t j = 0; j < nc; ++j) {
          if (j == dj) continue;
          int32_t cp, ci, cs, ch;
          child(j, cp, ci, cs, ch);
          const int64_t r = get_res(cp, ci);
          const bool after = r > pr || (r == pr && j > pk);
          if (after && (r < br || (r == br && j < bk))) {
            br = r;
            bk = j;
            bid = ci;
          }
        }
        if (trib + acc + br <= scap - lseg && base + acc + br <= scap) acc += br;
        else is_root[bid] = 1;
        pr = br;
        pk = bk;
      }
      put(p, i, (int32_t)(base + acc), keep ? 1 + dstem : 1);
    };
    int32_t s = lo, e = lvl_next[lo];
    int32_t e2 = e < hi ? lvl_next[e] : hi;
    SplitRow pr0{};
    if (s + tid < e) pr0 = tab[s + tid];
    while (s < hi) {
      SplitRow nr{};
      if (e + tid < e2) nr = tab[e + tid];
      const int32_t e3 = e2 < hi ? lvl_next[e2] : hi;
      for (int32_t p = s + tid; p < e; p += blockDim.x) step(p, p == s + tid ? pr0 : tab[p]);
      if (in_lds) {
        lds_barrier_dg();
      } else {
        __threadfence_block();
        __syncthreads();
      }
      s = e;
      e = e2;
      e2 = e3;
      pr0 = nr;
    }
    // (resid / stem are read by this kernel only: the LDS copies are not written back)
    __syncthreads();  // (the next basin reuses the LDS)
  }
}

// the first pass's split threshold (graph.cpp plan_init: cap x 100 % without a dominant basin, 80 % with
// one), from the largest basin -- so the host reads the statistics only with the first piece table
__global__ void k_scap(int64_t n, int64_t cap, int32_t pct_override, int32_t* agg) {
  const int64_t pct = pct_override > 0 ? pct_override : ((int64_t)agg[2] * 10 < n ? 100 : 80);
  agg[3] = (int32_t)(cap * pct / 100);
}

// piece roots: outlets and the reaches the split cut off
__global__ void k_piece_flags(int64_t n, const int32_t* down, uint8_t* is_root, int32_t* f) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool r = down[i] < 0 || is_root[i];
  is_root[i] = r ? 1 : 0;
  f[i] = r ? 1 : 0;
}
// piece of every reach (numbered by descending root index: np - 1 - rank of its root) and the piece
// table (graph.cpp PieceTable); tab is [8][np]
__global__ void k_pieces(int64_t n, const int32_t* np_dev, const int32_t* down, const int32_t* prank, const int32_t* q,
                         int32_t* piece) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) piece[i] = *np_dev - 1 - prank[q[i]];
}
// column c of piece p at tab[c * n + p]
__global__ void k_piece_table(int64_t n, const int32_t* down, const uint8_t* is_root, const int32_t* piece,
                              const int32_t* dloc, const int32_t* crow, const int32_t* ht, const int32_t* dist,
                              int32_t* tab) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = i < n;
  const int32_t p = in ? piece[i] : 0;
  wave_atomic<0>(tab + 1 * n, p, 1, in);
  wave_atomic<1>(tab + 2 * n, p, in ? dloc[i] : 0, in);
  const int32_t deg = in ? crow[i + 1] - crow[i] : 0;
  wave_atomic<0>(tab + 3 * n, p, deg, in && deg > 2);
  if (!in) return;
  if (is_root[i]) {
    const int32_t d = down[i];
    tab[0 * n + p] = (int32_t)i;
    tab[4 * n + p] = d < 0 ? -1 : piece[d];
    tab[5 * n + p] = d < 0 ? 0 : dloc[d];
    tab[6 * n + p] = ht[i];
    tab[7 * n + p] = dist[i];
  }
}

// ---- schedule emission --------------------------------------------------------------------------
__global__ void k_emit_key(int64_t n, const int32_t* piece, const int32_t* dloc, const int32_t* bop,
                           const int32_t* bdmax, int64_t omax1, int32_t* blk, int32_t* offv, uint64_t* key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t b = bop[piece[i]];
  const int32_t o = bdmax[b] - dloc[i];
  blk[i] = b;
  offv[i] = o;
  key[i] = (uint64_t)b * (uint64_t)omax1 + (uint64_t)o;
}
// per internal position: reach, counts for the prefix sums
__global__ void k_emit_counts(int64_t n, const int32_t* order, const int32_t* blk, const int32_t* down,
                              const int32_t* crow, const int32_t* col, const BlockDesc* blocks, int32_t* pos,
                              int32_t* local, int32_t* upc, int32_t* cutf, int32_t* nv, int32_t* nx,
                              int32_t* pos_of_ref, int32_t* block_of_pos) {
  const int64_t P = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (P >= n) return;
  const int32_t i = order[P];
  const int32_t b = blk[i];
  pos[i] = (int32_t)P;
  local[i] = (int32_t)(P - blocks[b].pos0);
  pos_of_ref[i] = (int32_t)P;
  block_of_pos[P] = b;
  const int32_t k0 = crow[i], k1 = crow[i + 1];
  upc[P] = k1 - k0;
  const int32_t d = down[i];
  cutf[P] = (d >= 0 && blk[d] != b) ? 1 : 0;
  int32_t v = 0;
  for (int32_t k = k0; k < k1; ++k) v += (blk[col[k]] != b);
  nv[P] = v;
  nx[P] = (k1 - k0) > 2 ? (k1 - k0) : 0;
}
__global__ void k_emit_cut(int64_t n, const int32_t* order, const int32_t* blk, const int32_t* down,
                           const int32_t* local, const BlockDesc* blocks, const int32_t* cutf, const int32_t* eid,
                           const int32_t* nx, const int32_t* xbase, int32_t* ref, int32_t* offs, const int32_t* offv,
                           int32_t* cut, int32_t* cout_loc, int32_t* edge_of, int32_t* xoff, int32_t* dl) {
  const int64_t P = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (P >= n) return;
  const int32_t i = order[P];
  const int32_t b = blk[i];
  const BlockDesc& B = blocks[b];
  ref[P] = i;
  offs[P] = offv[i];
  if (cutf[P]) {
    cut[P] = eid[P];
    cout_loc[eid[P]] = (int32_t)(P - B.pos0);
    edge_of[i] = eid[P];
  } else {
    cut[P] = -1;
    edge_of[i] = -1;
  }
  xoff[P] = nx[P] ? xbase[P] - B.xl0 : -1;
  const int32_t d = down[i];
  dl[P] = (d >= 0 && blk[d] == b) ? local[d] : -1;
}
__global__ void k_emit_up(int64_t n, const int32_t* order, const int32_t* blk, const int32_t* crow,
                          const int32_t* col, const int32_t* local, const BlockDesc* blocks, const int32_t* upb,
                          const int32_t* vbase, const int32_t* nx, const int32_t* xbase, const int32_t* offv,
                          const int32_t* edge_of, int32_t* uplist, int32_t* v_edge, int32_t* v_off,
                          int32_t* v_dloc, int32_t* xlist) {
  const int64_t P = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (P >= n) return;
  const int32_t i = order[P];
  const int32_t b = blk[i];
  const BlockDesc& B = blocks[b];
  const int32_t k0 = crow[i], k1 = crow[i + 1];
  const int32_t u0 = upb[P];
  int32_t v = vbase[P];
  for (int32_t k = k0; k < k1; ++k) {
    const int32_t j = col[k];
    int32_t u;
    if (blk[j] == b) {
      u = local[j];
    } else {
      // virtual inflow of cut edge j -> i
      u = B.nloc + (v - B.virt0);
      v_edge[v] = edge_of[j];
      v_off[v] = offv[i] - 1;
      v_dloc[v] = (int32_t)(P - B.pos0);
      ++v;
    }
    uplist[u0 + (k - k0)] = u;
  }
  if (nx[P]) {
    // confluence list: [c, u1, ..., u_{c-1}] (route.hip pack_up)
    const int32_t x = xbase[P];
    xlist[x] = k1 - k0;
    for (int32_t k = 1; k < k1 - k0; ++k) xlist[x + k] = uplist[u0 + k];
  }
}
__global__ void k_rs_loc(int64_t n, const int32_t* rs_ref, const int32_t* local, int32_t* rs_loc) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) rs_loc[k] = local[rs_ref[k]];
}
__global__ void k_widen(int64_t n, const int32_t* a, int64_t* b) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = a[i];
}


// ---- per-batch gauge union on the device (builders.py:55-109, merit.py:197-238) -----------------
// union of the subsets' (row, col) pairs keyed by the upstream reach (dendritic: one downstream each),
// active marks of rows, cols and gauges (CONUS numbering)
__global__ void k_union(int64_t n_conus, int64_t e, const int32_t* rows, const int32_t* cols, int32_t* down,
                        int32_t* mark, unsigned long long* err) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= e) return;
  const int32_t r = rows[k], c = cols[k];
  if (r < 0 || r >= n_conus || c < 0 || c >= n_conus) {
    atomicMin(err + kErrRange, (unsigned long long)k);
    return;
  }
  if (c >= r) {
    atomicMin(err + kErrLower, (unsigned long long)k);
    return;
  }
  const int32_t old = atomicCAS(down + c, -1, r);
  if (old != -1 && old != r) atomicMin(err + kErrDend, (unsigned long long)c);
  mark[r] = 1;
  mark[c] = 1;
}
__global__ void k_mark_gauges(int64_t n_conus, int64_t G, const int32_t* gidx, int32_t* mark,
                              unsigned long long* err) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  const int32_t x = gidx[g];
  if (x < 0 || x >= n_conus) atomicMin(err + kErrRange, (unsigned long long)g);
  else mark[x] = 1;
}
// active reaches in CONUS (= topological) order; the compressed downstream of each
__global__ void k_compress(int64_t n_conus, const int32_t* mark, const int32_t* remap, const int32_t* down,
                           int32_t* active, int32_t* down_c) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_conus || !mark[i]) return;
  const int32_t a = remap[i];
  active[a] = (int32_t)i;
  down_c[a] = down[i] >= 0 ? remap[down[i]] : -1;
}
__global__ void k_has_down(int64_t n, const int32_t* down_c, int32_t* f, int32_t* deg) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= n) return;
  f[a] = down_c[a] >= 0 ? 1 : 0;
  if (down_c[a] >= 0) atomicAdd(deg + down_c[a], 1);
}
__global__ void k_union_coo(int64_t n, const int32_t* down_c, const int32_t* kpos, int32_t* rows_c, int32_t* cols_c) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a < n && down_c[a] >= 0) {
    rows_c[kpos[a]] = down_c[a];
    cols_c[kpos[a]] = (int32_t)a;
  }
}
// outflow_idx of gauge g: the compressed upstream reaches of its reach (ascending), itself without any
__global__ void k_outflow_count(int64_t G, const int32_t* gidx, const int32_t* remap, const int32_t* crow,
                                int32_t* gage_c, int64_t* cnt) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  const int32_t x = remap[gidx[g]];
  gage_c[g] = x;
  const int32_t d = crow[x + 1] - crow[x];
  cnt[g] = d > 0 ? d : 1;
}
__global__ void k_outflow_fill(int64_t G, const int32_t* gage_c, const int32_t* crow, const int32_t* col,
                               const int64_t* off, int32_t* out_idx) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  const int32_t x = gage_c[g];
  const int32_t k0 = crow[x], k1 = crow[x + 1];
  const int64_t o = off[g];
  if (k1 == k0) out_idx[o] = x;
  for (int32_t k = k0; k < k1; ++k) out_idx[o + (k - k0)] = col[k];
}

// Temporaries of one build (pooled device blocks), returned stream-ordered when the build returns.
struct Scratch {
  hipStream_t s;
  std::vector<void*> ptrs;
  hipError_t err = hipSuccess;
  explicit Scratch(hipStream_t st) : s(st) {}
  template <typename T>
  T* get(int64_t n) {
    void* p = device_get((size_t)std::max<int64_t>(n, 1) * sizeof(T), s);
    if (!p) {
      err = hipErrorOutOfMemory;
      return nullptr;
    }
    ptrs.push_back(p);
    return static_cast<T*>(p);
  }
  ~Scratch() {
    for (void* p : ptrs) device_put(p, s);
  }
};

#define DDR_SCR(ptr)                                                        \
  do {                                                                      \
    if (!(ptr)) return ::ddr::hip_fail(scr.err, "device graph: scratch allocation"); \
  } while (0)

template <typename T>
ddr_status exclusive_sum(Scratch& scr, const T* in, T* out, int64_t n, hipStream_t s) {
  size_t bytes = 0;
  DDR_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, (int)n, s));
  void* tmp = scr.get<unsigned char>((int64_t)bytes);
  DDR_SCR(tmp);
  DDR_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, bytes, in, out, (int)n, s));
  return DDR_OK;
}
template <typename K>
ddr_status sort_pairs(Scratch& scr, const K* kin, K* kout, const int32_t* vin, int32_t* vout, int64_t n, int bits,
                      hipStream_t s) {
  size_t bytes = 0;
  DDR_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, kin, kout, vin, vout, (int)n, 0, bits, s));
  void* tmp = scr.get<unsigned char>((int64_t)bytes);
  DDR_SCR(tmp);
  DDR_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, bytes, kin, kout, vin, vout, (int)n, 0, bits, s));
  return DDR_OK;
}

// Pointer jumping to the nearest ancestor-or-self with down < 0 (or stop[i] != 0): p = that reach,
// d = hops to it.  `rounds` >= ceil(log2(longest path)) + 1.
ddr_status jump(Scratch& scr, int64_t n, const int32_t* down, const uint8_t* stop, int rounds, int32_t*& p,
                int32_t*& d, hipStream_t s) {
  int32_t* p2 = scr.get<int32_t>(n);
  int32_t* d2 = scr.get<int32_t>(n);
  DDR_SCR(p2);
  DDR_SCR(d2);
  hipLaunchKernelGGL(k_jump_init, dim3(nblk(n)), dim3(kTB), 0, s, n, down, stop, p, d);
  for (int r = 0; r < rounds; ++r) {
    hipLaunchKernelGGL(k_jump, dim3(nblk(n)), dim3(kTB), 0, s, n, p, d, p2, d2);
    std::swap(p, p2);
    std::swap(d, d2);
  }
  DDR_HIP(hipGetLastError());
  return DDR_OK;
}

// The default memory pool returns freed memory to the driver at every synchronisation unless told to
// keep it: a build per training batch would then pay fresh allocations each time.

int log2_rounds(int64_t len) {
  int r = 1;
  while ((int64_t(1) << (r - 1)) < len + 1) ++r;
  return r;
}

}  // namespace

// One device build in two halves (ddr_graph_build_device_begin / _finish): begin() enqueues every
// device pass up to the first piece table and its copy into pinned host memory, without waiting for
// anything; finish() waits for that copy (by then long done when the build was begun a training step
// ahead), packs the pieces on the host, and enqueues the schedule emission.  A re-split (the packer
// changed the plan: rare, see plan_init) costs one synchronous round trip per extra pass.
struct DevBuild {
  int64_t n = 0, e = 0;
  const int32_t* rows = nullptr;
  const int32_t* cols = nullptr;
  ddr_build_opts opts{};
  bool has_opts = false;
  hipStream_t s = nullptr;
  Scratch scr;
  std::unique_ptr<Graph> g;
  bool dbg = false, tdbg = false;
  double t_begin = 0.0, t_pack = 0.0, t_wait = 0.0;
  // device arrays
  int32_t *down = nullptr, *deg = nullptr, *agg = nullptr, *crow = nullptr, *iota = nullptr, *kids = nullptr;
  unsigned long long* err = nullptr;
  int32_t *basin = nullptr, *dist = nullptr, *ord = nullptr, *seg_lo = nullptr, *seg_hi = nullptr, *lvl_next = nullptr;
  int32_t *roots = nullptr, *sub = nullptr, *ht = nullptr, *resid = nullptr, *stem = nullptr, *pflag = nullptr;
  int32_t *prank = nullptr, *q = nullptr, *dloc = nullptr, *piece = nullptr, *tab = nullptr;
  int32_t* inv = nullptr;            // level position of every reach (level walks in LDS)
  SplitRow* split_tab = nullptr;     // the split's static inputs per level position (k_split_lds)
  bool level_lds = true;
  uint8_t* is_root = nullptr;
  unsigned basin_grid = 1;
  // host side of the piece-table reads: pinned, so the copies are truly asynchronous
  struct Pinned {
    unsigned long long err[kErrWords];
    int32_t agg[4];
    int32_t np;
  };
  Pinned* pin = nullptr;
  int32_t* ptab = nullptr;  // [8][guess] pinned
  int64_t guess = 0;
  hipEvent_t tab_ev = nullptr;
  PackPlan plan;
  bool first = true;
  int64_t D = 0, prev_np = 0;

  explicit DevBuild(hipStream_t st) : s(st), scr(st) {}
  ~DevBuild() {
    // a build that failed after the slab or the staging block was attached: both go back to their pools
    // stream-ordered (after whatever the build queued on s), not leaked as handed out
    if (g) destroy_graph(g.release(), s);
    if (tab_ev) (void)hipEventDestroy(tab_ev);
    pinned_put(pin, s);  // its copies were waited for (read_table), or are queued on s
    pinned_put(ptab, s);
  }
  const ddr_build_opts* options() const { return has_opts ? &opts : nullptr; }

  void phase(const char* what, double& tp) const {
    if (!dbg) return;
    (void)hipStreamSynchronize(s);
    const double t = now_ms();
    fprintf(stderr, "[dpart] %-10s %8.2f ms\n", what, t - tp);
    tp = t;
  }

  ddr_status begin() {
    g = std::make_unique<Graph>();
    g->n = n;
    g->nnz = e;
    double tp = now_ms();
    // ---- validation, down[], CSR --------------------------------------------------------------
    down = scr.get<int32_t>(n);
    deg = scr.get<int32_t>(n + 1);
    err = scr.get<unsigned long long>(kErrWords);
    agg = scr.get<int32_t>(4);
    DDR_SCR(down);
    DDR_SCR(deg);
    DDR_SCR(err);
    DDR_SCR(agg);
    DDR_HIP(hipMemsetAsync(down, 0xFF, sizeof(int32_t) * n, s));
    DDR_HIP(hipMemsetAsync(deg, 0, sizeof(int32_t) * (n + 1), s));
    DDR_HIP(hipMemsetAsync(err, 0xFF, sizeof(unsigned long long) * kErrWords, s));
    DDR_HIP(hipMemsetAsync(agg, 0, sizeof(int32_t) * 4, s));
    if (e > 0) hipLaunchKernelGGL(k_coo, dim3(nblk(e)), dim3(kTB), 0, s, n, e, rows, cols, down, deg, err);
    DDR_HIP(hipGetLastError());
    crow = scr.get<int32_t>(n + 1);
    DDR_SCR(crow);
    ddr_status st;
    if ((st = exclusive_sum<int32_t>(scr, deg, crow, n + 1, s))) return st;
    uint32_t* dkey = scr.get<uint32_t>(n);
    uint32_t* dkey2 = scr.get<uint32_t>(n);
    iota = scr.get<int32_t>(n);
    kids = scr.get<int32_t>(n);  // reaches sorted by (downstream, index): the CSR's col
    DDR_SCR(dkey);
    DDR_SCR(dkey2);
    DDR_SCR(iota);
    DDR_SCR(kids);
    hipLaunchKernelGGL(k_down_key, dim3(nblk(n)), dim3(kTB), 0, s, n, down, dkey);
    hipLaunchKernelGGL(k_iota, dim3(nblk(n)), dim3(kTB), 0, s, iota, n);
    DDR_HIP(hipGetLastError());
    if ((st = sort_pairs<uint32_t>(scr, dkey, dkey2, iota, kids, n, bits_for((uint64_t)n), s))) return st;
    // ---- distance to outlet, basin --------------------------------------------------------------
    basin = scr.get<int32_t>(n);
    dist = scr.get<int32_t>(n);
    DDR_SCR(basin);
    DDR_SCR(dist);
    if ((st = jump(scr, n, down, nullptr, log2_rounds(n), basin, dist, s))) return st;
    int32_t* bsize = scr.get<int32_t>(n);
    DDR_SCR(bsize);
    DDR_HIP(hipMemsetAsync(bsize, 0, sizeof(int32_t) * n, s));
    hipLaunchKernelGGL(k_stats, dim3(nblk(n)), dim3(kTB), 0, s, n, down, basin, dist, bsize, agg);
    hipLaunchKernelGGL(k_bmax, dim3(nblk(n)), dim3(kTB), 0, s, n, down, bsize, agg);
    DDR_HIP(hipGetLastError());
    phase("csr+tree", tp);
    // (no host round trip yet: the error words and the statistics are read with the first piece table)
    // ---- level order per basin (deepest level first), subtree size and height ------------------
    uint64_t* lkey = scr.get<uint64_t>(n);
    uint64_t* lkey2 = scr.get<uint64_t>(n);
    ord = scr.get<int32_t>(n);
    int32_t* smark = scr.get<int32_t>(n);
    int32_t* smax = scr.get<int32_t>(n);
    seg_lo = scr.get<int32_t>(n);
    seg_hi = scr.get<int32_t>(n);
    lvl_next = scr.get<int32_t>(n);
    int32_t* oflag = scr.get<int32_t>(n + 1);
    int32_t* orank = scr.get<int32_t>(n + 1);
    roots = scr.get<int32_t>(n);
    sub = scr.get<int32_t>(n);
    ht = scr.get<int32_t>(n);
    DDR_SCR(lkey); DDR_SCR(lkey2); DDR_SCR(ord); DDR_SCR(smark); DDR_SCR(smax); DDR_SCR(seg_lo); DDR_SCR(seg_hi);
    DDR_SCR(lvl_next); DDR_SCR(oflag); DDR_SCR(orank); DDR_SCR(roots); DDR_SCR(sub); DDR_SCR(ht);
    // key = basin * n + (n - 1 - dist): the depth bound n - 1 stands in for the deepest reach (unknown here)
    hipLaunchKernelGGL(k_level_key, dim3(nblk(n)), dim3(kTB), 0, s, n, basin, dist, n - 1, lkey);
    DDR_HIP(hipGetLastError());
    if ((st = sort_pairs<uint64_t>(scr, lkey, lkey2, iota, ord, n,
                                   bits_for((uint64_t)(n - 1) * (uint64_t)n + (uint64_t)(n - 1)), s)))
      return st;
    hipLaunchKernelGGL(k_level_marks, dim3(nblk(n)), dim3(kTB), 0, s, n, lkey2, ord, basin, smark, seg_lo, seg_hi);
    DDR_HIP(hipGetLastError());
    {
      size_t bytes = 0;
      DDR_HIP(hipcub::DeviceScan::InclusiveScan(nullptr, bytes, smark, smax, hipcub::Max(), (int)n, s));
      void* tmp = scr.get<unsigned char>((int64_t)bytes);
      DDR_SCR(tmp);
      DDR_HIP(hipcub::DeviceScan::InclusiveScan(tmp, bytes, smark, smax, hipcub::Max(), (int)n, s));
    }
    hipLaunchKernelGGL(k_level_links, dim3(nblk(n)), dim3(kTB), 0, s, n, lkey2, smax, lvl_next);
    hipLaunchKernelGGL(k_is_outlet, dim3(nblk(n)), dim3(kTB), 0, s, n, down, oflag);
    DDR_HIP(hipGetLastError());
    if ((st = exclusive_sum<int32_t>(scr, oflag, orank, n, s))) return st;
    hipLaunchKernelGGL(k_roots, dim3(nblk(n)), dim3(kTB), 0, s, n, down, orank, roots);
    basin_grid = (unsigned)std::min<int64_t>(n, 8192);  // workgroups striding over the basins
    {
      const char* v = getenv("DDR_DEVBUILD_LEVEL_LDS");
      level_lds = v == nullptr || atoi(v) != 0;
    }
    if (level_lds) {
      inv = scr.get<int32_t>(n);
      int32_t* ccnt = scr.get<int32_t>(n);
      int4* cpos = scr.get<int4>(n);
      split_tab = scr.get<SplitRow>(n);
      DDR_SCR(inv); DDR_SCR(ccnt); DDR_SCR(cpos); DDR_SCR(split_tab);
      hipLaunchKernelGGL(k_inv, dim3(nblk(n)), dim3(kTB), 0, s, n, ord, inv);
      hipLaunchKernelGGL(k_child_tab, dim3(nblk(n)), dim3(kTB), 0, s, n, ord, crow, kids, inv, ccnt, cpos);
      const int lds = kLevelLds * 6;
      DDR_HIP(hipFuncSetAttribute((const void*)k_sub_ht_lds, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
      hipLaunchKernelGGL(k_sub_ht_lds, dim3(basin_grid), dim3(256), lds, s, roots, agg + 1, seg_lo, seg_hi, lvl_next, ord,
                         crow, kids, inv, ccnt, cpos, sub, ht);
      hipLaunchKernelGGL(k_split_tab, dim3(nblk(n)), dim3(kTB), 0, s, n, ord, ccnt, cpos, sub, ht, split_tab);
    } else {
      hipLaunchKernelGGL(k_sub_ht, dim3(basin_grid), dim3(256), 0, s, roots, agg + 1, seg_lo, seg_hi, lvl_next, ord, crow,
                         kids, sub, ht);
    }
    DDR_HIP(hipGetLastError());
    phase("sub+ht", tp);
    // ---- the first split pass (its threshold chosen on the device from the largest basin) -----
    if ((st = plan_init(n, 0, options(), plan))) return st;
#ifdef DDR_SCAP_PCT
    const int32_t pct_override = DDR_SCAP_PCT;
#else
    const int32_t pct_override = 0;
#endif
    hipLaunchKernelGGL(k_scap, dim3(1), dim3(1), 0, s, n, plan.cap, pct_override, agg);
    g->device = plan.device;
    resid = scr.get<int32_t>(n);
    stem = scr.get<int32_t>(n);
    is_root = scr.get<uint8_t>(n);
    pflag = scr.get<int32_t>(n + 1);
    prank = scr.get<int32_t>(n + 1);
    q = scr.get<int32_t>(n);
    dloc = scr.get<int32_t>(n);
    piece = scr.get<int32_t>(n);
    tab = scr.get<int32_t>(8 * n);
    DDR_SCR(resid); DDR_SCR(stem); DDR_SCR(is_root); DDR_SCR(pflag); DDR_SCR(prank); DDR_SCR(q); DDR_SCR(dloc);
    DDR_SCR(piece); DDR_SCR(tab);
    pin = static_cast<Pinned*>(pinned_get(sizeof(Pinned)));
    guess = std::min<int64_t>(n, 16384);
    ptab = static_cast<int32_t*>(pinned_get(sizeof(int32_t) * 8 * (size_t)guess));
    if (!pin || !ptab) return fail(DDR_ERR_HIP, "device graph: pinned host memory");
    DDR_HIP(hipEventCreateWithFlags(&tab_ev, hipEventDisableTiming));
    D = n - 1;
    return pass();
  }

  // Enqueue one split pass with the current plan and the read of its piece table.
  ddr_status pass() {
    ddr_status st;
    DDR_HIP(hipMemsetAsync(is_root, 0, n, s));
    if (level_lds) {
      const int lds = kLevelLds * 6;
      DDR_HIP(hipFuncSetAttribute((const void*)k_split_lds, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
      hipLaunchKernelGGL(k_split_lds, dim3(basin_grid), dim3(256), lds, s, roots, agg + 1, seg_lo, seg_hi, lvl_next, ord,
                         crow, kids, inv, split_tab, sub, ht, resid, stem, is_root, first ? int64_t(-1) : plan.scap(), agg);
    } else {
      hipLaunchKernelGGL(k_split, dim3(basin_grid), dim3(256), 0, s, roots, agg + 1, seg_lo, seg_hi, lvl_next, ord, crow,
                         kids, sub, ht, resid, stem, is_root, first ? int64_t(-1) : plan.scap(), agg);
    }
    hipLaunchKernelGGL(k_piece_flags, dim3(nblk(n)), dim3(kTB), 0, s, n, down, is_root, pflag);
    DDR_HIP(hipGetLastError());
    DDR_HIP(hipMemsetAsync(pflag + n, 0, 4, s));  // prank[n] = number of pieces
    if ((st = exclusive_sum<int32_t>(scr, pflag, prank, n + 1, s))) return st;
    if ((st = jump(scr, n, down, is_root, log2_rounds(first ? n : D + 1), q, dloc, s))) return st;
    // the table is [8][n] (column stride n: no host round trip for the piece count first); a bounded
    // prefix of every column and the count go to pinned memory, a second read only for many pieces
    hipLaunchKernelGGL(k_pieces, dim3(nblk(n)), dim3(kTB), 0, s, n, prank + n, down, prank, q, piece);
    DDR_HIP(hipMemsetAsync(tab, 0, sizeof(int32_t) * 8 * (size_t)n, s));
    hipLaunchKernelGGL(k_piece_table, dim3(nblk(n)), dim3(kTB), 0, s, n, down, is_root, piece, dloc, crow, ht, dist,
                       tab);
    DDR_HIP(hipGetLastError());
    DDR_HIP(hipMemcpyAsync(&pin->np, prank + n, 4, hipMemcpyDeviceToHost, s));
    DDR_HIP(hipMemcpy2DAsync(ptab, sizeof(int32_t) * guess, tab, sizeof(int32_t) * n, sizeof(int32_t) * guess, 8,
                             hipMemcpyDeviceToHost, s));
    if (first) {
      DDR_HIP(hipMemcpyAsync(pin->err, err, sizeof(pin->err), hipMemcpyDeviceToHost, s));
      DDR_HIP(hipMemcpyAsync(pin->agg, agg, sizeof(pin->agg), hipMemcpyDeviceToHost, s));
    }
    DDR_HIP(hipEventRecord(tab_ev, s));
    return DDR_OK;
  }

  // Wait for the pass's table; validation errors and statistics on the first one.
  ddr_status read_table(PieceTable& pt) {
    ddr_status st;
    {
      const double t0 = now_ms();
      DDR_HIP(hipEventSynchronize(tab_ev));
      t_wait += now_ms() - t0;
    }
    if (first) {
      // errors in the host builder's order of precedence (graph.cpp): the first bad entry, then
      // duplicates, then a reach draining into two reaches.  (The passes so far ran on the forest the
      // valid entries form: no out-of-range access.)
      const unsigned long long none = ~0ull;
      const unsigned long long* herr = pin->err;
      auto entry = [&](unsigned long long k, int32_t* rc) -> ddr_status {
        DDR_HIP(hipMemcpy(rc, rows + k, 4, hipMemcpyDeviceToHost));
        DDR_HIP(hipMemcpy(rc + 1, cols + k, 4, hipMemcpyDeviceToHost));
        return DDR_OK;
      };
      int32_t rc[2];
      if (herr[kErrRange] != none || herr[kErrLower] != none) {
        if (herr[kErrRange] < herr[kErrLower]) return fail(DDR_ERR_ARG, "COO index out of range");
        if ((st = entry(herr[kErrLower], rc))) return st;
        return fail(DDR_ERR_NOT_LOWER, "adjacency entry (" + std::to_string(rc[0]) + "," + std::to_string(rc[1]) +
                                           ") is not strictly lower triangular (network not topologically sorted)");
      }
      if (herr[kErrDup] != none) {
        if ((st = entry(herr[kErrDup], rc))) return st;
        return fail(DDR_ERR_DUPLICATE, "duplicate edge (" + std::to_string(rc[0]) + "," + std::to_string(rc[1]) + ")");
      }
      if (herr[kErrDend] != none)
        return fail(DDR_ERR_NOT_DENDRITIC, "reach " + std::to_string(herr[kErrDend]) + " drains into two reaches");
      D = pin->agg[0];  // deepest reach's distance
      g->max_depth = D + 1;
      g->n_basins = pin->agg[1];
      PackPlan p2;
      if ((st = plan_init(n, pin->agg[2], options(), p2))) return st;
      plan.scap_pct = p2.scap_pct;  // the threshold k_scap chose (same rule)
      if (plan.scap() != pin->agg[3]) return fail(DDR_ERR_ARG, "internal: split threshold mismatch");
      first = false;
    }
    const int64_t np = pin->np;
    std::vector<int32_t> big;
    const int32_t* src = ptab;
    int64_t stride = guess;
    if (np > guess) {
      big.resize(8 * (size_t)np);
      DDR_HIP(hipMemcpy2D(big.data(), sizeof(int32_t) * np, tab, sizeof(int32_t) * n, sizeof(int32_t) * np, 8,
                          hipMemcpyDeviceToHost));
      src = big.data();
      stride = np;
    }
    prev_np = np;
    pt = PieceTable{};
    auto col_of = [&](int c, std::vector<int64_t>& v) { v.assign(src + (size_t)c * stride, src + (size_t)c * stride + np); };
    col_of(0, pt.root);
    col_of(1, pt.size);
    col_of(2, pt.dmax);
    col_of(3, pt.xl);
    col_of(4, pt.parent);
    col_of(5, pt.dloc_down);
    col_of(6, pt.ht_root);
    col_of(7, pt.dist_root);
    return DDR_OK;
  }

  ddr_status finish(Graph** out) {
    double tp = now_ms();
    ddr_status st;
    PieceTable pt;
    PackResult pr;
    for (;;) {
      if ((st = read_table(pt))) return st;
      phase("split", tp);
      int outcome = kPackDone;
      const double tpk = now_ms();
      if ((st = pack_pieces(plan, pt, pr, &outcome))) return st;
      t_pack += now_ms() - tpk;
      phase("pack", tp);
      if (outcome == kPackDone) break;
      if ((st = pass())) return st;  // a re-split: its table is waited for at the top of the loop
    }
    g->n_pieces = (int64_t)pt.count();
    if ((st = finalize_blocks(g.get(), plan, pr))) return st;
    const int64_t nb = pr.nblocks, ncut = pr.ncut, nx_total = g->n_xlist;
    const int32_t* col = kids;
    // ---- persistent arrays (one allocation) -------------------------------------------------
    const int64_t words = (n + 1) + e + 4 * n        // crow, col, down, dist, basin, block
                          + 11 * n + e               // ref off upb upc dloc cut xoff pos_of_ref block_of_pos rs_loc rs_ref, uplist
                          + 4 * ncut + nx_total;     // v_edge v_off v_dloc cout_loc, xlist
    const size_t bytes = sizeof(int32_t) * (size_t)words + sizeof(BlockDesc) * (size_t)nb + 64;
    // a pooled block: releasing a batch's graph (ddr_graph_destroy_async on the training stream) is
    // stream-ordered and never waits on the host (neither hipFree nor hipFreeAsync is called)
    void* slab = device_get(bytes, s);
    if (!slab) return fail(DDR_ERR_HIP, "device graph: out of device memory");
    g->async_allocations.push_back(slab);
    int32_t* w = static_cast<int32_t*>(slab);
    auto carve = [&](int64_t k) {
      int32_t* p = w;
      w += k;
      return p;
    };
    DeviceViews& V = g->dviews;
    V.crow = carve(n + 1);
    V.col = carve(e);
    V.down = carve(n);
    V.dist = carve(n);
    V.basin = carve(n);
    V.block = carve(n);
    DevSchedule& S = g->dev;
    S.ref = carve(n);
    S.off = carve(n);
    S.upb = carve(n);
    S.upc = carve(n);
    S.dloc = carve(n);
    S.cut = carve(n);
    S.xoff = carve(n);
    S.pos_of_ref = carve(n);
    S.block_of_pos = carve(n);
    S.rs_loc = carve(n);
    S.rs_ref = carve(n);
    S.uplist = carve(e);
    S.v_edge = carve(ncut);
    S.v_off = carve(ncut);
    S.v_dloc = carve(ncut);
    S.cout_loc = carve(ncut);
    S.xlist = carve(nx_total);
    {
      uintptr_t a = reinterpret_cast<uintptr_t>(w);
      a = (a + 15) & ~uintptr_t(15);
      S.blocks = reinterpret_cast<BlockDesc*>(a);
    }
    // host sources of the asynchronous uploads live as long as the graph (pinned: truly asynchronous)
    const size_t nstage = sizeof(BlockDesc) * (size_t)nb + sizeof(int32_t) * ((size_t)pt.count() + (size_t)nb);
    g->staging = pinned_get(std::max<size_t>(nstage, 16));
    if (!g->staging) return fail(DDR_ERR_HIP, "device graph: pinned host memory");
    BlockDesc* hblk = static_cast<BlockDesc*>(g->staging);
    std::copy(g->blocks.begin(), g->blocks.end(), hblk);
    int32_t* hbop = reinterpret_cast<int32_t*>(hblk + nb);
    int32_t* hbdmax = hbop + pt.count();
    for (size_t p = 0; p < pt.count(); ++p) hbop[p] = (int32_t)pr.block_of_piece[p];
    int64_t omax = 0;
    for (int64_t b = 0; b < nb; ++b) {
      hbdmax[b] = (int32_t)pr.bdmax[b];
      omax = std::max<int64_t>(omax, pr.bdmax[b]);
    }
    DDR_HIP(hipMemcpyAsync(S.blocks, hblk, sizeof(BlockDesc) * nb, hipMemcpyHostToDevice, s));
    DDR_HIP(hipMemcpyAsync(V.crow, crow, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToDevice, s));
    if (e > 0) DDR_HIP(hipMemcpyAsync(V.col, col, sizeof(int32_t) * e, hipMemcpyDeviceToDevice, s));
    DDR_HIP(hipMemcpyAsync(V.down, down, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, s));
    DDR_HIP(hipMemcpyAsync(V.dist, dist, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, s));
    DDR_HIP(hipMemcpyAsync(V.basin, basin, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, s));
    // ---- emission ------------------------------------------------------------------------------
    int32_t* bop = scr.get<int32_t>((int64_t)pt.count());
    int32_t* bdmax = scr.get<int32_t>(nb);
    uint64_t* ekey = scr.get<uint64_t>(n);
    uint64_t* ekey2 = scr.get<uint64_t>(n);
    int32_t* offv = scr.get<int32_t>(n);
    int32_t* order = scr.get<int32_t>(n);
    int32_t* pos = scr.get<int32_t>(n);
    int32_t* local = scr.get<int32_t>(n);
    int32_t* cutf = scr.get<int32_t>(n);
    int32_t* nv = scr.get<int32_t>(n);
    int32_t* nx = scr.get<int32_t>(n);
    int32_t* eid = scr.get<int32_t>(n);
    int32_t* vbase = scr.get<int32_t>(n);
    int32_t* xbase = scr.get<int32_t>(n);
    int32_t* edge_of = scr.get<int32_t>(n);
    uint32_t* bkey2 = scr.get<uint32_t>(n);
    DDR_SCR(bop); DDR_SCR(bdmax); DDR_SCR(ekey); DDR_SCR(ekey2); DDR_SCR(offv); DDR_SCR(order); DDR_SCR(pos);
    DDR_SCR(local); DDR_SCR(cutf); DDR_SCR(nv); DDR_SCR(nx); DDR_SCR(eid); DDR_SCR(vbase); DDR_SCR(xbase);
    DDR_SCR(edge_of); DDR_SCR(bkey2);
    DDR_HIP(hipMemcpyAsync(bop, hbop, sizeof(int32_t) * pt.count(), hipMemcpyHostToDevice, s));
    DDR_HIP(hipMemcpyAsync(bdmax, hbdmax, sizeof(int32_t) * nb, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_emit_key, dim3(nblk(n)), dim3(kTB), 0, s, n, piece, dloc, bop, bdmax, omax + 1, V.block, offv,
                       ekey);
    DDR_HIP(hipGetLastError());
    if ((st = sort_pairs<uint64_t>(scr, ekey, ekey2, iota, order, n,
                                   bits_for((uint64_t)(nb - 1) * (uint64_t)(omax + 1) + (uint64_t)omax), s)))
      return st;
    hipLaunchKernelGGL(k_emit_counts, dim3(nblk(n)), dim3(kTB), 0, s, n, order, V.block, down, crow, col, S.blocks, pos,
                       local, S.upc, cutf, nv, nx, S.pos_of_ref, S.block_of_pos);
    DDR_HIP(hipGetLastError());
    if ((st = exclusive_sum<int32_t>(scr, S.upc, S.upb, n, s))) return st;
    if ((st = exclusive_sum<int32_t>(scr, cutf, eid, n, s))) return st;
    if ((st = exclusive_sum<int32_t>(scr, nv, vbase, n, s))) return st;
    if ((st = exclusive_sum<int32_t>(scr, nx, xbase, n, s))) return st;
    hipLaunchKernelGGL(k_emit_cut, dim3(nblk(n)), dim3(kTB), 0, s, n, order, V.block, down, local, S.blocks, cutf, eid,
                       nx, xbase, S.ref, S.off, offv, S.cut, S.cout_loc, edge_of, S.xoff, S.dloc);
    hipLaunchKernelGGL(k_emit_up, dim3(nblk(n)), dim3(kTB), 0, s, n, order, V.block, crow, col, local, S.blocks, S.upb,
                       vbase, nx, xbase, offv, edge_of, S.uplist, S.v_edge, S.v_off, S.v_dloc, S.xlist);
    DDR_HIP(hipGetLastError());
    // per block, its reaches in ascending reference order (the q' gather's reads): a stable sort by block
    {
      const uint32_t* bk = reinterpret_cast<const uint32_t*>(V.block);
      if ((st = sort_pairs<uint32_t>(scr, bk, bkey2, iota, S.rs_ref, n,
                                     bits_for((uint64_t)std::max<int64_t>(nb - 1, 1)), s)))
        return st;
    }
    hipLaunchKernelGGL(k_rs_loc, dim3(nblk(n)), dim3(kTB), 0, s, n, S.rs_ref, local, S.rs_loc);
    DDR_HIP(hipGetLastError());
    // no final synchronisation: the graph is complete once `ready` fires; every launch that uses it
    // waits for the event on its own stream first (graph_ready)
    DDR_HIP(hipEventCreateWithFlags(&g->ready, hipEventDisableTiming));
    DDR_HIP(hipEventRecord(g->ready, s));
    phase("emit", tp);
    if (tdbg)
      fprintf(stderr, "[devbuild] n %ld begin->finish %.2f ms, waited %.2f ms, pack %.2f ms, blocks %ld gen %ld\n",
              (long)n, now_ms() - t_begin, t_wait, t_pack, (long)nb, (long)g->generations);
    g->uploaded = true;
    g->device_built = true;
    *out = g.release();
    return DDR_OK;
  }
};

ddr_status build_graph_device_begin(int64_t n, int64_t e, const int32_t* rows, const int32_t* cols,
                                    const ddr_build_opts* opts, hipStream_t s, DevBuild** out) {
  if (n <= 0) return fail(DDR_ERR_ARG, "graph must have at least one reach");
  if (n >= (int64_t(1) << 31) - 1 || e >= (int64_t(1) << 31) - 1)
    return fail(DDR_ERR_ARG, "graph too large for int32 reach ids");
  if (e < 0 || (e > 0 && (!rows || !cols))) return fail(DDR_ERR_ARG, "bad COO arrays");
  if (opts && (opts->flags & DDR_BUILD_HOST_ONLY)) return fail(DDR_ERR_ARG, "a device build cannot be host-only");
  auto b = std::make_unique<DevBuild>(s);
  b->n = n;
  b->e = e;
  b->rows = rows;
  b->cols = cols;
  if (opts) {
    b->opts = *opts;
    b->has_opts = true;
  }
  b->dbg = getenv("DDR_DEBUG_PART") != nullptr;
  b->tdbg = getenv("DDR_DEBUG_BUILD_TIMING") != nullptr;
  b->t_begin = now_ms();
  ddr_status st = b->begin();
  if (st) return st;
  *out = b.release();
  return DDR_OK;
}

ddr_status build_graph_device_finish(DevBuild* b, Graph** out) {
  std::unique_ptr<DevBuild> own(b);
  return b->finish(out);
}

void build_graph_device_cancel(DevBuild* b) { delete b; }

ddr_status build_graph_device(int64_t n, int64_t e, const int32_t* rows, const int32_t* cols,
                              const ddr_build_opts* opts, hipStream_t s, Graph** out) {
  DevBuild* b = nullptr;
  ddr_status st = build_graph_device_begin(n, e, rows, cols, opts, s, &b);
  if (st) return st;
  return build_graph_device_finish(b, out);
}

ddr_status collate_gauges_device(int64_t n_conus, int64_t n_gauges, int64_t e, const int32_t* rows,
                                 const int32_t* cols, const int32_t* gage_idx, int32_t* active, int64_t active_cap,
                                 int64_t* n_active_out, int32_t* rows_c, int32_t* cols_c, int64_t* nnz_out,
                                 int64_t* crow_out, int32_t* col_out, int64_t* out_off, int32_t* out_idx,
                                 int64_t out_idx_cap, int32_t* gage_c, hipStream_t s) {
  if (n_conus <= 0 || n_conus >= (int64_t(1) << 31) - 1) return fail(DDR_ERR_ARG, "bad CONUS size");
  if (e < 0 || e >= (int64_t(1) << 31) - 1 || (e > 0 && (!rows || !cols))) return fail(DDR_ERR_ARG, "bad subset COO");
  if (n_gauges < 0 || (n_gauges > 0 && (!gage_idx || !gage_c || !out_idx))) return fail(DDR_ERR_ARG, "bad gauge arrays");
  if (!active || !n_active_out || !nnz_out || !crow_out || !out_off || (e > 0 && (!rows_c || !cols_c || !col_out)))
    return fail(DDR_ERR_ARG, "null output");
  Scratch scr(s);
  int32_t* down = scr.get<int32_t>(n_conus);
  int32_t* mark = scr.get<int32_t>(n_conus + 1);
  int32_t* remap = scr.get<int32_t>(n_conus + 1);
  unsigned long long* err = scr.get<unsigned long long>(kErrWords);
  DDR_SCR(down);
  DDR_SCR(mark);
  DDR_SCR(remap);
  DDR_SCR(err);
  DDR_HIP(hipMemsetAsync(down, 0xFF, sizeof(int32_t) * n_conus, s));
  DDR_HIP(hipMemsetAsync(mark, 0, sizeof(int32_t) * (n_conus + 1), s));
  DDR_HIP(hipMemsetAsync(err, 0xFF, sizeof(unsigned long long) * kErrWords, s));
  if (e > 0) hipLaunchKernelGGL(k_union, dim3(nblk(e)), dim3(kTB), 0, s, n_conus, e, rows, cols, down, mark, err);
  if (n_gauges > 0)
    hipLaunchKernelGGL(k_mark_gauges, dim3(nblk(n_gauges)), dim3(kTB), 0, s, n_conus, n_gauges, gage_idx, mark, err);
  DDR_HIP(hipGetLastError());
  ddr_status st;
  if ((st = exclusive_sum<int32_t>(scr, mark, remap, n_conus + 1, s))) return st;
  unsigned long long herr[kErrWords];
  int32_t na = 0;
  DDR_HIP(hipMemcpyAsync(herr, err, sizeof(herr), hipMemcpyDeviceToHost, s));
  DDR_HIP(hipMemcpyAsync(&na, remap + n_conus, 4, hipMemcpyDeviceToHost, s));
  DDR_HIP(hipStreamSynchronize(s));
  const unsigned long long none = ~0ull;
  if (herr[kErrRange] != none) return fail(DDR_ERR_ARG, "subset COO index or gage_idx out of range");
  if (herr[kErrLower] != none) {
    int32_t rc[2];
    DDR_HIP(hipMemcpy(rc, rows + herr[kErrLower], 4, hipMemcpyDeviceToHost));
    DDR_HIP(hipMemcpy(rc + 1, cols + herr[kErrLower], 4, hipMemcpyDeviceToHost));
    return fail(DDR_ERR_NOT_LOWER, "subset entry (" + std::to_string(rc[0]) + "," + std::to_string(rc[1]) +
                                       ") is not strictly lower triangular");
  }
  if (herr[kErrDend] != none)
    return fail(DDR_ERR_NOT_DENDRITIC, "reach " + std::to_string(herr[kErrDend]) +
                                           " drains into two different reaches in the batch union");
  if (na > active_cap) return fail(DDR_ERR_ARG, "active reaches exceed active_cap");
  const int64_t n = na;
  int32_t* down_c = scr.get<int32_t>(n);
  int32_t* f = scr.get<int32_t>(n + 1);
  int32_t* kpos = scr.get<int32_t>(n + 1);
  int32_t* deg = scr.get<int32_t>(n + 1);
  int32_t* crow = scr.get<int32_t>(n + 1);
  DDR_SCR(down_c); DDR_SCR(f); DDR_SCR(kpos); DDR_SCR(deg); DDR_SCR(crow);
  DDR_HIP(hipMemsetAsync(deg, 0, sizeof(int32_t) * (n + 1), s));
  DDR_HIP(hipMemsetAsync(f + n, 0, 4, s));
  hipLaunchKernelGGL(k_compress, dim3(nblk(n_conus)), dim3(kTB), 0, s, n_conus, mark, remap, down, active, down_c);
  hipLaunchKernelGGL(k_has_down, dim3(nblk(n)), dim3(kTB), 0, s, n, down_c, f, deg);
  DDR_HIP(hipGetLastError());
  if ((st = exclusive_sum<int32_t>(scr, f, kpos, n + 1, s))) return st;
  if ((st = exclusive_sum<int32_t>(scr, deg, crow, n + 1, s))) return st;
  int32_t nnz = 0;
  DDR_HIP(hipMemcpyAsync(&nnz, kpos + n, 4, hipMemcpyDeviceToHost, s));
  hipLaunchKernelGGL(k_union_coo, dim3(nblk(n)), dim3(kTB), 0, s, n, down_c, kpos, rows_c, cols_c);
  // CSR columns: the compressed reaches sorted by (downstream, index) -- a stable radix sort
  uint32_t* key = scr.get<uint32_t>(n);
  uint32_t* key2 = scr.get<uint32_t>(n);
  int32_t* iota = scr.get<int32_t>(n);
  int32_t* kids = scr.get<int32_t>(n);
  DDR_SCR(key); DDR_SCR(key2); DDR_SCR(iota); DDR_SCR(kids);
  hipLaunchKernelGGL(k_down_key, dim3(nblk(n)), dim3(kTB), 0, s, n, down_c, key);
  hipLaunchKernelGGL(k_iota, dim3(nblk(n)), dim3(kTB), 0, s, iota, n);
  DDR_HIP(hipGetLastError());
  if ((st = sort_pairs<uint32_t>(scr, key, key2, iota, kids, n, bits_for((uint64_t)n), s))) return st;
  DDR_HIP(hipStreamSynchronize(s));
  if (nnz > 0) DDR_HIP(hipMemcpyAsync(col_out, kids, sizeof(int32_t) * nnz, hipMemcpyDeviceToDevice, s));
  hipLaunchKernelGGL(k_widen, dim3(nblk(n + 1)), dim3(kTB), 0, s, n + 1, crow, crow_out);
  if (n_gauges > 0) {
    int64_t* cnt = scr.get<int64_t>(n_gauges + 1);
    DDR_SCR(cnt);
    DDR_HIP(hipMemsetAsync(cnt + n_gauges, 0, 8, s));
    hipLaunchKernelGGL(k_outflow_count, dim3(nblk(n_gauges)), dim3(kTB), 0, s, n_gauges, gage_idx, remap, crow, gage_c,
                       cnt);
    DDR_HIP(hipGetLastError());
    if ((st = exclusive_sum<int64_t>(scr, cnt, out_off, n_gauges + 1, s))) return st;
    int64_t total = 0;
    DDR_HIP(hipMemcpyAsync(&total, out_off + n_gauges, 8, hipMemcpyDeviceToHost, s));
    DDR_HIP(hipStreamSynchronize(s));
    if (total > out_idx_cap)
      return fail(DDR_ERR_ARG, "outflow_idx lists exceed out_idx_cap (" + std::to_string(out_idx_cap) + " entries)");
    hipLaunchKernelGGL(k_outflow_fill, dim3(nblk(n_gauges)), dim3(kTB), 0, s, n_gauges, gage_c, crow, kids, out_off,
                       out_idx);
  } else {
    DDR_HIP(hipMemsetAsync(out_off, 0, 8, s));
  }
  DDR_HIP(hipGetLastError());
  DDR_HIP(hipStreamSynchronize(s));
  *n_active_out = n;
  *nnz_out = nnz;
  return DDR_OK;
}

// Host copies of the CSR / structure of a device-built graph (ddr_graph_csr, ddr_graph_structure).
ddr_status device_views_to_host(const Graph* g, int64_t* crow, int64_t* col, int64_t* down, int64_t* dist,
                                int64_t* basin, int64_t* block) {
  if (g->ready) DDR_HIP(hipEventSynchronize(g->ready));
  const DeviceViews& V = g->dviews;
  const int64_t n = g->n;
  std::vector<int32_t> tmp;
  auto get = [&](const int32_t* src, int64_t k, int64_t* dst) -> ddr_status {
    if (!dst || k == 0) return DDR_OK;
    tmp.resize(k);
    DDR_HIP(hipMemcpy(tmp.data(), src, sizeof(int32_t) * k, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < k; ++i) dst[i] = tmp[i];
    return DDR_OK;
  };
  ddr_status st;
  if ((st = get(V.crow, n + 1, crow))) return st;
  if ((st = get(V.col, g->nnz, col))) return st;
  if ((st = get(V.down, n, down))) return st;
  if ((st = get(V.dist, n, dist))) return st;
  if ((st = get(V.basin, n, basin))) return st;
  if ((st = get(V.block, n, block))) return st;
  return DDR_OK;
}

// The schedule arrays of a device-built graph, copied to the host (tests: compared with a host build).
ddr_status device_schedule_to_host(const Graph* g, HostSchedule& H) {
  if (g->ready) DDR_HIP(hipEventSynchronize(g->ready));
  const DevSchedule& S = g->dev;
  const int64_t n = g->n;
  auto get = [&](const int32_t* src, int64_t k, std::vector<int32_t>& dst) -> ddr_status {
    dst.resize(k);
    if (k) DDR_HIP(hipMemcpy(dst.data(), src, sizeof(int32_t) * k, hipMemcpyDeviceToHost));
    return DDR_OK;
  };
  ddr_status st;
  if ((st = get(S.ref, n, H.ref)) || (st = get(S.off, n, H.off)) || (st = get(S.upb, n, H.upb)) ||
      (st = get(S.upc, n, H.upc)) || (st = get(S.dloc, n, H.dloc)) || (st = get(S.cut, n, H.cut)) ||
      (st = get(S.xoff, n, H.xoff)) || (st = get(S.uplist, g->nnz, H.uplist)) ||
      (st = get(S.xlist, g->n_xlist, H.xlist)) || (st = get(S.v_edge, g->n_cut, H.v_edge)) ||
      (st = get(S.v_off, g->n_cut, H.v_off)) || (st = get(S.v_dloc, g->n_cut, H.v_dloc)) ||
      (st = get(S.cout_loc, g->n_cut, H.cout_loc)) || (st = get(S.pos_of_ref, n, H.pos_of_ref)) ||
      (st = get(S.block_of_pos, n, H.block_of_pos)) || (st = get(S.rs_loc, n, H.rs_loc)) ||
      (st = get(S.rs_ref, n, H.rs_ref)))
    return st;
  return DDR_OK;
}

}  // namespace ddr
