// Per-batch gauge union: the subset COO adjacencies of a training batch's gauges (each in CONUS
// numbering) -> one compressed network (the active reaches, renumbered in CONUS order) as canonical
// CSR, the gauges' compressed indices and their outflow_idx lists.
//
// Reference behaviour reproduced (file:line in /root/reference):
//   src/ddr/io/builders.py:55-109        construct_network_matrix: union of (row, col) pairs (a set)
//   src/ddr/geodatazoo/merit.py:197-238  _collate_gages: active = unique(rows | cols | gauges),
//                                        compressed COO -> .tocsr(), outflow_idx, gage compressed idx
//   src/ddr/geodatazoo/lynker_hydrofabric.py:198-266 (the same steps)
// The reference builds a Python set of tuples and dict remaps per batch; here it is two passes over
// the edges and one over a CONUS-sized mark array.  Dendritic input means every upstream reach (col)
// has one downstream (row), so the union is keyed by col: a col seen with two different rows is a
// non-dendritic union and is rejected (the reference would pass it on to the solver).
#include <algorithm>
#include <cstring>
#include <vector>

#include "internal.h"

namespace ddr {

ddr_status collate_gauges(int64_t n_conus, int64_t n_gauges, const int64_t* sub_off, const int32_t* rows,
                          const int32_t* cols, const int32_t* gage_idx, int32_t* active, int64_t* n_active,
                          int64_t* crow, int32_t* col, int64_t* nnz, int64_t* out_off, int32_t* out_idx,
                          int64_t out_idx_cap, int32_t* gage_c) {
  if (n_conus <= 0 || n_conus >= (int64_t(1) << 31) - 1) return fail(DDR_ERR_ARG, "bad CONUS size");
  if (n_gauges < 0 || !sub_off || (n_gauges > 0 && !gage_idx)) return fail(DDR_ERR_ARG, "bad gauge arrays");
  if (!active || !n_active || !crow || !nnz || !out_off || (n_gauges > 0 && (!out_idx || !gage_c)))
    return fail(DDR_ERR_ARG, "null output");
  const int64_t e_all = sub_off[n_gauges];
  if (sub_off[0] != 0 || e_all < 0 || (e_all > 0 && (!rows || !cols || !col)))
    return fail(DDR_ERR_ARG, "bad subset offsets");
  for (int64_t g = 0; g < n_gauges; ++g)
    if (sub_off[g + 1] < sub_off[g]) return fail(DDR_ERR_ARG, "subset offsets must be non-decreasing");
  // downstream of every upstream reach in the union (-1: none), and the active mark
  std::vector<int32_t> down(n_conus, -1);
  std::vector<int32_t> remap(n_conus, -1);  // doubles as the mark (0) until renumbered
  for (int64_t k = 0; k < e_all; ++k) {
    const int32_t r = rows[k], c = cols[k];
    if (r < 0 || r >= n_conus || c < 0 || c >= n_conus) return fail(DDR_ERR_ARG, "subset COO index out of range");
    if (c >= r)
      return fail(DDR_ERR_NOT_LOWER, "subset entry (" + std::to_string(r) + "," + std::to_string(c) +
                                         ") is not strictly lower triangular");
    if (down[c] < 0) {
      down[c] = r;
    } else if (down[c] != r) {
      return fail(DDR_ERR_NOT_DENDRITIC, "reach " + std::to_string(c) + " drains into " + std::to_string(down[c]) +
                                             " and " + std::to_string(r) + " in the batch union");
    }
    remap[r] = remap[c] = 0;
  }
  for (int64_t g = 0; g < n_gauges; ++g) {
    const int32_t x = gage_idx[g];
    if (x < 0 || x >= n_conus) return fail(DDR_ERR_ARG, "gage_idx out of range");
    remap[x] = 0;
  }
  // active reaches in CONUS (= topological) order, renumbered 0..n_active-1
  int64_t na = 0;
  for (int64_t i = 0; i < n_conus; ++i)
    if (remap[i] == 0) {
      active[na] = (int32_t)i;
      remap[i] = (int32_t)na++;
    }
  *n_active = na;
  // canonical CSR of the compressed union: rows ascending; a row's columns ascending because the
  // upstream reaches are visited in ascending order
  std::fill(crow, crow + na + 1, 0);
  for (int64_t a = 0; a < na; ++a) {
    const int32_t d = down[active[a]];
    if (d >= 0) crow[remap[d] + 1]++;
  }
  for (int64_t a = 0; a < na; ++a) crow[a + 1] += crow[a];
  *nnz = crow[na];
  {
    std::vector<int64_t> fill(crow, crow + na);
    for (int64_t a = 0; a < na; ++a) {
      const int32_t d = down[active[a]];
      if (d >= 0) col[fill[remap[d]]++] = (int32_t)a;
    }
  }
  // outflow_idx: the compressed upstream reaches draining into each gauge reach (the gauge itself
  // for a headwater gauge), merit.py:227-235; gage compressed index, merit.py:237
  out_off[0] = 0;
  for (int64_t g = 0; g < n_gauges; ++g) {
    const int32_t x = remap[gage_idx[g]];
    gage_c[g] = x;
    const int64_t k0 = crow[x], k1 = crow[x + 1];
    int64_t o = out_off[g];
    // several gauges on one reach each list its inflows: inconsistent subsets can exceed E + G entries
    if (o + std::max<int64_t>(k1 - k0, 1) > out_idx_cap)
      return fail(DDR_ERR_ARG, "outflow_idx lists exceed out_idx_cap (" + std::to_string(out_idx_cap) + " entries)");
    if (k1 > k0) {
      for (int64_t k = k0; k < k1; ++k) out_idx[o++] = col[k];
    } else {
      out_idx[o++] = x;
    }
    out_off[g + 1] = o;
  }
  return DDR_OK;
}

}  // namespace ddr
