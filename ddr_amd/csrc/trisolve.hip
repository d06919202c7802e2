// General sparse triangular solve for the per-step API (routing/utils.py:695 triangular_sparse_solve)
// and the CSR value gradient (routing/utils.py:321-389).  Not on the fused hot path: the routing
// kernels never call it.  The matrix may have any lower-triangular pattern and a non-unit diagonal.
//
// Arithmetic follows SciPy's spsolve_triangular on fp64 copies (utils.py:587-600; SciPy 1.15.3):
// the matrix is right-scaled by diag^-1 (unit diagonal), the unit system is solved by a column sweep,
// then x = y * diag^-1.  Rows are processed level by level (host-computed level sets) inside one
// workgroup, so every accumulation keeps SciPy's order.
#include <algorithm>
#include <vector>

#include "internal.h"

namespace ddr {
namespace {

__global__ void __launch_bounds__(1024) tri_solve_kernel(int64_t n, const int64_t* lvl_ptr, int64_t nlvl,
                                                         const int64_t* order, const int64_t* eptr,
                                                         const int64_t* edep, const int64_t* eval,
                                                         const int64_t* diag_k, const float* values,
                                                         const float* b, double* y, float* x,
                                                         unsigned* singular) {
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const int64_t k = diag_k[i];
    const float d = k >= 0 ? values[k] : 0.0f;
    if (d == 0.0f) atomicOr(singular, 1u);
  }
  __syncthreads();
  for (int64_t l = 0; l < nlvl; ++l) {
    for (int64_t w = lvl_ptr[l] + threadIdx.x; w < lvl_ptr[l + 1]; w += blockDim.x) {
      const int64_t i = order[w];
      double acc = (double)b[i];
      for (int64_t e = eptr[i]; e < eptr[i + 1]; ++e) {
        const int64_t j = edep[e];
        const double invd_j = 1.0 / (double)values[diag_k[j]];
        const double lij = (double)values[eval[e]] * invd_j;
        acc = acc - lij * y[j];
      }
      y[i] = acc;
    }
    __syncthreads();
  }
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const double invd = 1.0 / (double)values[diag_k[i]];
    x[i] = (float)(y[i] * invd);
  }
}

__global__ void grad_values_kernel(int64_t n, const int64_t* crow, const int64_t* col, const float* gradb,
                                   const float* x, float* gv) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float g = gradb[i];
  for (int64_t k = crow[i]; k < crow[i + 1]; ++k) gv[k] = -g * x[col[k]];
}

}  // namespace
}  // namespace ddr

using namespace ddr;

extern "C" ddr_status ddr_tri_solve(int64_t n, int64_t nnz, const int64_t* crow, const int64_t* col,
                                    const float* values, const float* b, float* x, int32_t lower,
                                    int32_t transpose, void* stream) {
  try {
    if (n <= 0 || !crow || (nnz > 0 && !col) || !values || !b || !x) return fail(DDR_ERR_ARG, "bad tri_solve args");
    if (crow[0] != 0 || crow[n] != nnz) return fail(DDR_ERR_ARG, "inconsistent CSR row pointers");
    // Effective triangle of the system actually solved: A (lower/upper) or A^T.
    const bool eff_lower = transpose ? !lower : (bool)lower;
    std::vector<int64_t> diag_k(n, -1);
    // dependency lists per unknown: (dependency index j, value index k)
    std::vector<std::vector<std::pair<int64_t, int64_t>>> deps(n);
    for (int64_t i = 0; i < n; ++i) {
      for (int64_t k = crow[i]; k < crow[i + 1]; ++k) {
        const int64_t j = col[k];
        if (j < 0 || j >= n) return fail(DDR_ERR_ARG, "column index out of range");
        if (j == i) {
          diag_k[i] = k;
          continue;
        }
        const int64_t r = transpose ? j : i, c = transpose ? i : j;  // entry of the solved matrix
        if (eff_lower ? (c > r) : (c < r)) return fail(DDR_ERR_ARG, "entry outside the solved triangle");
        deps[r].push_back({c, k});
      }
    }
    for (int64_t i = 0; i < n; ++i)
      if (diag_k[i] < 0) return fail(DDR_ERR_SINGULAR, "A is singular: zero entry on diagonal");
    // SciPy column sweep order: lower -> ascending dependency, upper -> descending dependency
    for (auto& d : deps)
      std::sort(d.begin(), d.end(), [&](auto a, auto c) { return eff_lower ? a.first < c.first : a.first > c.first; });
    std::vector<int64_t> level(n, 0);
    int64_t nlvl = 0;
    auto visit = [&](int64_t i) {
      int64_t l = 0;
      for (auto& d : deps[i]) l = std::max(l, level[d.first] + 1);
      level[i] = l;
      nlvl = std::max(nlvl, l + 1);
    };
    if (eff_lower)
      for (int64_t i = 0; i < n; ++i) visit(i);
    else
      for (int64_t i = n - 1; i >= 0; --i) visit(i);
    std::vector<int64_t> lvl_ptr(nlvl + 1, 0), order(n), eptr(n + 1, 0), edep, eval;
    for (int64_t i = 0; i < n; ++i) lvl_ptr[level[i] + 1]++;
    for (int64_t l = 0; l < nlvl; ++l) lvl_ptr[l + 1] += lvl_ptr[l];
    std::vector<int64_t> fillp(lvl_ptr.begin(), lvl_ptr.end() - 1);
    for (int64_t i = 0; i < n; ++i) order[fillp[level[i]]++] = i;
    for (int64_t i = 0; i < n; ++i) {
      eptr[i + 1] = eptr[i] + (int64_t)deps[i].size();
      for (auto& d : deps[i]) {
        edep.push_back(d.first);
        eval.push_back(d.second);
      }
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    const size_t bytes_i = sizeof(int64_t) * ((nlvl + 1) + n + (n + 1) + 2 * edep.size() + n) + sizeof(double) * n + 16;
    char* buf = nullptr;
    DDR_HIP(hipMalloc(&buf, bytes_i));
    int64_t* d_lvl = reinterpret_cast<int64_t*>(buf);
    int64_t* d_order = d_lvl + (nlvl + 1);
    int64_t* d_eptr = d_order + n;
    int64_t* d_edep = d_eptr + (n + 1);
    int64_t* d_eval = d_edep + edep.size();
    int64_t* d_diag = d_eval + eval.size();
    double* d_y = reinterpret_cast<double*>(d_diag + n);
    unsigned* d_flag = reinterpret_cast<unsigned*>(d_y + n);
    auto up = [&](int64_t* dst, const std::vector<int64_t>& v) {
      return v.empty() ? hipSuccess : hipMemcpyAsync(dst, v.data(), sizeof(int64_t) * v.size(), hipMemcpyHostToDevice, s);
    };
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = up(d_lvl, lvl_ptr);
    if (e == hipSuccess) e = up(d_order, order);
    if (e == hipSuccess) e = up(d_eptr, eptr);
    if (e == hipSuccess) e = up(d_edep, edep);
    if (e == hipSuccess) e = up(d_eval, eval);
    if (e == hipSuccess) e = up(d_diag, diag_k);
    if (e == hipSuccess) e = hipMemsetAsync(d_flag, 0, sizeof(unsigned), s);
    if (e == hipSuccess) {
      hipLaunchKernelGGL(tri_solve_kernel, dim3(1), dim3(1024), 0, s, n, d_lvl, nlvl, d_order, d_eptr, d_edep, d_eval,
                         d_diag, values, b, d_y, x, d_flag);
      e = hipGetLastError();
    }
    unsigned flag = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&flag, d_flag, sizeof(unsigned), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(buf);
    if (e != hipSuccess) return hip_fail(e, "ddr_tri_solve");
    if (flag) return fail(DDR_ERR_SINGULAR, "A is singular: zero entry on diagonal");
    return DDR_OK;
  } catch (...) {
    return fail(DDR_ERR_ARG, "internal error in ddr_tri_solve");
  }
}

extern "C" ddr_status ddr_tri_grad_values(int64_t n, int64_t nnz, const int64_t* crow, const int64_t* col,
                                          const float* gradb, const float* x, float* gv, void* stream) {
  if (n <= 0 || !crow || !gradb || !x || (nnz > 0 && (!col || !gv))) return fail(DDR_ERR_ARG, "bad tri_grad args");
  const int threads = 256;
  hipLaunchKernelGGL(grad_values_kernel, dim3((unsigned)((n + threads - 1) / threads)), dim3(threads), 0,
                     static_cast<hipStream_t>(stream), n, crow, col, gradb, x, gv);
  DDR_HIP(hipGetLastError());
  return DDR_OK;
}
