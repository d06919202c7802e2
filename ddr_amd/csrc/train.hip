// The tail of the C3 training step (bench.py --workload c3; the reference loop scripts/train.py:54-104) in three
// launches instead of ~15 PyTorch ones:
//   daily_l1_kernel   the objective, torch.nn.functional.l1_loss over gauges x days after the warm-up
//                     (train.py:91-94), and its gradient w.r.t. the daily series in the same pass;
//   adam_norm_kernel + adam_step_kernel  torch.nn.utils.clip_grad_norm_(max_norm) (train.py:99) and the Adam
//                     update (train.py:100, torch.optim.Adam without weight decay / amsgrad) over one flat
//                     parameter vector.
// The objective is one workgroup (G x D = 256 x 89 values: a few microseconds); the optimizer spreads its vector
// over 64 workgroups.  Both reductions are deterministic (fixed slices, LDS trees and partial order).
#include "internal.h"
#include "train.h"

namespace ddr {

namespace {

constexpr int kTThreads = 1024;

// fp64 sum of one value per thread over the workgroup (fixed tree: deterministic); every thread gets the total
__device__ double block_sum(double v, double* red) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
  for (int s = kTThreads / 2; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  const double t = red[0];
  __syncthreads();
  return t;
}

// loss = sum_{g, d >= wd} |daily[g, d] - obs[g, d]| * inv_count;  grad[g, d] = sign(daily - obs) * inv_count
// (0 before the warm-up; sign(0) = 0 as in PyTorch's abs backward)
__global__ void __launch_bounds__(kTThreads) daily_l1_kernel(int64_t G, int64_t D, int64_t wd, const float* daily,
                                                             const float* obs, float inv_count, float* loss,
                                                             float* grad) {
  __shared__ double red[kTThreads];
  double acc = 0.0;
  const int64_t total = G * D;
  for (int64_t i = threadIdx.x; i < total; i += kTThreads) {
    const int64_t d = i % D;
    float gv = 0.0f;
    if (d >= wd) {
      const float diff = daily[i] - obs[i];
      acc += (double)fabsf(diff);
      gv = diff > 0.0f ? inv_count : (diff < 0.0f ? -inv_count : (diff != diff ? diff : 0.0f));
    }
    if (grad) grad[i] = gv;
  }
  const double s = block_sum(acc, red);
  if (threadIdx.x == 0) loss[0] = (float)(s * (double)inv_count);
}

struct AdamArgs {
  int64_t n;
  float* param;
  const float* grad;
  float* m;
  float* v;
  float lr, beta1, beta2, eps;
  float* step;      // device step counter (fp32, like torch's capturable Adam): incremented by this update
  float max_norm;   // <= 0: no clipping
  float* norm_out;  // the gradient's total norm before clipping (clip_grad_norm_'s return value), or null
  double* partial;  // [kAdamWgs] per-workgroup sums of squares
};

// Two launches over kAdamWgs workgroups (a single workgroup spent ~40 us on a 34k-parameter vector in
// memory latency): sums of squares per workgroup slice, then every workgroup reduces the kAdamWgs partials
// in the same fixed order (deterministic, identical in every workgroup) and updates its slice.
constexpr int kAdamWgs = 64;
constexpr int kAdamThreads = 256;

__device__ double block_sum256(double v, double* red) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
  for (int s = kAdamThreads / 2; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  return red[0];
}

__global__ void __launch_bounds__(kAdamThreads) adam_norm_kernel(AdamArgs a) {
  __shared__ double red[kAdamThreads];
  double ss = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * kAdamThreads + threadIdx.x; i < a.n; i += (int64_t)kAdamWgs * kAdamThreads) {
    const float g = a.grad[i];
    ss += (double)g * (double)g;
  }
  const double s = block_sum256(ss, red);
  if (threadIdx.x == 0) a.partial[blockIdx.x] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) a.step[0] = a.step[0] + 1.0f;  // read by adam_step_kernel, next launch
}

__global__ void __launch_bounds__(kAdamThreads) adam_step_kernel(AdamArgs a) {
  __shared__ float coef_s, step_s, bc2s_s;
  if (threadIdx.x == 0) {
    // bias corrections of this step on the device (torch's capturable Adam: fp32 step tensor)
    const float t = a.step[0];
    step_s = a.lr / (1.0f - powf(a.beta1, t));
    bc2s_s = sqrtf(1.0f - powf(a.beta2, t));
    double s = 0.0;
    for (int w = 0; w < kAdamWgs; ++w) s += a.partial[w];
    const float norm = (float)sqrt(s);
    if (blockIdx.x == 0 && a.norm_out) a.norm_out[0] = norm;
    // clip_coef = max_norm / (norm + 1e-6), clamped to <= 1 (torch/nn/utils/clip_grad.py)
    coef_s = a.max_norm > 0.0f ? fminf(a.max_norm / (norm + 1e-6f), 1.0f) : 1.0f;
  }
  __syncthreads();
  const float coef = coef_s, step = step_s, bc2_sqrt = bc2s_s;
  const float omb1 = 1.0f - a.beta1, omb2 = 1.0f - a.beta2;
  for (int64_t i = (int64_t)blockIdx.x * kAdamThreads + threadIdx.x; i < a.n; i += (int64_t)kAdamWgs * kAdamThreads) {
    const float g = a.grad[i] * coef;
    const float m = fmaf(omb1, g - a.m[i], a.m[i]);           // exp_avg.lerp_(grad, 1 - beta1)
    const float v = fmaf(a.beta2, a.v[i], omb2 * g * g);      // exp_avg_sq * beta2 + (1 - beta2) g^2
    a.m[i] = m;
    a.v[i] = v;
    const float den = sqrtf(v) / bc2_sqrt + a.eps;
    a.param[i] = a.param[i] - step * (m / den);
  }
}

}  // namespace

hipError_t launch_daily_l1(int64_t G, int64_t D, int64_t wd, const float* daily, const float* obs, float inv_count,
                           float* loss, float* grad, hipStream_t stream) {
  hipLaunchKernelGGL(daily_l1_kernel, dim3(1), dim3(kTThreads), 0, stream, G, D, wd, daily, obs, inv_count, loss, grad);
  return hipGetLastError();
}

size_t clip_adam_work_bytes() { return sizeof(double) * kAdamWgs; }

hipError_t launch_clip_adam(int64_t n, float* param, const float* grad, float* m, float* v, float lr, float beta1,
                            float beta2, float eps, float* step, float max_norm, float* norm_out, void* work,
                            hipStream_t stream) {
  AdamArgs a{n, param, grad, m, v, lr, beta1, beta2, eps, step, max_norm, norm_out, static_cast<double*>(work)};
  hipLaunchKernelGGL(adam_norm_kernel, dim3(kAdamWgs), dim3(kAdamThreads), 0, stream, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(adam_step_kernel, dim3(kAdamWgs), dim3(kAdamThreads), 0, stream, a);
  return hipGetLastError();
}

}  // namespace ddr
