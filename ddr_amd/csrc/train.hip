// The tail of the C3 training step (bench.py --workload c3; the reference loop scripts/train.py:54-104) in two
// launches instead of ~15 PyTorch ones:
//   daily_l1_kernel   the objective, torch.nn.functional.l1_loss over gauges x days after the warm-up
//                     (train.py:91-94), and its gradient w.r.t. the daily series in the same pass;
//   clip_adam_kernel  torch.nn.utils.clip_grad_norm_(max_norm) (train.py:99) and the Adam update (train.py:100,
//                     torch.optim.Adam without weight decay / amsgrad) over one flat parameter vector.
// Both are one workgroup: the C3 objective is G x D = 256 x 89 values and the parameter network ~34k parameters,
// so a single CU finishes in a few microseconds and the reductions need no second launch (deterministic: every
// thread's slice and the LDS tree are fixed).
#include "internal.h"

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
  float bc1;        // 1 - beta1^step
  float bc2_sqrt;   // sqrt(1 - beta2^step)
  float max_norm;   // <= 0: no clipping
  float* norm_out;  // the gradient's total norm before clipping (clip_grad_norm_'s return value), or null
};

__global__ void __launch_bounds__(kTThreads) clip_adam_kernel(AdamArgs a) {
  __shared__ double red[kTThreads];
  // total 2-norm of the gradient (clip_grad_norm_ with one parameter tensor: its norm)
  double ss = 0.0;
  for (int64_t i = threadIdx.x; i < a.n; i += kTThreads) {
    const float g = a.grad[i];
    ss += (double)g * (double)g;
  }
  const float norm = (float)sqrt(block_sum(ss, red));
  if (threadIdx.x == 0 && a.norm_out) a.norm_out[0] = norm;
  // clip_coef = max_norm / (norm + 1e-6), clamped to <= 1 (torch/nn/utils/clip_grad.py)
  float coef = 1.0f;
  if (a.max_norm > 0.0f) coef = fminf(a.max_norm / (norm + 1e-6f), 1.0f);
  const float omb1 = 1.0f - a.beta1, omb2 = 1.0f - a.beta2;
  const float step = a.lr / a.bc1;
  for (int64_t i = threadIdx.x; i < a.n; i += kTThreads) {
    const float g = a.grad[i] * coef;
    const float m = fmaf(omb1, g - a.m[i], a.m[i]);           // exp_avg.lerp_(grad, 1 - beta1)
    const float v = fmaf(a.beta2, a.v[i], omb2 * g * g);      // exp_avg_sq * beta2 + (1 - beta2) g^2
    a.m[i] = m;
    a.v[i] = v;
    const float den = sqrtf(v) / a.bc2_sqrt + a.eps;
    a.param[i] = a.param[i] - step * (m / den);
  }
}

}  // namespace

hipError_t launch_daily_l1(int64_t G, int64_t D, int64_t wd, const float* daily, const float* obs, float inv_count,
                           float* loss, float* grad, hipStream_t stream) {
  hipLaunchKernelGGL(daily_l1_kernel, dim3(1), dim3(kTThreads), 0, stream, G, D, wd, daily, obs, inv_count, loss, grad);
  return hipGetLastError();
}

hipError_t launch_clip_adam(int64_t n, float* param, const float* grad, float* m, float* v, float lr, float beta1,
                            float beta2, float eps, float bc1, float bc2_sqrt, float max_norm, float* norm_out,
                            hipStream_t stream) {
  AdamArgs a{n, param, grad, m, v, lr, beta1, beta2, eps, bc1, bc2_sqrt, max_norm, norm_out};
  hipLaunchKernelGGL(clip_adam_kernel, dim3(1), dim3(kTThreads), 0, stream, a);
  return hipGetLastError();
}

}  // namespace ddr
