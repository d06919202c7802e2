// ULP error of the fp32 pows of ddr_amd/csrc/fastmath.h against the correctly rounded value
// ((float)pow((double)x, (double)y)) over the operand ranges of the routing physics:
//   x log-uniform in [1e-7, 1.6e5]; y = 2/3 (a quarter of samples), else uniform in [0, 1]
// (expo = 3 / (5 + 3 qe) in [0.375, 0.6], qe in [1e-6, 1 + 1e-6]).
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/pow_check.hip -o build/pow_check && ./build/pow_check [n]
// Prints, per implementation, the histogram of |ulp error| (0, 1, 2, 3, >3) and the max.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../ddr_amd/csrc/fastmath.h"

using namespace ddr;

__device__ __forceinline__ unsigned long long mix(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ double unif(unsigned long long h) { return (h >> 11) * 0x1.0p-53; }

constexpr int kImpl = 3;  // pow_faithful, exp2(y log2 x) hardware, pow_pos (fp64 tables)
struct Hist {
  unsigned long long bins[kImpl][5];
  unsigned long long maxulp[kImpl];
};

__global__ void check(unsigned long long n, unsigned long long seed, Hist* out) {
  load_math_tables();
  __syncthreads();
  unsigned long long b[kImpl][5] = {};
  unsigned long long mx[kImpl] = {};
  for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
       i += (unsigned long long)gridDim.x * blockDim.x) {
    const unsigned long long h1 = mix(seed ^ (2 * i)), h2 = mix(seed ^ (2 * i + 1));
    const float x = (float)exp(-16.0 + 28.0 * unif(h1));
    const float y = (i & 3) == 0 ? (float)(2.0 / 3.0) : (float)unif(h2);
    const float ref = (float)pow((double)x, (double)y);
    float v[kImpl];
    v[0] = pow_faithful(x, y);
    v[1] = __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
    v[2] = pow_pos(x, y);
#pragma unroll
    for (int k = 0; k < kImpl; ++k) {
      long long d = (long long)__float_as_int(v[k]) - (long long)__float_as_int(ref);
      if (d < 0) d = -d;
      b[k][d > 3 ? 4 : d]++;
      if ((unsigned long long)d > mx[k]) mx[k] = (unsigned long long)d;
    }
  }
  for (int k = 0; k < kImpl; ++k) {
    for (int j = 0; j < 5; ++j) atomicAdd(&out->bins[k][j], b[k][j]);
    atomicMax(&out->maxulp[k], mx[k]);
  }
}

int main(int argc, char** argv) {
  const unsigned long long n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 400000000ull;
  Hist* d;
  if (hipMalloc(&d, sizeof(Hist)) != hipSuccess) return 2;
  (void)hipMemset(d, 0, sizeof(Hist));
  hipLaunchKernelGGL(check, dim3(4096), dim3(256), (2 * kLnTabN + kExpTabN) * sizeof(double), 0, n, 777ull, d);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  Hist h;
  (void)hipMemcpy(&h, d, sizeof(Hist), hipMemcpyDeviceToHost);
  const char* names[kImpl] = {"pow_faithful (fp32, split exponent)", "exp2(y*log2 x) hardware (fast math)",
                              "pow_pos (fp64 tables, exact mode)"};
  printf("samples %llu; |ulp error| vs the correctly rounded x^y\n", n);
  for (int k = 0; k < kImpl; ++k)
    printf("%-40s 0:%.6f 1:%.6f 2:%.6f 3:%.6f >3:%.6f  max %llu\n", names[k], h.bins[k][0] / (double)n,
           h.bins[k][1] / (double)n, h.bins[k][2] / (double)n, h.bins[k][3] / (double)n, h.bins[k][4] / (double)n,
           h.maxulp[k]);
  return 0;
}
