// Exhaustive check of fastmath.h sqrt_rn_normal against the library's correctly rounded sqrtf over every
// fp32 value in [2^-96, FLT_MAX] (~1.9e9 values).
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
//         tools/sqrt_check.hip -o build/sqrt_check && ./build/sqrt_check
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../ddr_amd/csrc/fastmath.h"

__global__ void check(unsigned lo, unsigned hi, unsigned long long* bad, unsigned* first) {
  unsigned long long nb = 0;
  for (unsigned long long u = lo + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; u < hi;
       u += (unsigned long long)gridDim.x * blockDim.x) {
    const float x = __uint_as_float((unsigned)u);
    const float a = ddr::sqrt_rn_normal(x), b = sqrtf(x);
    if (__float_as_uint(a) != __float_as_uint(b)) {
      ++nb;
      atomicMin(first, (unsigned)u);
    }
  }
  if (nb) atomicAdd(bad, nb);
}

int main() {
  unsigned long long* bad;
  unsigned* first;
  hipMalloc(&bad, 8);
  hipMalloc(&first, 4);
  hipMemset(bad, 0, 8);
  hipMemset(first, 0xFF, 4);
  const unsigned lo = 0x0F800000u;  // 2^-96
  const unsigned hi = 0x7F800000u;  // +inf (exclusive)
  hipLaunchKernelGGL(check, dim3(4096), dim3(256), 0, 0, lo, hi, bad, first);
  unsigned long long h = 0;
  unsigned f = 0;
  hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
  hipMemcpy(&f, first, 4, hipMemcpyDeviceToHost);
  printf("sqrt_rn_normal vs sqrtf over [2^-96, FLT_MAX]: %llu of %u values differ%s", h, hi - lo, h ? "" : "\n");
  if (h) printf(" (first 0x%08x = %g)\n", f, (double)__builtin_bit_cast(float, f));
  return h ? 1 : 0;
}
