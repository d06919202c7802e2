// Dependent-chain latency of one reach-step, the floor of a light-load tick.
// One workgroup of W waves; every lane runs K steps whose input depends on the previous step's
// output, as a reach's step t + 1 depends on its step t:
//   mode 0 fwd-exact      coefficients_np<float, 1> (correctly rounded pow), fp64 solve row, clamp
//   mode 1 fwd-fast       coefficients_fast
//   mode 2 fwd-faithful   coefficients_faithful (the default forward)
//   mode 3 bwd            adjoint_step_fast with Q independent of the chain (the saved state), gb on it
//   mode 4 sync only      a multiply-add, no physics
// With lds = 1 each step also publishes its value to an LDS slot, passes a workgroup barrier and reads
// a neighbour's slot (the tick's hand-off); lds = 0 keeps the chain in registers.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
//     tools/chain_lat.hip -o build/chain_lat && ./build/chain_lat
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

#include "../ddr_amd/csrc/physics.h"

using namespace ddr;

template <int MODE, bool LDS>
__global__ void __launch_bounds__(1024) chain(int K, float* out, unsigned long long* clk) {
  __shared__ double sx[2][1024];
  load_math_tables();
  __syncthreads();
  const int tid = threadIdx.x, nt = blockDim.x;
  const Consts<float> cs{3600.0f, 1e-4f, 0.01f, 15.0f, 0.01f, 0.01f, 0.5f, 50.0f, pow_consts_vgpr(), std::log(0.01)};
  const ReachStatic<float> st = make_static<float>(0.04f + 1e-5f * tid, 0.5f, 21.0f, 1e-3f, 3000.0f, 0.3f);
  float Q = 1.0f + 1e-3f * (tid & 63), In = 0.5f, qc = 0.2f, gb = 1.0f;
  double xu = 0.3;
  unsigned long long t0 = 0, c0 = 0;
  if (tid == 0) {
    t0 = wall_clock64();
    c0 = clock64();
  }
#pragma unroll 1
  for (int k = 0; k < K; ++k) {
    double x;
    if constexpr (MODE == 3) {
      const float Qk = Q + 1e-7f * (float)k;  // the saved state: off the chain
      const AdjOut o = adjoint_step_fast<false>(st, Qk, cs, gb, 0.9f * Qk, (float)xu, In);
      x = (double)(0.5f + o.gQ * 0.25f + o.gn * 1e-3f + o.gq * 1e-3f + o.gp * 1e-3f) + (double)o.c1 * xu;
    } else if constexpr (MODE == 4) {
      x = 0.999 * xu + (double)Q;
    } else {
      PhysOut<float> ph;
      if constexpr (MODE == 1) {
        ph = coefficients_fast(st, Q, cs);
      } else if constexpr (MODE == 2) {
        ph = coefficients_faithful(st, Q, cs);
      } else {
        ReachStatic<float> sa[1] = {st};
        float qa[1] = {Q};
        PhysOut<float> pa[1];
        coefficients_np<float, 1>(sa, qa, cs, pa);
        ph = pa[0];
      }
      const float b = ((ph.c2 * In) + (ph.c3 * Q)) + (ph.c4 * qc);
      x = (double)b + (double)ph.c1 * xu;
    }
    if constexpr (LDS) {
      sx[k & 1][tid] = x;
      __syncthreads();
      xu = sx[k & 1][(tid + 1) % nt];
    } else {
      xu = x;
    }
    if constexpr (MODE == 3) gb = (float)xu;
    else {
      Q = rmax_nan((float)x, cs.qlb);
      In = (float)xu;
    }
  }
  if (tid == 0) {
    clk[0] = wall_clock64() - t0;
    clk[1] = clock64() - c0;
  }
  out[blockIdx.x * nt + tid] = (float)xu + Q + gb;
}

template <int MODE, bool LDS>
void run(const char* name, int K, int W, float* out, unsigned long long* clk) {
  hipLaunchKernelGGL((chain<MODE, LDS>), dim3(1), dim3(64 * W), 0, 0, K, out, clk);
  hipLaunchKernelGGL((chain<MODE, LDS>), dim3(1), dim3(64 * W), 0, 0, K, out, clk);  // (timed: warm)
  unsigned long long h[2];
  hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
  int mhz = 100;
  hipDeviceGetAttribute(&mhz, hipDeviceAttributeWallClockRate, 0);  // kHz
  const double ns = (double)h[0] * 1e6 / (double)mhz / K;
  printf("%-14s lds=%d waves=%2d  %8.1f ns/step  %8.1f shader-clock/step\n", name, (int)LDS, W, ns, (double)h[1] / K);
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 20000;
  float* out;
  unsigned long long* clk;
  hipMalloc(&out, 1024 * sizeof(float));
  hipMalloc(&clk, 2 * sizeof(unsigned long long));
  for (int W : {1, 4, 8, 16}) {
    run<0, false>("fwd-exact", K, W, out, clk);
    run<1, false>("fwd-fast", K, W, out, clk);
    run<2, false>("fwd-faithful", K, W, out, clk);
    run<3, false>("bwd", K, W, out, clk);
    run<4, false>("sync-only", K, W, out, clk);
    run<0, true>("fwd-exact", K, W, out, clk);
    run<1, true>("fwd-fast", K, W, out, clk);
    run<2, true>("fwd-faithful", K, W, out, clk);
    run<3, true>("bwd", K, W, out, clk);
    run<4, true>("sync-only", K, W, out, clk);
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
