// Lane mapping of the DPP / swizzle / permlane exchanges geometry.hip relies on (gfx950): prints, per
// pattern, whether lane l receives lane f(l) for the intended f.
//   hipcc -O3 --offload-arch=gfx950 tools/dpp_check.hip -o build/dpp_check && ./build/dpp_check
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k(int* out) {
  const int l = threadIdx.x;
  out[0 * 64 + l] = __builtin_amdgcn_mov_dpp(l, 0x134, 0xF, 0xF, true);  // wave_rol:1, want (l + 1) & 63
  out[1 * 64 + l] = __builtin_amdgcn_mov_dpp(l, 0xB1, 0xF, 0xF, true);   // want l ^ 1
  out[2 * 64 + l] = __builtin_amdgcn_mov_dpp(l, 0x4E, 0xF, 0xF, true);   // want l ^ 2
  out[3 * 64 + l] = __builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp(l, 0x141, 0xF, 0xF, true), 0x1B, 0xF, 0xF, true);  // l ^ 4
  out[4 * 64 + l] = __builtin_amdgcn_mov_dpp(l, 0x128, 0xF, 0xF, true);  // want l ^ 8
  out[5 * 64 + l] = __builtin_amdgcn_ds_swizzle(l, 0x401F);             // want l ^ 16
  const auto pr = __builtin_amdgcn_permlane32_swap(l, l, false, false);
  out[6 * 64 + l] = (l & 32) ? pr[0] : pr[1];                          // want l ^ 32
}

int main() {
  int* d;
  int h[7 * 64];
  hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* name[7] = {"rol1", "xor1", "xor2", "xor4", "xor8", "xor16", "xor32"};
  int bad = 0;
  for (int p = 0; p < 7; ++p) {
    int ok = 0;
    for (int l = 0; l < 64; ++l) {
      const int want = p == 0 ? ((l + 1) & 63) : (l ^ (1 << (p - 1)));
      ok += h[p * 64 + l] == want;
    }
    printf("%-6s %2d/64 lanes as intended (lane 0 <- %d, lane 63 <- %d)\n", name[p], ok, h[p * 64], h[p * 64 + 63]);
    bad += ok != 64;
  }
  return bad;
}
