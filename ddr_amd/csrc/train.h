// Launchers of the C3 training step's tail (train.hip), called by the C ABI (capi.cpp: ddr_daily_l1_f32,
// ddr_clip_adam_f32).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace ddr {
hipError_t launch_daily_l1(int64_t G, int64_t D, int64_t wd, const float* daily, const float* obs, float inv_count,
                           float* loss, float* grad, hipStream_t stream);
// device scratch of launch_clip_adam (per-workgroup partial sums of squares)
size_t clip_adam_work_bytes();
hipError_t launch_clip_adam(int64_t n, float* param, const float* grad, float* m, float* v, float lr, float beta1,
                            float beta2, float eps, float* step, float max_norm, float* norm_out, void* work,
                            hipStream_t stream);
}  // namespace ddr
