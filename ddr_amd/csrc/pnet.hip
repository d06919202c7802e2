// Fused parameter network of the C3 training step (bench.py --workload c3): the KAN stand-in
// attributes (N, F) -> Linear(F, 128) -> SiLU -> Linear(128, 128) -> SiLU -> Linear(128, 128) -> SiLU ->
// Linear(128, 3) -> sigmoid -> denormalize (utils.py:166-185) -> (n, q_spatial, p_spatial), forward and backward
// in two persistent launches on the fp32 matrix cores (v_mfma_f32_16x16x4_f32: exact f32 products, one
// rounding per product, at the f32 vector rate).  The reference's network is pykan's KAN (src/ddr/nn/kan.py:11-62;
// pykan is not installed here), whose output contract -- (N, 3) in [0, 1] through sigmoid, denormalised by
// the routing engine -- this network keeps.  It replaces the ~60 PyTorch launches (hipBLASLt GEMMs, SiLU and
// its backward, bias reductions, sigmoid, denormalize) of the same network per training step.
//
// Layout: one workgroup of 4 waves per CU, persistent over 64-row tiles.  Every GEMM is a 64 x 128 (or 128 x
// 128) tile product on 16x16x4 fragments; wave w owns output columns [32w, 32w + 32) (two 16-column blocks).
// The weight slices a wave multiplies by stay in its registers for the whole launch; activations move through
// LDS images with a 132-float row stride (conflict-free for the fragment reads).  The forward saves the
// pre-activations Z1..Z3 (3 x N x 128) and the sigmoid U (N x 3) for the backward; the backward accumulates
// its weight gradients in registers over its tiles and writes one partial per workgroup, summed in a fixed
// order by pnet_reduce_kernel (deterministic).
#include <atomic>

#include "internal.h"

namespace ddr {

namespace {

constexpr int kPH = 128;           // hidden width
constexpr int kPO = 3;             // outputs (n, q_spatial, p_spatial)
constexpr int kPF = 12;            // max input features (padded to 3 k-steps of 4)
constexpr int kPM = 64;            // rows per tile
constexpr int kPS = 132;           // LDS row stride (floats)
constexpr int kPThreads = 256;

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 mfma(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
// hardware reciprocal (1 ulp): the network is a stand-in whose only contract is the reference's output range
__device__ __forceinline__ float sigm(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float silu(float z) { return z * sigm(z); }
// d silu / dz = s (1 + z (1 - s))
__device__ __forceinline__ float dsilu(float z) {
  const float s = sigm(z);
  return s * (1.0f + z * (1.0f - s));
}

// Flat parameter layout (PnetLayout): W1 (128, F) | b1 | W2 (128, 128) | b2 | W3 | b3 | W4 (3, 128) | b4 (3)
struct PnetLayout {
  int F;
  __host__ __device__ int w1() const { return 0; }
  __host__ __device__ int b1() const { return kPH * F; }
  __host__ __device__ int w2() const { return b1() + kPH; }
  __host__ __device__ int b2() const { return w2() + kPH * kPH; }
  __host__ __device__ int w3() const { return b2() + kPH; }
  __host__ __device__ int b3() const { return w3() + kPH * kPH; }
  __host__ __device__ int w4() const { return b3() + kPH; }
  __host__ __device__ int b4() const { return w4() + kPO * kPH; }
  __host__ __device__ int total() const { return b4() + kPO; }
};

struct PnetArgs {
  int64_t N;
  int32_t F;
  int32_t ntiles;
  const float* X;       // (N, F)
  const float* P;       // flat parameters
  float scale[kPO];     // denormalize: y = U * scale + offset, exp(y) for a log-space output
  float offset[kPO];
  int32_t logsp[kPO];
  float* Z;             // (3, N, 128) pre-activations of the hidden layers
  float* U;             // (N, 3) sigmoid outputs
  float* out[kPO];      // (N) each: n, q_spatial, p_spatial
  const float* gout[kPO];  // backward: dL/d(n, q, p)
  float* partial;       // backward: [gridDim][total] weight-gradient partials
};

// The A fragment of rows [16 mb, 16 mb + 16) and k-step s of an LDS image (lane: row l & 15, k 4 s + l >> 4)
__device__ __forceinline__ float afrag(const float* img, int mb, int s, int lane) {
  return img[(16 * mb + (lane & 15)) * kPS + 4 * s + (lane >> 4)];
}

// img[r][c] = silu(Z[r0 + r][c]) for a 64 x 128 tile (zero past N), in two halves so that the loads (eight 16-B
// loads per thread) are issued early and land under other work: load_tile, then store_silu
__device__ __forceinline__ void load_tile(float4 (&v)[8], const float* Z, int64_t r0, int64_t N, int tid) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int e = tid + j * kPThreads;  // float4 index in the tile: row e / 32, columns 4 (e % 32) ..
    const int64_t row = r0 + (e >> 5);
    v[j] = row < N ? *reinterpret_cast<const float4*>(Z + row * kPH + 4 * (e & 31)) : make_float4(0, 0, 0, 0);
  }
}
__device__ __forceinline__ void store_silu(float* img, const float4 (&v)[8], int64_t r0, int64_t N, int tid) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int e = tid + j * kPThreads;
    const bool in = r0 + (e >> 5) < N;
    float* d = img + (e >> 5) * kPS + 4 * (e & 31);
    d[0] = in ? silu(v[j].x) : 0.0f;
    d[1] = in ? silu(v[j].y) : 0.0f;
    d[2] = in ? silu(v[j].z) : 0.0f;
    d[3] = in ? silu(v[j].w) : 0.0f;
  }
}

// Forward: one tile = 64 rows, eight waves; wave w owns output columns [16 w, 16 w + 16) (one 16-column block).
// acc[mb]: rows 16 mb + 4 (l >> 4) + i, column 16 w + (l & 15)
constexpr int kPFwdThreads = 512;
__global__ void __launch_bounds__(kPFwdThreads) pnet_forward_kernel(PnetArgs a) {
  __shared__ float H[kPM * kPS];
  __shared__ float Xs[kPM * 16];  // X tile, 16-float rows (zero-padded)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lq = lane & 15, lh = lane >> 4;
  const PnetLayout L{a.F};
  const float* P = a.P;
  const int F = a.F;
  // weight slices in registers: B[k][n] = W[n][k] for the wave's columns n = 16 w + lq
  const int n = 16 * w + lq;
  float w1r[kPF / 4], w2r[kPH / 4], w3r[kPH / 4], w4r[kPH / 4];
#pragma unroll
  for (int s = 0; s < kPF / 4; ++s) {
    const int k = 4 * s + lh;
    w1r[s] = k < F ? P[L.w1() + n * F + k] : 0.0f;
  }
#pragma unroll
  for (int s = 0; s < kPH / 4; ++s) {
    w2r[s] = P[L.w2() + n * kPH + 4 * s + lh];
    w3r[s] = P[L.w3() + n * kPH + 4 * s + lh];
  }
  const float bb1 = P[L.b1() + n], bb2 = P[L.b2() + n], bb3 = P[L.b3() + n];
  // the last layer: one 16-column block (columns 0..2 real), waves 0..3 take rows [16 w, 16 w + 16)
#pragma unroll
  for (int s = 0; s < kPH / 4; ++s) w4r[s] = (lq < kPO && w < 4) ? P[L.w4() + lq * kPH + 4 * s + lh] : 0.0f;
  const float bb4 = lq < kPO ? P[L.b4() + lq] : 0.0f;

  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    const int64_t r0 = (int64_t)tile * kPM;
    // X tile (zero-padded to 16 features, rows past N zero)
    for (int e = tid; e < kPM * 16; e += kPFwdThreads) {
      const int r = e >> 4, f = e & 15;
      const int64_t row = r0 + r;
      Xs[e] = (f < F && row < a.N) ? a.X[row * F + f] : 0.0f;
    }
    __syncthreads();
    f4 acc[4];
    auto init = [&](float bb) {
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) acc[mb] = f4{bb, bb, bb, bb};
    };
    // acc += H * W^T over the 32 k-steps of a 128-wide layer (weights: the wave's register slice)
    auto mm128 = [&](const float (&wr)[kPH / 4]) {
#pragma unroll
      for (int s = 0; s < kPH / 4; ++s) {
        float av[4];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) av[mb] = afrag(H, mb, s, lane);
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) acc[mb] = mfma(av[mb], wr[s], acc[mb]);
      }
    };
    // save Z (layer l), write silu(Z) into H -- after every wave has read H
    auto emit = [&](int layer) {
      __syncthreads();
      float* Zl = a.Z + (int64_t)layer * a.N * kPH;
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 16 * mb + 4 * lh + i;
          const float z = acc[mb][i];
          if (r0 + r < a.N) Zl[(r0 + r) * kPH + n] = z;
          H[r * kPS + n] = silu(z);
        }
      __syncthreads();
    };
    // layer 1 (K = F <= 12: three k-steps, zero-padded)
    init(bb1);
#pragma unroll
    for (int s = 0; s < kPF / 4; ++s)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) acc[mb] = mfma(Xs[(16 * mb + lq) * 16 + 4 * s + lh], w1r[s], acc[mb]);
    emit(0);
    init(bb2);
    mm128(w2r);
    emit(1);
    init(bb3);
    mm128(w3r);
    emit(2);
    // output layer: rows [16 w, 16 w + 16), columns 0..15 (0..2 real)
    if (w < 4) {
      f4 o = f4{bb4, bb4, bb4, bb4};
#pragma unroll
      for (int s = 0; s < kPH / 4; ++s) o = mfma(afrag(H, w, s, lane), w4r[s], o);
      if (lq < kPO) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t row = r0 + 16 * w + 4 * lh + i;
          if (row >= a.N) continue;
          const float u = sigm(o[i]);
          a.U[row * kPO + lq] = u;
          float y = u * a.scale[lq] + a.offset[lq];
          if (a.logsp[lq]) y = expf(y);
          a.out[lq][row] = y;
        }
      }
    }
    __syncthreads();  // H and Xs are rewritten by the next tile
  }
}

// Backward.  Per tile: dZ4 = dL/dU * U (1 - U) (dL/dU from the denormalize's VJP); dH3 = dZ4 W4; dZ3 = dH3 silu'(Z3);
// dW4 += dZ4^T H3; dW3 += dZ3^T H2; dH2 = dZ3 W3; dZ2 = dH2 silu'(Z2); dW2 += dZ2^T H1; dH1 = dZ2 W2;
// dZ1 = dH1 silu'(Z1); dW1 += dZ1^T X; the bias gradients are the column sums of dZ.
// The weight-gradient accumulators D[o][i] are fragments with o on the rows (wave w: o in [32 w, 32 w + 32)) and
// i on the columns (all 128: eight blocks).
constexpr size_t kPnetBwdLds = sizeof(float) * (3 * kPM * kPS + 2 * kPM * 16);
__global__ void __launch_bounds__(kPThreads) pnet_backward_kernel(PnetArgs a) {
  extern __shared__ __attribute__((aligned(16))) float psm[];
  float* HA = psm;                  // H3, then H1
  float* HB = HA + kPM * kPS;       // H2
  float* G = HB + kPM * kPS;        // dZ3, then dZ2, then dZ1
  float* D4 = G + kPM * kPS;        // dZ4 (64 x 16, columns 3..15 zero)
  float* Xs = D4 + kPM * 16;        // X tile (64 x 16, zero-padded)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lq = lane & 15, lh = lane >> 4;
  const PnetLayout L{a.F};
  const float* P = a.P;
  const int F = a.F;
  // B[k = o][n = i] = W[o][i] for the data gradients dH = dZ W (wave columns i = 32 w + 16 nb + lq): W4's in
  // registers; W2's and W3's fragments are read from the L2-resident weights inside the product (the registers
  // hold the weight-gradient accumulators instead)
  float w4t[2];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) w4t[nb] = lh < kPO ? P[L.w4() + lh * kPH + 32 * w + 16 * nb + lq] : 0.0f;
  f4 gw3[2][8], gw2[2][8], gw1[2], gw4[2];
#pragma unroll
  for (int ob = 0; ob < 2; ++ob) {
#pragma unroll
    for (int ib = 0; ib < 8; ++ib) gw3[ob][ib] = gw2[ob][ib] = f4{0, 0, 0, 0};
    gw1[ob] = gw4[ob] = f4{0, 0, 0, 0};
  }
  float gb1[2] = {0, 0}, gb2[2] = {0, 0}, gb3[2] = {0, 0}, gb4 = 0.0f;
  const int64_t NH = a.N * kPH;

  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    const int64_t r0 = (int64_t)tile * kPM;
    // the thread's values of an (N, 128) array in fragment layout: rows 16 mb + 4 lh + i, columns 32 w + 16 nb + lq
    auto load_frag = [&](float (&z)[32], const float* Zl) {
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = 16 * mb + 4 * lh + i, c = 32 * w + 16 * nb + lq;
            z[(mb * 2 + nb) * 4 + i] = r0 + r < a.N ? Zl[(r0 + r) * kPH + c] : 0.0f;
          }
    };
    // every global load of the tile's first phase in one round trip: dL/dU inputs and X (four entries of the
    // 64 x 16 images per thread), the Z2 tile (for H2) and the thread's Z3 values in fragment layout
    float uin[4], gin[4], xin[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = tid + j * kPThreads, r = e >> 4, c = e & 15;
      const int64_t row = r0 + r;
      const bool ok = c < kPO && row < a.N;
      uin[j] = ok ? a.U[row * kPO + c] : 0.0f;
      gin[j] = ok ? a.gout[c < kPO ? c : 0][row] : 0.0f;
      xin[j] = (c < F && row < a.N) ? a.X[row * F + c] : 0.0f;
    }
    float4 zt[8];
    load_tile(zt, a.Z + NH, r0, a.N, tid);
    float zd[32];
    load_frag(zd, a.Z + 2 * NH);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = tid + j * kPThreads, c = e & 15;
      float d = 0.0f;
      if (c < kPO) {
        // denormalize VJP: y = U scale + offset (log space: y = exp(...), dy/dU = y scale); sigmoid' = U (1 - U)
        const float u = uin[j];
        float dy = a.scale[c];
        if (a.logsp[c]) dy = expf(u * a.scale[c] + a.offset[c]) * a.scale[c];
        d = gin[j] * dy * (u * (1.0f - u));
      }
      D4[e] = d;
      Xs[e] = xin[j];
    }
    store_silu(HB, zt, r0, a.N, tid);  // H2 = silu(Z2)
    __syncthreads();
    // dH3 = dZ4 W4 (one k-step: k = output j), rows all 64, wave columns; dZ3 = dH3 silu'(Z3); H3 = silu(Z3)
    f4 acc[4][2];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      const float av = D4[(16 * mb + lq) * 16 + lh];
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = mfma(av, w4t[nb], f4{0, 0, 0, 0});
    }
    if (lq < kPO) {
      for (int r = 16 * w + lh; r < 16 * w + 16; r += 4) gb4 += D4[r * 16 + lq];  // the wave's 16 rows
    }
    // dZ = dH silu'(Z) from the thread's fragment-layout Z values; bias partials; optionally H = silu(Z)
    auto to_dz = [&](const float (&z)[32], float (&gb)[2], float* himg) {
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = 16 * mb + 4 * lh + i, c = 32 * w + 16 * nb + lq;
            const bool in = r0 + r < a.N;
            const float zz = z[(mb * 2 + nb) * 4 + i];
            const float dz = in ? acc[mb][nb][i] * dsilu(zz) : 0.0f;
            G[r * kPS + c] = dz;
            gb[nb] += dz;
            if (himg) himg[r * kPS + c] = in ? silu(zz) : 0.0f;
          }
    };
    to_dz(zd, gb3, HA);
    __syncthreads();
    // dW4 += dZ4^T H3: A[m = j][k = r] = D4[r][j], B[k = r][n = i] = H3[r][i]
#pragma unroll 4
    for (int s = 0; s < kPM / 4; ++s) {
      const float av = D4[(4 * s + lh) * 16 + lq];
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) gw4[nb] = mfma(av, HA[(4 * s + lh) * kPS + 32 * w + 16 * nb + lq], gw4[nb]);
    }
    // dW_l += dZ^T H_{l-1}: A[m = o][k = r] = G[r][o] (wave rows o = 32 w + 16 ob + lq), B[k = r][n = i] = H[r][i]
    auto wgrad = [&](f4 (&gw)[2][8], const float* himg) {
      // (s indexes LDS only: a partial unroll keeps the fragments of two k-steps in flight, not sixteen)
#pragma unroll 2
      for (int s = 0; s < kPM / 4; ++s) {
        const int r = 4 * s + lh;
        float av[2], bv[8];
#pragma unroll
        for (int ob = 0; ob < 2; ++ob) av[ob] = G[r * kPS + 32 * w + 16 * ob + lq];
#pragma unroll
        for (int ib = 0; ib < 8; ++ib) bv[ib] = himg[r * kPS + 16 * ib + lq];
#pragma unroll
        for (int ob = 0; ob < 2; ++ob)
#pragma unroll
          for (int ib = 0; ib < 8; ++ib) gw[ob][ib] = mfma(av[ob], bv[ib], gw[ob][ib]);
      }
    };
    // dH = dZ W: A[m = r][k = o] = G[r][o], B = the wave's transposed weight slice
    auto dgrad = [&](const float* W) {
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = f4{0, 0, 0, 0};
      const float* wc = W + lh * kPH + 32 * w + lq;
#pragma unroll 4
      for (int s = 0; s < kPH / 4; ++s) {
        float av[4];
        const float b0 = wc[4 * s * kPH], b1 = wc[4 * s * kPH + 16];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) av[mb] = afrag(G, mb, s, lane);
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
          acc[mb][0] = mfma(av[mb], b0, acc[mb][0]);
          acc[mb][1] = mfma(av[mb], b1, acc[mb][1]);
        }
      }
    };
    // the second phase's loads (Z2 and Z1 in fragment layout, the Z1 tile), in flight under the dW3 / dH2 products
    float zd2[32], zd1[32];
    load_frag(zd2, a.Z + NH);
    load_frag(zd1, a.Z);
    load_tile(zt, a.Z, r0, a.N, tid);
    wgrad(gw3, HB);
    dgrad(P + L.w3());
    __syncthreads();  // G (dZ3) and HA (H3) are rewritten below
    to_dz(zd2, gb2, nullptr);
    store_silu(HA, zt, r0, a.N, tid);  // H1 = silu(Z1)
    __syncthreads();
    wgrad(gw2, HA);
    dgrad(P + L.w2());
    __syncthreads();
    to_dz(zd1, gb1, nullptr);
    __syncthreads();
    // dW1 += dZ1^T X: A[m = o][k = r] = G[r][o], B[k = r][n = f] = X[r][f]
#pragma unroll 4
    for (int s = 0; s < kPM / 4; ++s) {
      const int r = 4 * s + lh;
      const float bv = Xs[r * 16 + lq];
#pragma unroll
      for (int ob = 0; ob < 2; ++ob) gw1[ob] = mfma(G[r * kPS + 32 * w + 16 * ob + lq], bv, gw1[ob]);
    }
    __syncthreads();  // every buffer is rewritten by the next tile
  }

  // this workgroup's partial gradient, in the flat parameter layout
  float* out = a.partial + (int64_t)blockIdx.x * L.total();
  // fragment D[m][n] of block (mb, nb): row 16 mb + 4 lh + i, column 16 nb + lq
#pragma unroll
  for (int ob = 0; ob < 2; ++ob)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int o = 32 * w + 16 * ob + 4 * lh + i;
#pragma unroll
      for (int ib = 0; ib < 8; ++ib) {
        const int c = 16 * ib + lq;
        out[L.w3() + o * kPH + c] = gw3[ob][ib][i];
        out[L.w2() + o * kPH + c] = gw2[ob][ib][i];
      }
      if (lq < F) out[L.w1() + o * F + lq] = gw1[ob][i];
    }
  // dW4[j][i]: block rows j (4 lh + i' < 3), columns i = 32 w + 16 nb + lq
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = 4 * lh + i;
      if (j < kPO) out[L.w4() + j * kPH + 32 * w + 16 * nb + lq] = gw4[nb][i];
    }
  // bias partials: lanes sharing a column (the four lh groups) combine through LDS
  __syncthreads();
  float* red = G;  // [4 lh][128 columns] x 3 layers, then b4
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    const int c = 32 * w + 16 * nb + lq;
    red[(0 * 4 + lh) * kPH + c] = gb1[nb];
    red[(1 * 4 + lh) * kPH + c] = gb2[nb];
    red[(2 * 4 + lh) * kPH + c] = gb3[nb];
  }
  if (lq < kPO) red[12 * kPH + w * 64 + lh * 16 + lq] = gb4;
  __syncthreads();
  if (tid < kPH) {
    const int c = tid;
    for (int l = 0; l < 3; ++l) {
      float v = 0.0f;
      for (int g = 0; g < 4; ++g) v += red[(l * 4 + g) * kPH + c];
      out[(l == 0 ? L.b1() : (l == 1 ? L.b2() : L.b3())) + c] = v;
    }
  }
  if (tid < kPO) {
    float v = 0.0f;
    for (int q = 0; q < 16; ++q) v += red[12 * kPH + q * 16 + tid];
    out[L.b4() + tid] = v;
  }
}

// grad[p] = sum over workgroups (ascending) of partial[wg][p]: a fixed order, so the result is deterministic
__global__ void pnet_reduce_kernel(const float* partial, int nwg, int total, float* grad) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= total) return;
  float v = 0.0f;
  int g = 0;
  for (; g + 16 <= nwg; g += 16) {  // sixteen loads in flight, summed in ascending order
    float t[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) t[j] = partial[(int64_t)(g + j) * total + p];
#pragma unroll
    for (int j = 0; j < 16; ++j) v += t[j];
  }
  for (; g < nwg; ++g) v += partial[(int64_t)g * total + p];
  grad[p] = v;
}

// CUs of the current device, queried once per device (three calls per training step: no device-properties
// query on the host's critical path)
int device_cus() {
  constexpr int kDevs = 64;
  static std::atomic<int> cache[kDevs] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kDevs) return 256;
  int cus = cache[dev].load(std::memory_order_relaxed);
  if (cus == 0) {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    cache[dev].store(cus, std::memory_order_relaxed);
  }
  return cus;
}
int pnet_grid(int64_t ntiles) { return (int)std::max<int64_t>(1, std::min<int64_t>(ntiles, device_cus())); }

}  // namespace

int pnet_param_count(int F) { return PnetLayout{F}.total(); }

int64_t pnet_work_bytes(int64_t N, int F) {
  const int64_t ntiles = (N + kPM - 1) / kPM;
  return (int64_t)pnet_grid(ntiles) * PnetLayout{F}.total() * (int64_t)sizeof(float);
}

hipError_t launch_pnet_forward(int64_t N, int F, const float* X, const float* P, const float* denorm, float* Z, float* U,
                               float* const out[3], hipStream_t stream) {
  PnetArgs a{};
  a.N = N;
  a.F = F;
  a.ntiles = (int)((N + kPM - 1) / kPM);
  a.X = X;
  a.P = P;
  for (int j = 0; j < kPO; ++j) {
    a.scale[j] = denorm[3 * j];
    a.offset[j] = denorm[3 * j + 1];
    a.logsp[j] = denorm[3 * j + 2] != 0.0f;
    a.out[j] = out[j];
  }
  a.Z = Z;
  a.U = U;
  if (a.ntiles == 0) return hipSuccess;
  const int64_t wgs = std::min<int64_t>(a.ntiles, 2 * (int64_t)pnet_grid(a.ntiles));
  hipLaunchKernelGGL(pnet_forward_kernel, dim3((unsigned)wgs), dim3(kPFwdThreads), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_pnet_backward(int64_t N, int F, const float* X, const float* P, const float* denorm, const float* Z,
                                const float* U, const float* const gout[3], float* grad, void* work, hipStream_t stream) {
  PnetArgs a{};
  a.N = N;
  a.F = F;
  a.ntiles = (int)((N + kPM - 1) / kPM);
  a.X = X;
  a.P = P;
  for (int j = 0; j < kPO; ++j) {
    a.scale[j] = denorm[3 * j];
    a.offset[j] = denorm[3 * j + 1];
    a.logsp[j] = denorm[3 * j + 2] != 0.0f;
    a.gout[j] = gout[j];
  }
  a.Z = const_cast<float*>(Z);
  a.U = const_cast<float*>(U);
  a.partial = static_cast<float*>(work);
  const int total = PnetLayout{F}.total();
  if (a.ntiles == 0) return hipMemsetAsync(grad, 0, sizeof(float) * total, stream);
  const int nwg = pnet_grid(a.ntiles);
  hipError_t e = hipFuncSetAttribute((const void*)pnet_backward_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)kPnetBwdLds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(pnet_backward_kernel, dim3(nwg), dim3(kPThreads), kPnetBwdLds, stream, a);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(pnet_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, a.partial, nwg, total, grad);
  return hipGetLastError();
}

}  // namespace ddr
