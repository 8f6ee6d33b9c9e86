// fp32 GEMM for the precision='highest' lm_head (reference model.py:698-736: only the lm_head honours
// `precision`, jax_test.py:433 runs the parity harness with precision='highest').
//
// y[M, N] = x[M, K] @ W[N, K]^T with fp32 inputs, fp32 accumulation and fp32 output on the exact-f32 MFMA
// (v_mfma_f32_32x32x2_f32: a k-ordered fmaf chain, no xf32 shortcut on gfx950). Opt-in path (the default
// lm_head is the bf16 GEMV/GEMM), so the design is simple and robust rather than tuned: 128 x 128 output tile per
// 256-thread workgroup, four waves of 64 x 64 (2 x 2 MFMA tiles), K staged 32 deep through LDS in k-major images
// ([k][row]) so a lane's fragment element (row l & 31, k l >> 5) is one conflict-free ds_read_b32.
#include "common.h"
#include "launchers.h"

namespace jla {

constexpr int GF_BM = 128, GF_BN = 128, GF_BK = 32, GF_THREADS = 256;

using f32x16 = __attribute__((ext_vector_type(16))) float;

__global__ void __launch_bounds__(GF_THREADS)
    gemm_f32_kernel(const float* __restrict__ x, const float* __restrict__ w, float* __restrict__ y, int M, int N,
                    int K) {
  __shared__ float As[GF_BK][GF_BM];
  __shared__ float Bs[GF_BK][GF_BN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * GF_BM, n0 = blockIdx.x * GF_BN;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  for (int k0 = 0; k0 < K; k0 += GF_BK) {
    // stage: 128 rows x 32 k of x and of W, one float4 (4 consecutive k) per thread and step
#pragma unroll
    for (int it = 0; it < (GF_BM * GF_BK / 4) / GF_THREADS; ++it) {
      const int e = it * GF_THREADS + tid;  // float4 index in the tile
      const int row = e / (GF_BK / 4), kq = (e % (GF_BK / 4)) * 4;
      const int gk = k0 + kq;
      float av[4] = {0.f, 0.f, 0.f, 0.f}, bv[4] = {0.f, 0.f, 0.f, 0.f};
      const int gm = m0 + row, gn = n0 + row;
      if (gm < M) {
        if (gk + 3 < K && (K & 3) == 0) {
          const float4 v = *reinterpret_cast<const float4*>(x + (size_t)gm * K + gk);
          av[0] = v.x; av[1] = v.y; av[2] = v.z; av[3] = v.w;
        } else {
          for (int q = 0; q < 4; ++q) av[q] = gk + q < K ? x[(size_t)gm * K + gk + q] : 0.f;
        }
      }
      if (gn < N) {
        if (gk + 3 < K && (K & 3) == 0) {
          const float4 v = *reinterpret_cast<const float4*>(w + (size_t)gn * K + gk);
          bv[0] = v.x; bv[1] = v.y; bv[2] = v.z; bv[3] = v.w;
        } else {
          for (int q = 0; q < 4; ++q) bv[q] = gk + q < K ? w[(size_t)gn * K + gk + q] : 0.f;
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        As[kq + q][row] = av[q];
        Bs[kq + q][row] = bv[q];
      }
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < GF_BK / 2; ++kk) {
      const int kr = 2 * kk + (lane >> 5);
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[kr][wm * 64 + i * 32 + (lane & 31)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[kr][wn * 64 + j * 32 + (lane & 31)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // C/D map of the 32x32 shapes: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 64 + j * 32 + (lane & 31);
      if (col >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row < M) y[(size_t)row * N + col] = acc[i][j][r];
      }
    }
}

int gemm_f32(const float* x, const float* w, float* y, int M, int N, int K, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return M < 0 || N < 0 || K < 0 ? -1 : 0;
  dim3 grid((N + GF_BN - 1) / GF_BN, (M + GF_BM - 1) / GF_BM);
  if (grid.y > 65535) return -2;
  gemm_f32_kernel<<<grid, GF_THREADS, 0, s>>>(x, w, y, M, N, K);
  JLA_CHECK_LAUNCH();
  return 0;
}

}  // namespace jla
