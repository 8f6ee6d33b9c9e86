// Prefill linear layer (M > 64 rows): y[M, N] = epilogue( x[M, K] @ W[N, K]^T ), bf16 MFMA.
//
// Same epilogues as the skinny decode kernel (gemv.hip): store bf16/fp32, accumulate into the fp32
// residual stream, or SiLU(gate)*up over the interleaved [w1;w3] weight. The RMSNorm scale is
// applied to x beforehand (rms_scale), so x arrives as bf16.
//
// Tiling (CDNA4): 128 x 128 output tile per 256-thread workgroup, 4 waves in 2 x 2, each wave a
// 64 x 64 sub-tile = 4 x 4 v_mfma_f32_16x16x32_bf16 accumulators. K advances 64 per stage. Both
// operands are staged into LDS in the MFMA *fragment* layout (16 rows x 32 k = 64 lanes x 16 B),
// so every LDS fragment read is a lane-linear ds_read_b128 (bank-conflict free) and the packed
// weights are copied verbatim (each 1 KiB fragment is already contiguous in HBM). Double-buffered
// LDS; the next stage's global loads are issued before the current stage's MFMAs and written to
// LDS after them (issue-early / write-late), one barrier per stage.
#include "common.h"
#include "launchers.h"

namespace jla {

constexpr int GB_M = 128, GB_N = 128;
constexpr int G_THREADS = 256;
// fragments per stage: A 8 m-tiles x 2 k-steps, B 8 n-tiles x 2 k-steps (1 KiB each)
constexpr int G_AFR = 16, G_BFR = 16;
constexpr int G_STAGE_U4 = (G_AFR + G_BFR) * 64;  // u32x4 per stage (32 KiB); 8 per thread

template <int MODE>
__global__ void __launch_bounds__(G_THREADS)
    gemm_kernel(const bf16_t* __restrict__ x, const u32x4* __restrict__ W, void* __restrict__ out, int M, int N,
                int K, int accumulate, int out_f32, bf16_t* __restrict__ mirror) {
  __shared__ u32x4 lds[2][G_STAGE_U4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;
  const int n0 = blockIdx.x * GB_N, m0 = blockIdx.y * GB_M;
  const int KS = K >> 5, NTT = N >> 4;
  const int KT = (KS + 1) >> 1;  // stages of 2 k-steps (last may be half)

  // per-thread staging slots: fragment f = tid/64 + 4*j (j = 0..7), lane = tid & 63
  // f in [0,16): A fragment (mt = f>>1, ks = f&1); f in [16,32): B fragment (nt = (f-16)>>1, ks = f&1)
  const bf16_t* asrc[4];
  const u32x4* bsrc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int f = w + 4 * j;  // 0..15 -> A
    const int mt = f >> 1, ks = f & 1;
    const int row = min(m0 + mt * 16 + (lane & 15), M - 1);
    asrc[j] = x + (size_t)row * K + ks * 32 + 8 * (lane >> 4);
    const int fb = f;  // B fragment index 0..15
    const int nt = min((n0 >> 4) + (fb >> 1), NTT - 1), ksb = fb & 1;
    bsrc[j] = W + ((size_t)nt * KS + ksb) * 64 + lane;
  }

  u32x4 stage[8];
  auto gload = [&](int kt) {
    const int kbase = kt * 2;
    if ((kbase + 1) < KS) {  // uniform branch: only the last stage of an odd-KS GEMM is half
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        stage[j] = *reinterpret_cast<const u32x4*>(asrc[j] + (size_t)kbase * 32);
        stage[4 + j] = bsrc[j][(size_t)kbase * 64];
      }
    } else {
      // this thread's fragments all have ks == (w & 1); ks == 1 is past the end -> zeros
      const bool ok = (w & 1) == 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        stage[j] = u32x4{0, 0, 0, 0};
        stage[4 + j] = u32x4{0, 0, 0, 0};
      }
      if (ok) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          stage[j] = *reinterpret_cast<const u32x4*>(asrc[j] + (size_t)kbase * 32);
          stage[4 + j] = bsrc[j][(size_t)kbase * 64];
        }
      }
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      lds[buf][(w + 4 * j) * 64 + lane] = stage[j];
      lds[buf][(G_AFR + w + 4 * j) * 64 + lane] = stage[4 + j];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  gload(0);
  swrite(0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < KT) gload(kt + 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      u32x4 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = lds[buf][((wr * 4 + i) * 2 + ks) * 64 + lane];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = lds[buf][(G_AFR + (wc * 4 + j) * 2 + ks) * 64 + lane];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16x16x32(a[i], b[j], acc[i][j]);
    }
    if (kt + 1 < KT) swrite(buf ^ 1);
    __syncthreads();
  }

  // epilogue: lane holds C[4*(lane>>4) + r][lane & 15] of each 16x16 tile
  const int c = lane & 15;
  if (MODE == MODE_SWIGLU) {
    const int F = N >> 1;
    bf16_t* o = static_cast<bf16_t*>(out);
#pragma unroll
    for (int j = 0; j < 4; j += 2) {
      const int gtile = (n0 >> 4) + wc * 4 + j;  // even
      if (gtile + 1 >= NTT + 1) continue;
      const int col = (gtile >> 1) * 16 + c;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + (wr * 4 + i) * 16 + 4 * (lane >> 4) + r;
          if (row < M && gtile < NTT) o[(size_t)row * F + col] = f2bf(silu(acc[i][j][r]) * acc[i][j + 1][r]);
        }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int tile = (n0 >> 4) + wc * 4 + j;
      if (tile >= NTT) continue;
      const int col = tile * 16 + c;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + (wr * 4 + i) * 16 + 4 * (lane >> 4) + r;
          if (row >= M) continue;
          const size_t idx = (size_t)row * N + col;
          const float v = acc[i][j][r];
          if (MODE == MODE_RESIDUAL) {
            float* o = static_cast<float*>(out);
            const float nv = accumulate ? o[idx] + v : v;
            o[idx] = nv;
            if (mirror) mirror[idx] = f2bf(nv);
          } else if (out_f32) {
            static_cast<float*>(out)[idx] = v;
          } else {
            static_cast<bf16_t*>(out)[idx] = f2bf(v);
          }
        }
    }
  }
}

int gemm(const bf16_t* x, const void* W, void* out, int M, int N, int K, int mode, int accumulate, int out_f32,
         bf16_t* mirror, hipStream_t s) {
  if (M <= 0) return 0;
  if ((N & 15) || (K & 31)) return -1;
  if (mode == MODE_SWIGLU && (N & 31)) return -1;
  dim3 grid((N + GB_N - 1) / GB_N, (M + GB_M - 1) / GB_M);
  const u32x4* w = static_cast<const u32x4*>(W);
  switch (mode) {
    case MODE_STORE:
      gemm_kernel<MODE_STORE><<<grid, G_THREADS, 0, s>>>(x, w, out, M, N, K, accumulate, out_f32, nullptr);
      break;
    case MODE_RESIDUAL:
      gemm_kernel<MODE_RESIDUAL><<<grid, G_THREADS, 0, s>>>(x, w, out, M, N, K, accumulate, 1, mirror);
      break;
    case MODE_SWIGLU:
      gemm_kernel<MODE_SWIGLU><<<grid, G_THREADS, 0, s>>>(x, w, out, M, N, K, accumulate, 0, nullptr);
      break;
    default: return -1;
  }
  JLA_CHECK_LAUNCH();
  return 0;
}

}  // namespace jla
