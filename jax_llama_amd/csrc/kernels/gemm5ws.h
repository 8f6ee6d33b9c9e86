// gemm5: the weight-streaming GEMM for decode batches of 128-256 rows (tile config 11; split-K partial slabs summed by
// gemm_reduce_kernel, which runs every epilogue).
//
// At M = 256 the projections sit at the HBM / MFMA balance point (256 FLOP per weight byte; ~400 at the dense bf16
// peak), and the narrow tensor-parallel shards (Llama-3-70B at MP 8: qkv N 1280, w1|w3 N 7168, K 8192) have too few
// 256 x 256 output tiles to fill 256 CUs, so every plan splits K. The 256 x 256 LDS kernels (gemm2 / gemm4) then stage
// BOTH operands through LDS with one or two 64 KiB K-tiles in flight per CU -- at 1-2 us of HBM latency that caps a CU
// at ~30-60 GB/s, below what the W stream needs (profiles/r5_tp8_m256_gemm_plans_vs_hipblaslt.jsonl: w1|w3 57 us
// against an 18.7 us weight roofline).
//
// Here each wave owns ALL the tile's rows (MT m-tiles of 16) x NTW n-tiles of 16 and streams its weight fragments
// straight from HBM into registers (the packed 16 x 32 fragments are already the MFMA A operand: one 1 KiB nt load
// per fragment, no LDS hop), G5_A K-stages of 64 ahead in a hand-counted register ring; each weight fragment feeds MT
// MFMAs. Only x -- shared by the 4 waves, L2-resident -- goes through LDS (LDS-DMA, 8-row x 128-B pieces, the gemm4
// swizzled image), in G5_A + 1 stage slots. One barrier per 64-deep K-stage. Per CU ~4 x 8 KiB x G5_A of weights in
// flight (96 KiB at G5_A = 3), so a CU can pull ~60 GB/s from HBM.
//
// Workgroup tile: rows [16 MT tm, +16 MT) x columns [64 NTW tn, +64 NTW) (wave w: n-tiles 4 NTW tn + NTW w + j), K
// stages [kc split, +kc). MFMA: A = W fragment, B = x fragment, so lane (c = lane & 15, q = lane >> 4) of acc[j][i]
// holds output row 16 i + c at the 4 consecutive columns 16 (n-tile j) + 4 q .. +3 (C^T, as gemm4): one float4
// partial store per accumulator. Fused RMSNorm (rms != 0): wave w also sums the squares of m-tiles w, w + 4, ... from
// the staged x (the per-split partial statistic the reduce kernel expects).
//
// Reference ops: jax_llama/model.py:210 (wq/wk/wv), :294 (wo), :338 (w1/w3/w2) -- the decode projections at 128-256
// rows per step.
#pragma once
#include "common.h"
#include "gemm4w.h"
#include "ring.h"

namespace jla {

constexpr int G5_A = 3;              // K-stages in flight beyond the one being computed
constexpr int G5_SLOTS = G5_A + 1;   // x stage slots in LDS / weight register ring slots
constexpr int G5_TILE = 11;          // tile config id (gemm.hip dispatch, ops/autotune.py): NTW 4; 12: NTW 2
__device__ u32x4 g5_zero_frag[64];   // 1 KiB of zeros: the weight fragment of stages past the end (MFMA adds 0)

template <int MT, int NTW>
__global__ void __launch_bounds__(256, 1)
    gemm5_partial_kernel(const bf16_t* __restrict__ x, const u32x4* __restrict__ W, float* __restrict__ ws, int M,
                         int N, int K, int kc, int tiles_m, int tiles_n, float* __restrict__ ssq, int diag) {
  static_assert(MT == 8 || MT == 16, "rows per workgroup: 128 or 256");
  static_assert(NTW == 2 || NTW == 4, "n-tiles per wave");
  constexpr int ROWS = 16 * MT;
  constexpr int XS_U4 = ROWS * 8;      // one x stage: ROWS x 128 B
  constexpr int XP = ROWS / 8 / 4;     // x DMA pieces (8 rows x 128 B) per wave per stage
  constexpr int OPS = XP + 2 * NTW;    // vector-memory ops per wave per stage
  __shared__ u32x4 lds[G5_SLOTS * XS_U4];

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-aware bijective remap: consecutive ids share an XCD; the workgroups of one (split, m-tile) -- the same x
  // slab -- are consecutive
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tn = wgid % tiles_n, rest = wgid / tiles_n;
  const int tm = rest % tiles_m, split = rest / tiles_m;
  const int KS = K >> 5, KS64 = K >> 6;
  const int s0 = split * kc;
  const int NS = (diag & 16) ? 0 : min(KS64, s0 + kc) - s0;  // <= 0: a split past the end (writes zero slabs)
  const int NTT = N >> 4;
  const int m0 = tm * ROWS;
  const int nt0 = (tn * 4 + w) * NTW;

  f32x4 acc[NTW][MT];
#pragma unroll
  for (int j = 0; j < NTW; ++j)
#pragma unroll
    for (int i = 0; i < MT; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[MT / 4];
#pragma unroll
  for (int q = 0; q < MT / 4; ++q) ss[q] = 0.f;

  if (NS > 0) {
    // weight fragment (n-tile nt0 + j, k-step 2 (s0 + u) + h) at wp[j] + (2u + h) * 64 (clamped n-tiles re-read the last)
    const u32x4* wp[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) wp[j] = W + ((size_t)min(nt0 + j, NTT - 1) * KS + 2 * (size_t)s0) * 64 + lane;
    // x DMA: piece P = w + 4 i (rows 8P .. 8P + 7), lane L -> row 8P + L / 8, cell L % 8 <- k-chunk cell ^ swz(row)
    const char* const xbase = reinterpret_cast<const char*>(x + (size_t)s0 * 64);
    unsigned xoff[XP];
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      const int P = w + 4 * i;
      const int row = min(m0 + 8 * P + (lane >> 3), M - 1);
      const int chunk = (lane & 7) ^ (4 * (P & 1) + (lane >> 4));
      xoff[i] = (unsigned)row * (unsigned)K * 2u + 16u * (unsigned)chunk;
    }
    u32x4 r0[2][NTW], r1[2][NTW], r2[2][NTW], r3[2][NTW];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < NTW; ++j) r0[h][j] = r1[h][j] = r2[h][j] = r3[h][j] = u32x4{0u, 0u, 0u, 0u};

    // stage u into x slot `slot` / ring slot wr. Past the end (the ring is unrolled by 4 and never branches around
    // its loads: hipcc would merge in-flight registers with copies) x re-loads the last stage and the weights load the
    // zero fragment, so the extra MFMAs add 0
    const u32x4* const zf = g5_zero_frag + lane;
    // diag (tools only, wrong results): bit 0 no MFMAs, bit 1 weights from the (cached) zero fragment, bit 2 x DMA
    // from stage 0 of row block 0 (cached), bit 3 no partial stores, bit 4 no main loop
    auto issue = [&](int u, u32x4 (&wr)[2][NTW], int slot) {
      const bool live = u < NS && !(diag & 2);
      const int uc = (diag & 4) ? 0 : min(u, NS - 1);
      u32x4* const xs = lds + slot * XS_U4;
#pragma unroll
      for (int i = 0; i < XP; ++i) glds16_asm(xbase + (size_t)uc * 128 + xoff[i], xs + (w + 4 * i) * 64);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < NTW; ++j) asm_load_nt<true>(wr[h][j], live ? (const void*)(wp[j] + (size_t)(2 * uc + h) * 64)
                                                                  : (const void*)zf);
    };
    // x fragment of m-tile i, k-step half h of a stage: row 16 i + (lane & 15), k-chunk 4h + (lane >> 4)
    const int xrow = (lane & 15) * 8;
    const int xc0 = (lane >> 4) ^ ((lane >> 1) & 7), xc1 = (4 + (lane >> 4)) ^ ((lane >> 1) & 7);
    auto compute = [&](u32x4 (&wr)[2][NTW], int slot, bool live) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < NTW; ++j) pin(wr[h][j]);
      const u32x4* const xs = lds + slot * XS_U4;
      // x fragment e = (h, i) of the stage, read two fragments ahead of its MFMAs (the ds_read latency hides behind
      // 2 NTW MFMAs; hipcc otherwise issues each read right before its first use and waits lgkmcnt(0) on it)
      auto xfrag = [&](int e) { return xs[xrow + (e % MT) * 128 + (e < MT ? xc0 : xc1)]; };
      // (four registers in rotation: a read never targets the operand of the MFMAs issued just before it)
      u32x4 xq[4];
      xq[0] = xfrag(0);
      xq[1] = xfrag(1);
#pragma unroll
      for (int e = 0; e < 2 * MT; ++e) {
        if (e + 2 < 2 * MT) xq[(e + 2) % 4] = xfrag(e + 2);
        const int h = e / MT, i = e % MT;
        if (!(diag & 1)) {
#pragma unroll
          for (int j = 0; j < NTW; ++j) g4_mfma(acc[j][i], wr[h][j], xq[e % 4]);
        }
      }
      if (ssq != nullptr && live) {  // wave-uniform: this wave's rows of the fused-norm statistic
#pragma unroll
        for (int q = 0; q < MT / 4; ++q) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const u32x4 f = xs[xrow + (w + 4 * q) * 128 + (h ? xc1 : xc0)];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float lo = __uint_as_float(f[e] << 16), hi = __uint_as_float(f[e] & 0xffff0000u);
              ss[q] = fmaf(lo, lo, ss[q]);
              ss[q] = fmaf(hi, hi, ss[q]);
            }
          }
        }
      }
    };
    // one stage: wait for its loads (this wave's), barrier (every wave's x landed; every wave done with the slot the
    // next issue overwrites), refill that slot with stage u + G5_A, compute stage u
    auto stage = [&](int u, u32x4 (&cur)[2][NTW], int cslot, u32x4 (&nxt)[2][NTW], int nslot) {
      wait_vmcnt<(G5_A - 1) * OPS>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue(u + G5_A, nxt, nslot);
      compute(cur, cslot, u < NS);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    issue(0, r0, 0);
    issue(1, r1, 1);
    issue(2, r2, 2);
    static_assert(G5_A == 3, "the ring below is unrolled for 3 stages in flight");
    for (int u = 0; u < NS; u += 4) {
      stage(u, r0, 0, r3, 3);
      stage(u + 1, r1, 1, r0, 0);
      stage(u + 2, r2, 2, r1, 1);
      stage(u + 3, r3, 3, r2, 2);
    }
    // drain the ring (the clamped tail loads) before anything reuses its registers or the LDS
    wait_vmcnt<0>();
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        pin(r0[h][j]);
        pin(r1[h][j]);
        pin(r2[h][j]);
        pin(r3[h][j]);
      }
  }
  g4_acc_fence();
  // fp32 partial slab [split][M][N]: lane (c, q) of acc[j][i] -> row m0 + 16 i + c, columns 16 (nt0 + j) + 4q .. +3
  const int c = lane & 15, q4 = lane >> 4;
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int row = m0 + 16 * i + c;
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const f32x4 v = g4_take(acc[j][i]);
      const int col = 16 * (nt0 + j) + 4 * q4;
      if (row < M && nt0 + j < NTT && !(diag & 8)) *reinterpret_cast<f32x4*>(ws + ((size_t)split * M + row) * N + col) = v;
    }
  }
  if (ssq != nullptr && tn == 0) {
#pragma unroll
    for (int q = 0; q < MT / 4; ++q) {
      float v = ss[q];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const int row = m0 + 16 * (w + 4 * q) + c;
      if (q4 == 0 && row < M) ssq[(size_t)split * M + row] = v;
    }
  }
}

}  // namespace jla
