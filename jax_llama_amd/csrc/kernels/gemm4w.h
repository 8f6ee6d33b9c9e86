// gemm4w: the 256 x 256 GEMM main loop with ONE wave per SIMD (4 waves per workgroup, 2 x 2), each wave owning a
// 128 x 128 output block = 8 x 8 v_mfma_f32_16x16x32_bf16 accumulators (256 fp32 registers: the accumulator half of
// gfx950's 512-entry unified register file). K advances 64 per LDS tile (two 32-deep MFMA sub-steps), two LDS slots
// of 64 KiB each (x 32 KiB + W 32 KiB), both filled by LDS-DMA (global_load_lds_dwordx4, no VGPR staging):
//
//   sub-step (t, 0): 64 MFMAs on register set 0 (tile t, k 0..31) | ds_read set 1 <- tile t, k 32..63
//   -- lgkmcnt(0), vmcnt(0) (this wave's part of tile t+1 has landed), s_barrier --
//   sub-step (t, 1): 64 MFMAs on register set 1 | LDS-DMA of tile t+2 into tile t's slot | ds_read set 0 <- tile t+1
//
// so the single wave of a SIMD keeps its own MFMA pipe fed: every LDS read and DMA issue sits in the shadow of the
// MFMAs (sched_group_barrier pins a 4 MFMA : 1 ds_read : 1 DMA interleave), one barrier per 64-deep K-tile, and a
// DMA has one to two sub-steps (~1-2k cycles) to land. Per MFMA a wave reads 256 B of fragments from LDS (the
// 8-wave 128 x 64-per-wave ping-pong of gemm2 reads 384 B and pays a barrier pair per 32 MFMAs).
//
// LDS images (both lane-linear per DMA instruction, so each A / B fragment read is one conflict-free ds_read_b128):
//   x  : [256 rows][8 x 16-B cells] per slot, 8 rows x 128 B per DMA (full cache lines); cell c of row r holds the
//        row's 16-B k-chunk c ^ ((r & 15) >> 1) (the source address is permuted, the destination stays linear);
//   W  : the packed weight fragments (common.h: 16 n x 32 k per 1 KiB) copied verbatim, fragment (n-tile, k half).
// The MFMA runs with the weight fragment as the A operand, so each lane ends up holding 4 CONSECUTIVE output columns
// of one output row per 16 x 16 tile (C^T fragments): RoPE pairs, SwiGLU gate/up pairs and 8-byte packed stores
// fall out in-lane.
//
// Reference ops: jax_llama/model.py:210 (q/k/v projections), :294 (wo), :338 (SwiGLU MLP), :736 (lm_head).
#pragma once
#include "common.h"

namespace jla {

constexpr int G4_BM = 256, G4_BN = 256, G4_BK = 64, G4_GROUP_M = 8;
constexpr int G4_A_U4 = G4_BM * G4_BK * 2 / 16;  // 2048 u32x4 = 32 KiB
constexpr int G4_B_U4 = G4_BN * G4_BK * 2 / 16;  // 2048 u32x4 = 32 KiB
constexpr int G4_SLOT_U4 = G4_A_U4 + G4_B_U4;    // 64 KiB

// launch-order tile index -> (m tile, n tile), M-grouped by gm so consecutive workgroups share W columns
JLA_DEV void g4_tile_coords(int pid, int tiles_m, int tiles_n, int& tm, int& tn, int gm = G4_GROUP_M) {
  const int in_group = gm * tiles_n;
  const int first_m = (pid / in_group) * gm;
  const int gsz = min(tiles_m - first_m, gm);
  tm = first_m + (pid % in_group) % gsz;
  tn = (pid % in_group) / gsz;
}

// The accumulators are pinned to AGPRs through inline asm: with the intrinsic, hipcc (ROCm 7.2) splits the 256
// loop-carried accumulators between the two register files and shuffles them with v_accvgpr moves around every
// MFMA. Volatile, so the MFMAs keep their program order relative to the DMA issues and fragment reads placed between
// them. Hazards: the A / B fragments come from ds_reads (counted by hipcc: the asm names them as inputs), each
// accumulator is read by one MFMA per 64, and g4_acc_fence() pads the MFMA -> v_accvgpr_read hand-off after the loop.
JLA_DEV void g4_mfma(f32x4& acc, const u32x4& a, const u32x4& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
// an accumulator tile for the epilogue, read out of its AGPRs at this point in program order
JLA_DEV f32x4 g4_take(f32x4& a) {
  asm volatile("" : "+a"(a));
  return a;
}
JLA_DEV void g4_acc_fence() { asm volatile("s_nop 7\n\ts_nop 7" ::: "memory"); }

struct G4Args {
  const bf16_t* x;  // [M][K] row-major activations
  const u32x4* W;   // packed [N/16][K/32][64] fragments
  void* out;
  int M, N, K;
  int kc;           // 64-deep K-tiles per split (split = workgroup index / tiles)
  int tiles_m, tiles_n;
};

// The main loop; leaves the C^T accumulators of this wave in acc[j][i] (n-tile j, m-tile i of the wave's block).
// Returns nothing else; the caller's epilogue reads acc. `lds` is the workgroup's 128 KiB staging array.
// RMS: also accumulate the row sums of squares of x (the fused RMSNorm statistic, reference model.py:42-48) from
// the x fragments already in registers: wave (wr, wc) takes m-tiles 4wc..4wc+3 of its row block, ss[i] holds lane
// (row lane & 15, k-chunk lane >> 4)'s partial of m-tile 4wc + i, k32 step after k32 step in K order.
// DIAG (ablation builds for tools/bench_gemm.py --g5-diag 64 / 128, wrong results): 1 no MFMAs (the fragment reads
// kept alive), 2 no LDS-DMA past the prologue (every K-tile re-reads the first two tiles' slots). (Moving the
// sub-step's fragment reads or DMAs into its first 8 slots, two per slot, measured within noise or slower:
// profiles/r5_gemm4_schedule_ab.jsonl.)
template <bool RMS = false, typename Acc, int DIAG = 0, bool W3 = false>
JLA_DEV void g4_mainloop(const G4Args& g, u32x4* lds, int m0, int n0, int t0, int KT, int wu, int lane, Acc& acc,
                         float* ss = nullptr) {
  const int wr = wu >> 1, wc = wu & 1;
  const int K = g.K, KS = K >> 5, NTT = g.N >> 4;

  // ---- DMA sources (saddr form: a wave-uniform base per operand + a 32-bit per-lane offset)
  // x piece P = wu + 4j (j = 0..7): rows 8P + (lane >> 3), cell lane & 7 <- k-chunk (lane & 7) ^ swz(row)
  const char* const baseA = reinterpret_cast<const char*>(g.x + (size_t)m0 * K + (size_t)t0 * 64);
  const char* const baseB = reinterpret_cast<const char*>(g.W + ((size_t)(n0 >> 4) * KS + 2 * t0) * 64);
  unsigned offA[8], offB[8];
  const int mlast = g.M - 1 - m0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int P = wu + 4 * j;
    const int row = min(8 * P + (lane >> 3), mlast);
    const int chunk = (lane & 7) ^ (4 * (P & 1) + (lane >> 4));
    offA[j] = (unsigned)row * (unsigned)K * 2u + 16u * (unsigned)chunk;
    // W fragment f = wu + 4j: n-tile f >> 1, k half f & 1 (= wu & 1)
    const int f = wu + 4 * j;
    const int nt = min((n0 >> 4) + (f >> 1), NTT - 1) - (n0 >> 4);
    offB[j] = ((unsigned)nt * (unsigned)KS + (unsigned)(f & 1)) * 1024u + 16u * (unsigned)lane;
  }
  // slot images: two x + two W halves of 64 KiB slots, or (W3) x slots [0, 2) then three W slots
  auto xslot = [&](int sl) -> u32x4* { return lds + sl * (W3 ? G4_A_U4 : G4_SLOT_U4); };
  auto wslot = [&](int sl) -> u32x4* {
    return W3 ? lds + 2 * G4_A_U4 + sl * G4_B_U4 : lds + sl * G4_SLOT_U4 + G4_A_U4;
  };
  // the j-th of this wave's 16 DMAs of K-tile t (0..7 x into x slot t & 1, 8..15 W into W slot wsl)
  auto dma = [&](int t, int j, int wsl) {
    if (j < 8) {
      glds16(baseA + (size_t)t * 128 + offA[j], xslot(t & 1) + (wu + 4 * j) * 64);
    } else {
      glds16(baseB + (size_t)t * 2048 + offB[j - 8], wslot(wsl) + (wu + 4 * (j - 8)) * 64);
    }
  };

  // ---- fragment reads: A operand = W fragment of n-tile (wc*8 + j), B operand = x fragment of m-tile (wr*8 + i)
  // x: row r = wr*128 + 16i + (lane & 15), k-chunk 4h + (lane >> 4), stored at cell chunk ^ ((r & 15) >> 1)
  const int xrd = (wr * 128 + (lane & 15)) * 8;
  const int xc0 = (0 + (lane >> 4)) ^ ((lane >> 1) & 7), xc1 = (4 + (lane >> 4)) ^ ((lane >> 1) & 7);
  auto rd = [&](u32x4& dst, int xs, int wsl, int h, int q) {  // q 0..7: W n-tile q; 8..15: x m-tile q - 8
    if (q < 8)
      dst = wslot(wsl)[((wc * 8 + q) * 2 + h) * 64 + lane];
    else
      dst = xslot(xs)[xrd + (q - 8) * 128 + (h ? xc1 : xc0)];
  };

  u32x4 w0[8], x0[8], w1[8], x1[8];

  // one 64-MFMA sub-step on (wf, xf), interleaved with up to 16 fragment reads into (wn, xn) from x slot rslot / W slot
  // rw, the 8 x DMAs of tile td (do_dma) and the 8 W DMAs of tile tw into W slot tws (do_wdma)
  auto substep = [&](u32x4 (&wf)[8], u32x4 (&xf)[8], u32x4 (&wn)[8], u32x4 (&xn)[8], bool do_rd, int rslot, int rw,
                     int rh, bool do_dma, int td, bool do_wdma, int tw, int tws) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = 4 * q + u, j = e >> 3, i = e & 7;
        if constexpr (DIAG & 1)
          asm volatile("" ::"v"(wf[j]), "v"(xf[i]));
        else
          g4_mfma(acc[j][i], wf[j], xf[i]);
      }
      if (do_rd) rd(q < 8 ? wn[q] : xn[q - 8], rslot, rw, rh, q);
      if (!(DIAG & 2) && (q < 8 ? do_dma : do_wdma)) dma(q < 8 ? td : tw, q, tws);
      if constexpr (RMS) {
        if (q < 4) {  // m-tile 4wc + q: the runtime wc selects between two named fragments (no indexed array)
          const u32x4 f = wc ? xf[4 + q] : xf[q];
          // plain fp32 FMAs on the unpacked halves: v_dot2 beside the MFMAs costs ~10 cycles each (15 % of the loop)
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

  auto mid_barrier = [&]() {
    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0), visible to hipcc's own wait bookkeeping
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  if constexpr (W3) {
    // W three K-tiles deep (x stays two): tile t's W DMA is issued one K-tile before its x DMA, so the weight
    // stream -- the operand that comes from HBM when few tiles share it (small M) -- has ~3 sub-steps to land
    // instead of ~1.5. Issue order per sub-step: x DMAs then W DMAs; vmcnt retires in order, so "tile t+1 landed"
    // is vmcnt(8) while the next tile's W (the youngest 8) may stay in flight across the barrier.
    if (KT > 0) {
#pragma unroll
      for (int j = 0; j < 16; ++j) dma(0, j, 0);
    }
    if (KT > 1) {
#pragma unroll
      for (int j = 0; j < 16; ++j) dma(1, j, 1);
    }
    if (KT > 2) {
#pragma unroll
      for (int j = 8; j < 16; ++j) dma(2, j, 2);
      wait_vmcnt<24>();
    } else if (KT > 1) {
      wait_vmcnt<16>();
    } else {
      wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (KT > 0) {
#pragma unroll
      for (int q = 0; q < 16; ++q) rd(q < 8 ? w0[q] : x0[q - 8], 0, 0, 0, q);
    }
    // straight-line phases with constant DMA / wait choices (as the two-slot loop below): a single loop with
    // run-time tails merged the register sets and spilled
    auto vm8_barrier = [&]() {
      __builtin_amdgcn_s_waitcnt(0x0078);  // vmcnt(8) lgkmcnt(0): all but the youngest 8 (W of tile t+2)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };
    int t = 0, wt = 0;  // wt = t % 3: tile t's W slot
    for (; t + 3 < KT; ++t) {
      const int wn1 = wt == 2 ? 0 : wt + 1;
      substep(w0, x0, w1, x1, true, t & 1, wt, 1, false, 0, false, 0, 0);
      vm8_barrier();
      // x of tile t+2 into tile t's x slot, W of tile t+3 into tile t's W slot (both read out before the barrier)
      substep(w1, x1, w0, x0, true, (t + 1) & 1, wn1, 0, true, t + 2, true, t + 3, wt);
      wt = wn1;
    }
    if (t + 2 < KT) {  // third to last: the last x DMA, no W left to issue
      const int wn1 = wt == 2 ? 0 : wt + 1;
      substep(w0, x0, w1, x1, true, t & 1, wt, 1, false, 0, false, 0, 0);
      vm8_barrier();
      substep(w1, x1, w0, x0, true, (t + 1) & 1, wn1, 0, true, t + 2, false, 0, 0);
      wt = wn1;
      ++t;
    }
    if (t + 1 < KT) {  // second to last: nothing left to DMA
      const int wn1 = wt == 2 ? 0 : wt + 1;
      substep(w0, x0, w1, x1, true, t & 1, wt, 1, false, 0, false, 0, 0);
      mid_barrier();
      substep(w1, x1, w0, x0, true, (t + 1) & 1, wn1, 0, false, 0, false, 0, 0);
      wt = wn1;
      ++t;
    }
    if (t < KT) {  // last K-tile
      substep(w0, x0, w1, x1, true, t & 1, wt, 1, false, 0, false, 0, 0);
      substep(w1, x1, w0, x0, false, 0, 0, 0, false, 0, false, 0, 0);
    }
    wait_vmcnt<0>();
    g4_acc_fence();
    return;
  }

  // prologue: tiles 0 and 1 in flight, tile 0 landed, set 0 <- tile 0 k 0..31
  if (KT > 0) {
#pragma unroll
    for (int j = 0; j < 16; ++j) dma(0, j, 0);
  }
  if (KT > 1) {
#pragma unroll
    for (int j = 0; j < 16; ++j) dma(1, j, 1);
    wait_vmcnt<16>();
  } else {
    wait_vmcnt<0>();
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (KT > 0) {
#pragma unroll
    for (int q = 0; q < 16; ++q) rd(q < 8 ? w0[q] : x0[q - 8], 0, 0, 0, q);
  }

  int t = 0;
  for (; t + 2 < KT; ++t) {  // steady state: reads of tile t+1 and DMA of tile t+2 in every K-tile
    substep(w0, x0, w1, x1, true, t & 1, t & 1, 1, false, 0, false, 0, 0);
    mid_barrier();
    substep(w1, x1, w0, x0, true, (t + 1) & 1, (t + 1) & 1, 0, true, t + 2, true, t + 2, t & 1);
  }
  if (t + 1 < KT) {  // second to last: nothing left to DMA
    substep(w0, x0, w1, x1, true, t & 1, t & 1, 1, false, 0, false, 0, 0);
    mid_barrier();
    substep(w1, x1, w0, x0, true, (t + 1) & 1, (t + 1) & 1, 0, false, 0, false, 0, 0);
    ++t;
  }
  if (t < KT) {  // last K-tile
    substep(w0, x0, w1, x1, true, t & 1, t & 1, 1, false, 0, false, 0, 0);
    substep(w1, x1, w0, x0, false, 0, 0, 0, false, 0, false, 0, 0);
  }
  g4_acc_fence();
}

// ---------------------------------------------------------------------------------------------
// g4n_mainloop: the same loop for a 256 (M) x 32 NJ (N) workgroup tile -- each wave a 128 (M) x 16 NJ (N) block,
// NJ x 8 accumulators (NJ = 4: 256 x 128 tiles, 128 accumulator AGPRs per wave; NJ = 6: 256 x 192). Twice the
// tiles of the 256 x 256 loop for the outputs whose 256 x 256 grid quantises badly on 256 CUs (Llama-3-8B at M = 2048: o has 128 tiles ->
// 256 with no K split; w1|w3 896 = 3.5 waves -> 1792 = 7 whole waves), at 1.5x the operand bytes per MFMA. Same LDS
// images and slot layout (the W half of a slot is half used), same two sub-steps per 64-deep K-tile and one barrier;
// per sub-step 8 NJ MFMAs with the 8 + NJ fragment reads and 8 + NJ LDS-DMA issues spread over the first slots.
// No in-loop norm statistic (the caller precomputes it: RMSM 0 / 2 only).
template <int NJ, typename Acc, bool W3 = true>
JLA_DEV void g4n_mainloop(const G4Args& g, u32x4* lds, int m0, int n0, int t0, int KT, int wu, int lane, Acc& acc) {
  static_assert(NJ == 4 || NJ == 6 || NJ == 8, "n-tiles per wave");
  static_assert(W3, "the narrow tiles keep the weights three K-tiles deep (the two-slot form was removed in round 6)");
  constexpr int ND = NJ;           // W DMAs per wave per K-tile (2 NJ n-tiles x 2 k halves / 4 waves)
  constexpr int NQ = 8 + NJ;       // fragment reads / DMA issues per sub-step
  constexpr int MPS = (8 * NJ) / 16;  // MFMAs per slot (16 slots per sub-step)
  const int wr = wu >> 1, wc = wu & 1;
  const int K = g.K, KS = K >> 5, NTT = g.N >> 4;
  const char* const baseA = reinterpret_cast<const char*>(g.x + (size_t)m0 * K + (size_t)t0 * 64);
  const char* const baseB = reinterpret_cast<const char*>(g.W + ((size_t)(n0 >> 4) * KS + 2 * t0) * 64);
  unsigned offA[8], offB[ND];
  const int mlast = g.M - 1 - m0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int P = wu + 4 * j;
    const int row = min(8 * P + (lane >> 3), mlast);
    const int chunk = (lane & 7) ^ (4 * (P & 1) + (lane >> 4));
    offA[j] = (unsigned)row * (unsigned)K * 2u + 16u * (unsigned)chunk;
  }
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    const int f = wu + 4 * j;  // W fragment f: n-tile f >> 1 of the workgroup tile, k half f & 1
    const int nt = min((n0 >> 4) + (f >> 1), NTT - 1) - (n0 >> 4);
    offB[j] = ((unsigned)nt * (unsigned)KS + (unsigned)(f & 1)) * 1024u + 16u * (unsigned)lane;
  }
  // slot images as g4_mainloop: x + W halves of two 64 KiB slots, or (W3) two x slots then three W slots
  auto xslot = [&](int sl) -> u32x4* { return lds + sl * (W3 ? G4_A_U4 : G4_SLOT_U4); };
  auto wslot = [&](int sl) -> u32x4* {
    return W3 ? lds + 2 * G4_A_U4 + sl * G4_B_U4 : lds + sl * G4_SLOT_U4 + G4_A_U4;
  };
  auto dma = [&](int t, int j, int wsl) {  // the j-th of this wave's NQ DMAs of K-tile t (0..7 x, then W)
    if (j < 8)
      glds16(baseA + (size_t)t * 128 + offA[j], xslot(t & 1) + (wu + 4 * j) * 64);
    else
      glds16(baseB + (size_t)t * 2048 + offB[j - 8], wslot(wsl) + (wu + 4 * (j - 8)) * 64);
  };
  const int xrd = (wr * 128 + (lane & 15)) * 8;
  const int xc0 = (0 + (lane >> 4)) ^ ((lane >> 1) & 7), xc1 = (4 + (lane >> 4)) ^ ((lane >> 1) & 7);
  auto rd = [&](u32x4& dst, int xs, int wsl, int h, int q) {  // q < NJ: W n-tile q of the wave; else x m-tile q - NJ
    if (q < NJ)
      dst = wslot(wsl)[((wc * NJ + q) * 2 + h) * 64 + lane];
    else
      dst = xslot(xs)[xrd + (q - NJ) * 128 + (h ? xc1 : xc0)];
  };
  u32x4 w0[NJ], x0[8], w1[NJ], x1[8];
  auto substep = [&](u32x4 (&wf)[NJ], u32x4 (&xf)[8], u32x4 (&wn)[NJ], u32x4 (&xn)[8], bool do_rd, int rslot, int rw,
                     int rh, bool do_dma, int td, bool do_wdma, int tw, int tws) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
#pragma unroll
      for (int u = 0; u < MPS; ++u) {
        const int e = MPS * q + u, j = e >> 3, i = e & 7;
        g4_mfma(acc[j][i], wf[j], xf[i]);
      }
      if (q < NQ) {
        if (do_rd) rd(q < NJ ? wn[q] : xn[q - NJ], rslot, rw, rh, q);
        if (q < 8 ? do_dma : do_wdma) dma(q < 8 ? td : tw, q, tws);
      }
    }
  };
  auto mid_barrier = [&]() {
    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  {  // W three K-tiles deep (g4_mainloop W3): barriers wait for all but the youngest ND W DMAs
    static_assert(ND < 16, "vmcnt immediate");
    if (KT > 0) {
#pragma unroll
      for (int j = 0; j < NQ; ++j) dma(0, j, 0);
    }
    if (KT > 1) {
#pragma unroll
      for (int j = 0; j < NQ; ++j) dma(1, j, 1);
    }
    if (KT > 2) {
#pragma unroll
      for (int j = 8; j < NQ; ++j) dma(2, j, 2);
      wait_vmcnt<8 + 2 * ND>();
    } else if (KT > 1) {
      wait_vmcnt<8 + ND>();
    } else {
      wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (KT > 0) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) rd(q < NJ ? w0[q] : x0[q - NJ], 0, 0, 0, q);
    }
    auto vmw_barrier = [&]() {
      __builtin_amdgcn_s_waitcnt(0x0070 | ND);  // vmcnt(ND) lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };
    int t = 0, wt = 0;
    for (; t + 3 < KT; ++t) {
      const int wn1 = wt == 2 ? 0 : wt + 1;
      substep(w0, x0, w1, x1, true, t & 1, wt, 1, false, 0, false, 0, 0);
      vmw_barrier();
      substep(w1, x1, w0, x0, true, (t + 1) & 1, wn1, 0, true, t + 2, true, t + 3, wt);
      wt = wn1;
    }
    if (t + 2 < KT) {
      const int wn1 = wt == 2 ? 0 : wt + 1;
      substep(w0, x0, w1, x1, true, t & 1, wt, 1, false, 0, false, 0, 0);
      vmw_barrier();
      substep(w1, x1, w0, x0, true, (t + 1) & 1, wn1, 0, true, t + 2, false, 0, 0);
      wt = wn1;
      ++t;
    }
    if (t + 1 < KT) {
      const int wn1 = wt == 2 ? 0 : wt + 1;
      substep(w0, x0, w1, x1, true, t & 1, wt, 1, false, 0, false, 0, 0);
      mid_barrier();
      substep(w1, x1, w0, x0, true, (t + 1) & 1, wn1, 0, false, 0, false, 0, 0);
      wt = wn1;
      ++t;
    }
    if (t < KT) {
      substep(w0, x0, w1, x1, true, t & 1, wt, 1, false, 0, false, 0, 0);
      substep(w1, x1, w0, x0, false, 0, 0, 0, false, 0, false, 0, 0);
    }
    wait_vmcnt<0>();
    g4_acc_fence();
  }
}

// Staged bf16 epilogue, in two steps on the wave's private 32 KiB of the (now idle) staging array:
//  g4_stage_put: lane (c, q) puts its 4 bf16 of an output row (8 bytes at logical byte cb of local row r) -- rows of
//    CB bytes, 8-byte granules XOR-swizzled by (r & 15) so the 16 rows a lane group writes hit distinct banks;
//  g4_stage_rows: after lgkmcnt(0), each lane takes 16 contiguous bytes of a row (CB / 16 lanes per row) and hands
//    them to store(local row, 16-byte chunk index, data) -- full-row global stores instead of 16-row x 32-byte pieces
//    (the direct form cost 10+ % at prefill sizes: the epilogue runs with the CU's MFMA pipes idle).
template <int CB>
JLA_DEV constexpr int g4_swz(int r) { return ((r & 15) << 3) & (CB - 1); }  // (rows narrower than 128 B: fewer banks)
template <int CB>
JLA_DEV void g4_stage_put(char* wl, int r, int cb, u32x2 v) {
  *reinterpret_cast<u32x2*>(wl + r * CB + (cb ^ g4_swz<CB>(r))) = v;
}
template <int CB, typename F>
JLA_DEV void g4_stage_rows(const char* wl, int lane, F&& store) {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's own puts landed (the region is wave-private)
  constexpr int LPR = CB / 16, RPI = 64 / LPR;
  const int ch = lane % LPR;
#pragma unroll 4
  for (int s = 0; s < 128 / RPI; ++s) {
    const int r = RPI * s + lane / LPR;
    const int sw = g4_swz<CB>(r);
    u32x4 v = *reinterpret_cast<const u32x4*>(wl + r * CB + ((16 * ch) ^ (sw & ~15)));
    if (sw & 8) v = u32x4{v[2], v[3], v[0], v[1]};
    store(r, ch, v);
  }
}

// bf16 store of the wave's 128 x 128 block through LDS: each lane packs its 4 consecutive columns per tile into
// one 8-byte ds_write (row-XOR-swizzled at 8-byte granularity: conflict-free for the 16 rows of a lane group), then
// reads back 16 B of a row per lane and writes full 256-B row segments (32 x 16-B stores per lane). The caller has
// passed a barrier after the last fragment read; the wave uses its own 32 KiB of the staging array.
template <typename Acc>
JLA_DEV void g4_store_bf16(Acc& acc, u32x4* lds, bf16_t* out, int M, int N, int m0, int n0, int wu, int lane) {
  const int wr = wu >> 1, wc = wu & 1;
  char* const wl = reinterpret_cast<char*>(lds) + wu * 32768;
  const int c = lane & 15, q = lane >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = 16 * i + c;  // local row
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f32x4 v = acc[j][i];
      const u32x2 p = {pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
      const int cb = (32 * j + 8 * q) ^ (c << 3);
      *reinterpret_cast<u32x2*>(wl + r * 256 + cb) = p;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own writes landed (the region is wave-private)
  const int gcol = n0 + wc * 128 + 8 * c;
#pragma unroll 8
  for (int s = 0; s < 32; ++s) {
    const int r = 4 * s + q;
    const int sw = (r & 15) << 3;
    u32x4 v = *reinterpret_cast<const u32x4*>(wl + r * 256 + ((16 * c) ^ (sw & ~15)));
    if (sw & 8) v = u32x4{v[2], v[3], v[0], v[1]};
    const int grow = m0 + wr * 128 + r;
    if (grow < M && gcol < N) *reinterpret_cast<u32x4*>(out + (size_t)grow * N + gcol) = v;
  }
}


}  // namespace jla
