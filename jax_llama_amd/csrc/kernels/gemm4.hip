// gemm4: 256 x 256 output tile per workgroup of FOUR waves (2 x 2), each wave a 128 x 128 sub-tile
// (8 x 8 accumulators of v_mfma_f32_16x16x32_bf16 = 256 fp32 registers, held in the AGPR half of the
// unified register file): ONE wave per SIMD, no ping-pong partner.
//
// Why (profiles/r2_gemm_pmc_vs_hipblaslt.txt, gate_up at M = 4096): hipBLASLt's kernel for these shapes is a
// 256x256x64 macro tile on 4 waves; it moves the same L2 requests (TCP_TCC_READ_REQ identical) and issues the
// same MFMAs as gemm2 (8 waves of 128 x 64, ping-pong), but its waves sit in s_waitcnt / barriers 7.6 % of their
// cycles against gemm2's 27 %, and it finishes 1.23x sooner. A 128 x 128 wave tile also halves the LDS fragment
// reads per MFMA (8 A + 8 B fragments feed 64 MFMAs per 32-deep K-tile).
//
// Pipeline (one barrier per 32-deep K-tile; NBUF LDS slots of 32 KiB = 16 A + 16 B fragments):
//   * operands arrive by LDS-DMA (global_load_lds_dwordx4) in the MFMA fragment layout (1 KiB = 16 rows x 32 k,
//     lane-linear, so every ds_read_b128 is conflict-free): x gathered per lane (16 rows x 64 B per wave-load),
//     the packed weights copied verbatim; K-tile t + NBUF is issued into the slot of K-tile t;
//   * the fragments of K-tile t+1 are read into a second register set while K-tile t's 64 MFMAs run
//     (local-read prefetch), so the MFMAs never wait on LDS;
//   * per K-tile: 16 MFMAs -> [lgkmcnt(0); counted vmcnt (K-tile t+1 landed); s_barrier] -> LDS-DMA issue of
//     K-tile t + NBUF -> ds_reads of K-tile t+1 -> 48 MFMAs. The barrier wait overlaps the first MFMAs.
//     RAW: a wave's LDS-DMA writes of K-tile t+1 are retired by its own vmcnt before the barrier of iteration t,
//     and K-tile t+1 is read after it. WAR: the slot of K-tile t is refilled after the barrier of iteration t;
//     every wave read K-tile t in iteration t-1 and retired those reads (lgkmcnt(0)) before that barrier.
// Fused RMSNorm (RMS): row sums of squares of the A fragments already in registers; epilogue scales rows.
// Epilogues: store (bf16/fp32), residual add + bf16 mirror, SwiGLU over interleaved [w1;w3] tiles, greedy
// argmax partials. No K split: gemm4 serves prefill-sized M (enough 256x256 tiles to fill the chip).
#include "common.h"
#include "launchers.h"

namespace jla {

constexpr int G4_MT = 8, G4_NT = 8;  // 16x16 tiles per wave (128 x 128)
constexpr int G4_BF = 16;             // weight fragments per 32-deep K-tile (256 columns)
constexpr int G4_APIECES = 32;        // 8-row x 128-B x pieces per 64-deep K-tile pair (256 rows)
constexpr int G4_ASLOTS = 3, G4_BSLOTS = 4;
constexpr int G4_ARING = G4_ASLOTS * G4_APIECES * 64;  // u32x4 (96 KiB); the weight ring (64 KiB) follows
constexpr int G4_GROUP_M = 8;
constexpr int G4_PARTIAL = 7;  // == gemm.hip MODE_PARTIAL

JLA_DEV void g4_tile_coords(int pid, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int in_group = G4_GROUP_M * tiles_n;
  const int first_m = (pid / in_group) * G4_GROUP_M;
  const int gsz = min(tiles_m - first_m, G4_GROUP_M);
  tm = first_m + (pid % in_group) % gsz;
  tn = (pid % in_group) / gsz;
}

template <int N>
JLA_DEV void g4_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// The 8 x pieces a wave loads per K-tile pair are issued 4 + 4 with the pair's two K-tiles (issuing all 8 with the
// even K-tile measured 2-6 % slower).
template <int MODE, bool RMS, bool ILV, bool NOLOAD = false>
__global__ void __launch_bounds__(256, 1)
    gemm4_kernel(const bf16_t* __restrict__ x, const u32x4* __restrict__ W, void* __restrict__ out, int M, int N,
                 int K, int accumulate, int out_f32, bf16_t* __restrict__ mirror, int kc, int tiles_m, int tiles_n,
                 float rms_eps, float* __restrict__ ssq_ws, int diag) {
  __shared__ u32x4 lds[G4_ARING + G4_BSLOTS * G4_BF * 64];
  u32x4* const bring = lds + G4_ARING;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;

  // XCD-aware bijective remap, then (split, M-grouped tile) order
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tiles = tiles_m * tiles_n;
  const int split = wgid / tiles;
  const int pid = wgid - split * tiles;
  int tm, tn;
  g4_tile_coords(pid, tiles_m, tiles_n, tm, tn);
  // diagnostics only (wrong results): every workgroup streams the operands of tile column / row 0
  const int m0 = (diag & 4) ? 0 : tm * 256, n0 = (diag & 2) ? 0 : tn * 256;
  const int KS = K >> 5, NTT = N >> 4;
  const int ks0 = split * kc;
  const int KT = min(KS, ks0 + kc) - ks0;

  // x pieces of this wave: P = w + 4j (j < 8) = rows 8P .. 8P+7 of a 64-deep K-tile pair; lane l loads row
  // 8P + (l >> 3), 16-B chunk (l & 7) ^ swz(row) with swz(row) = (row & 15) >> 1 = 4 (P & 1) + (l >> 4), so the
  // LDS image is [row][8 chunks] XOR-swizzled and the A-fragment ds_read_b128s are conflict-free.
  const char* const baseA = reinterpret_cast<const char*>(x + (size_t)m0 * K + (size_t)ks0 * 32);
  const char* const baseB = reinterpret_cast<const char*>(W + ((size_t)(n0 >> 4) * KS + ks0) * 64);
  const unsigned cA = (unsigned)((lane & 7) ^ ((w & 1) * 4 + (lane >> 4)));
  unsigned offA[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int row = min(m0 + 8 * (w + 4 * j) + (lane >> 3), M - 1) - m0;
    offA[j] = (unsigned)row * (unsigned)K * 2u + 16u * cA;
  }
  // weight fragments w + 4j (j < 4) of a K-tile: 1 KiB contiguous in the packed layout
  unsigned bstride[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int nt = min((n0 >> 4) + w + 4 * j, NTT - 1) - (n0 >> 4);
    bstride[j] = __builtin_amdgcn_readfirstlane((unsigned)nt * (unsigned)KS * 1024u);
  }
  const unsigned offB = 16u * (unsigned)lane;
  // pair p (source) into the slot of pair ps (ps != p only past the end: clamped source)
  auto issueA = [&](int p, int j0, int nj, int ps) {
    u32x4* buf = lds + (ps % G4_ASLOTS) * G4_APIECES * 64;
#pragma unroll
    for (int j = j0; j < j0 + nj; ++j) glds16(baseA + (size_t)p * 128 + offA[j], buf + (w + 4 * j) * 64);
  };
  auto issueB = [&](int t, int ts) {
    u32x4* buf = bring + (ts % G4_BSLOTS) * G4_BF * 64;
#pragma unroll
    for (int j = 0; j < 4; ++j) glds16(baseB + (size_t)t * 1024 + bstride[j] + offB, buf + (w + 4 * j) * 64);
  };
  // fragments of K-tile t (h = t & 1: which half of its pair's 128-B lines)
  const int arow = (wr * 128 + (lane & 15)) * 8;
  auto read = [&](int t, auto HC, u32x4* a, u32x4* b) {
    constexpr int h = decltype(HC)::value;
    const u32x4* bbuf = bring + (t % G4_BSLOTS) * G4_BF * 64;
    const u32x4* abuf = lds + ((t >> 1) % G4_ASLOTS) * G4_APIECES * 64 + arow + ((4 * h + (lane >> 4)) ^ ((lane >> 1) & 7));
#pragma unroll
    for (int j = 0; j < G4_NT; ++j) b[j] = bbuf[(wc * G4_NT + j) * 64 + lane];
#pragma unroll
    for (int i = 0; i < G4_MT; ++i) a[i] = abuf[i * 128];
  };

  f32x4 acc[G4_MT][G4_NT];
#pragma unroll
  for (int i = 0; i < G4_MT; ++i)
#pragma unroll
    for (int j = 0; j < G4_NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[G4_MT];  // RMS: partial sums of squares of row (lane & 15) of m-tile i, k-chunk lane >> 4
#pragma unroll
  for (int i = 0; i < G4_MT; ++i) ss[i] = 0.f;

  // prologue: pairs 0, 1 and the weights of K-tiles 0..3 (what K-tiles -4..-1 would have issued); all landed
  if (KT > 0) issueA(0, 0, 8, 0);
  if (KT > 2) issueA(1, 0, 8, 1);
#pragma unroll
  for (int t = 0; t < 4; ++t)
    if (t < KT) issueB(t, t);
  g4_vmcnt<0>();
  __builtin_amdgcn_s_barrier();
  u32x4 a0[G4_MT], b0[G4_NT], a1[G4_MT], b1[G4_NT];
  if (KT > 0) read(0, std::integral_constant<int, 0>{}, a0, b0);

  // one K-tile: MFMAs on (a, b) = K-tile t; reads K-tile t+1 (pair half HN) into (an, bn).
  // Every K-tile issues x half (t & 1) of pair (t >> 1) + 2 and the weights of K-tile t + 4 (4 + 4 LDS-DMA per
  // wave); past the end the sources are clamped to the last pair / K-tile (loads into slots nobody reads again),
  // so the vmcnt below is a constant.
  //  RAW: K-tile t+1's weights were issued at K-tile t-3, its x pair at t-4 / t-3 (odd t+1) or t-3 / t-2 (even
  //       t+1); each wave retires its own part with the counted vmcnt (the loads issued after the last needed
  //       one: 16, or 12 when the x half of K-tile t-2 is needed), then the barrier.
  //  WAR: after the barrier of K-tile t, every wave has retired its reads of K-tile t (weights slot t % 4 is
  //       refilled with K-tile t+4) and of every K-tile of pair (t >> 1) - 1 (refilled with pair (t >> 1) + 2).
  // With one wave per SIMD nothing else hides the issue of the loads and LDS reads: they are interleaved with
  // the 48 MFMAs after the barrier (ILV).
  const int last_pair = (KT >> 1) - 1;
  auto step = [&](int t, auto HN, u32x4* a, u32x4* b, u32x4* an, u32x4* bn) {
    constexpr int hn = decltype(HN)::value;  // == (t + 1) & 1
    // rows 0..1 of the wave tile first: the barrier below overlaps them
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < G4_NT; ++j) acc[i][j] = mfma16x16x32(b[j], a[i], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of K-tile t retired (WAR)
    if constexpr (hn == 0)
      g4_vmcnt<12>();
    else
      g4_vmcnt<16>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);  // (s_setprio bounds a scheduling region: the loads, reads and MFMAs share one)
    if constexpr (!NOLOAD) {  // NOLOAD: diagnostic build without the steady-state LDS-DMA (wrong results)
      issueA(min((t >> 1) + 2, last_pair), hn == 0 ? 4 : 0, 4, (t >> 1) + 2);  // hn == 0 <=> t odd: second half
      issueB(min(t + 4, KT - 1), t + 4);
    }
    read(t + 1, HN, an, bn);  // t + 1 == KT: a harmless read of a slot that is not written any more
    if constexpr (RMS) {
#pragma unroll
      for (int i = 0; i < G4_MT; ++i) ss[i] = dot8_bf16(a[i], a[i], ss[i]);
    }
#pragma unroll
    for (int i = 2; i < G4_MT; ++i)
#pragma unroll
      for (int j = 0; j < G4_NT; ++j) acc[i][j] = mfma16x16x32(b[j], a[i], acc[i][j]);
    if constexpr (ILV) {
      // 8 LDS-DMA issues, then the 16 fragment reads, each behind one MFMA; the rest of the MFMAs last
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 24, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int t = 0; t < KT; t += 2) {  // KT is even (the launcher checks)
    step(t, std::integral_constant<int, 1>{}, a0, b0, a1, b1);
    step(t + 1, std::integral_constant<int, 0>{}, a1, b1, a0, b0);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

  // accumulator layout (weights are the MFMA A operand): acc[i][j][r] = C[row m0 + (wr*8 + i)*16 + (lane & 15)]
  // [col n0 + (wc*8 + j)*16 + 4*(lane >> 4) + r] -- one row and 4 consecutive columns per lane, so the stores
  // are 8 / 16 B per lane and the row statistics of the fused RMSNorm sit in the lane that needs them.
  const int q4 = 4 * (lane >> 4);
  if constexpr (!RMS) {
    // (register allocation: without a pass over the accumulators in (m-tile, row, n-tile) order here, hipcc
    // does not keep them in fixed AGPRs across the main loop -- most MFMAs then copied dst != srcC, plus
    // scratch spills. The factor is an opaque 1.0.)
    float unit = 1.f;
    asm volatile("" : "+v"(unit));
#pragma unroll
    for (int i = 0; i < G4_MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < G4_NT; ++j) acc[i][j][r] *= unit;
  }
  if constexpr (RMS) {
    // complete row sums over the 4 k-chunk lanes (row lane & 15 of m-tile i)
#pragma unroll
    for (int i = 0; i < G4_MT; ++i) {
      ss[i] += __shfl_xor(ss[i], 16, 64);
      ss[i] += __shfl_xor(ss[i], 32, 64);
    }
    if constexpr (MODE == G4_PARTIAL) {
      if (wc == 0 && lane < 16) {
#pragma unroll
        for (int i = 0; i < G4_MT; ++i) {
          const int row = m0 + (wr * G4_MT + i) * 16 + lane;
          if (row < M) ssq_ws[(size_t)split * M + row] = ss[i];
        }
      }
    } else {
      const float inv_k = 1.f / (float)K;
#pragma unroll
      for (int i = 0; i < G4_MT; ++i) {
        const float sc = 1.f / sqrtf(ss[i] * inv_k + rms_eps);
#pragma unroll
        for (int j = 0; j < G4_NT; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] *= sc;
      }
    }
  }

  if constexpr (MODE == MODE_SWIGLU) {
    const int F = N >> 1;
    bf16_t* o = static_cast<bf16_t*>(out);
#pragma unroll
    for (int j = 0; j < G4_NT; j += 2) {
      const int gtile = (n0 >> 4) + wc * G4_NT + j;  // even: gate tile, gtile + 1: its up tile
      if (gtile >= NTT) continue;
      const int col = (gtile >> 1) * 16 + q4;
#pragma unroll
      for (int i = 0; i < G4_MT; ++i) {
        const int row = m0 + (wr * G4_MT + i) * 16 + (lane & 15);
        if (row < M) {
          const f32x4 g = acc[i][j], u = acc[i][j + 1];
          *reinterpret_cast<uint2*>(o + (size_t)row * F + col) =
              make_uint2(pack2bf(silu(g[0]) * u[0], silu(g[1]) * u[1]), pack2bf(silu(g[2]) * u[2], silu(g[3]) * u[3]));
        }
      }
    }
  } else if constexpr (MODE == MODE_ARGMAX) {
    // per row, the first maximum over this wave's 128 columns -> partial [row][n0 / 128 + wc]
    float2* o = static_cast<float2*>(out);
    const int P = tiles_n * 2, slot = (n0 >> 7) + wc;
#pragma unroll
    for (int i = 0; i < G4_MT; ++i) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int j = 0; j < G4_NT; ++j) {
        const int tile = (n0 >> 4) + wc * G4_NT + j;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[i][j][r];
          if (tile < NTT && v > bv) {  // ascending column order: strict > keeps the first maximum
            bv = v;
            bi = tile * 16 + q4 + r;
          }
        }
      }
#pragma unroll
      for (int sh = 16; sh < 64; sh <<= 1) {
        const float ov = __shfl_xor(bv, sh, 64);
        const int oi = __shfl_xor(bi, sh, 64);
        if (ov > bv || (ov == bv && oi < bi)) {
          bv = ov;
          bi = oi;
        }
      }
      const int row = m0 + (wr * G4_MT + i) * 16 + lane;
      if (lane < 16 && row < M) o[(size_t)row * P + slot] = make_float2(bv, __int_as_float(bi));
    }
  } else {
#pragma unroll
    for (int j = 0; j < G4_NT; ++j) {
      const int tile = (n0 >> 4) + wc * G4_NT + j;
      if (tile >= NTT) continue;
      const int col = tile * 16 + q4;
#pragma unroll
      for (int i = 0; i < G4_MT; ++i) {
        const int row = m0 + (wr * G4_MT + i) * 16 + (lane & 15);
        if (row >= M) continue;
        const size_t idx = (size_t)row * N + col;
        const f32x4 v = acc[i][j];
        if constexpr (MODE == G4_PARTIAL) {
          *reinterpret_cast<f32x4*>(static_cast<float*>(out) + (size_t)split * M * N + idx) = v;
        } else if constexpr (MODE == MODE_RESIDUAL) {
          f32x4* o = reinterpret_cast<f32x4*>(static_cast<float*>(out) + idx);
          f32x4 nv = v;
          if (accumulate) nv += *o;
          *o = nv;
          if (mirror) *reinterpret_cast<uint2*>(mirror + idx) = make_uint2(pack2bf(nv[0], nv[1]), pack2bf(nv[2], nv[3]));
        } else if (out_f32) {
          *reinterpret_cast<f32x4*>(static_cast<float*>(out) + idx) = v;
        } else {
          *reinterpret_cast<uint2*>(static_cast<bf16_t*>(out) + idx) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
        }
      }
    }
  }
}

static int g_g4_variant = 0;
void gemm4_set_variant(int v) { g_g4_variant = v; }

template <int MODE, bool RMS>
static void g4_launch(int grid, const bf16_t* x, const u32x4* w, void* out, int M, int N, int K, int accumulate,
                      int out_f32, bf16_t* mirror, int kc, int tm, int tn, float rms_eps, float* ssq, hipStream_t s) {
  // variant bit 0: no MFMA / load interleave (A/B reference); bits 1-2: diagnostics (see the kernel)
  const int diag = g_g4_variant & 6;
  if constexpr (MODE == MODE_STORE && !RMS) {
    if (g_g4_variant & 8) {  // diagnostic: no steady-state loads
      gemm4_kernel<MODE, RMS, true, true><<<grid, 256, 0, s>>>(x, w, out, M, N, K, accumulate, out_f32, mirror, kc, tm,
                                                               tn, rms_eps, ssq, diag);
      return;
    }
  }
  if (g_g4_variant & 1)
    gemm4_kernel<MODE, RMS, false><<<grid, 256, 0, s>>>(x, w, out, M, N, K, accumulate, out_f32, mirror, kc, tm, tn,
                                                        rms_eps, ssq, diag);
  else
    gemm4_kernel<MODE, RMS, true><<<grid, 256, 0, s>>>(x, w, out, M, N, K, accumulate, out_f32, mirror, kc, tm, tn,
                                                       rms_eps, ssq, diag);
}

// mode: MODE_STORE / MODE_RESIDUAL / MODE_SWIGLU / MODE_ARGMAX / 7 (split-K fp32 partial); rms_eps >= 0: fused
// RMSNorm statistic (not in residual mode). Grid = 256x256 tiles x ksplit.
int gemm4_launch(int mode, const bf16_t* x, const void* wv, void* out, int M, int N, int K, int accumulate,
                 int out_f32, bf16_t* mirror, int kc, int ksplit, float rms_eps, float* ssq, hipStream_t s) {
  const u32x4* w = static_cast<const u32x4*>(wv);
  const int KS = K >> 5;
  // the main loop runs K-tile pairs (even number of 32-deep K-tiles); no K split (prefill-sized M)
  if ((KS & 1) || ksplit != 1) return -4;
  const int tm = (M + 255) / 256, tn = (N + 255) / 256;
  const int grid = tm * tn * ksplit;
  const bool rms = rms_eps >= 0.f && mode != MODE_RESIDUAL;
#define JLA_G4(MD)                                                                                       \
  if (rms)                                                                                               \
    g4_launch<MD, true>(grid, x, w, out, M, N, K, accumulate, out_f32, mirror, kc, tm, tn, rms_eps, ssq, s); \
  else                                                                                                   \
    g4_launch<MD, false>(grid, x, w, out, M, N, K, accumulate, out_f32, mirror, kc, tm, tn, rms_eps, ssq, s)
  switch (mode) {
    case MODE_STORE: JLA_G4(MODE_STORE); break;
    case MODE_RESIDUAL: g4_launch<MODE_RESIDUAL, false>(grid, x, w, out, M, N, K, accumulate, out_f32, mirror, kc, tm, tn,
                                                        rms_eps, ssq, s); break;
    case MODE_SWIGLU: JLA_G4(MODE_SWIGLU); break;
    case MODE_ARGMAX: JLA_G4(MODE_ARGMAX); break;
    default: return -1;
  }
#undef JLA_G4
  JLA_CHECK_LAUNCH();
  return 0;
}

}  // namespace jla
