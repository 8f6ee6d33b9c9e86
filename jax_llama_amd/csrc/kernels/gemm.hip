// Linear layer for M > 32 rows (prefill, and large-batch decode): y = epilogue(x[M, K] @ W[N, K]^T),
// bf16 MFMA. x arrives RMS-scaled in bf16 (rms_scale) when a norm precedes the projection.
//
// Tiling (CDNA4): 128 x 128 output tile per 256-thread workgroup, 4 waves in 2 x 2, each wave a
// 64 x 64 sub-tile = 4 x 4 v_mfma_f32_16x16x32_bf16 accumulators. K advances 64 per stage. Both
// operands are staged into LDS in the MFMA *fragment* layout (16 rows x 32 k = 64 lanes x 16 B),
// so every LDS fragment read is a lane-linear ds_read_b128 (bank-conflict free) and the packed
// weights are copied verbatim (each 1 KiB fragment is already contiguous in HBM). Double-buffered
// LDS; the next stage's global loads are issued before the current stage's MFMAs and written to
// LDS after them (issue-early / write-late), one barrier per stage.
//
// Decode at batch 64..512 has too few 128x128 tiles to fill 256 CUs, so K can be split over
// gridDim.z workgroups: each writes an fp32 partial tile, and gemm_reduce_kernel sums the splits in
// fixed order (deterministic) and runs the epilogue: store bf16/fp32, residual add (+ bf16 mirror),
// SiLU(gate)*up over the interleaved [w1;w3] tiles, or RoPE + KV-cache write for the fused qkv
// projection (reference ops: model.py:210/294/338/736, :58-92, :169-199, :392/:398).
#include <type_traits>

#include "car.h"
#include "common.h"
#include "gemm4w.h"
#include "gemm5ws.h"
#include "launchers.h"
#include "ring.h"

namespace jla {

constexpr int MODE_PARTIAL = 7;  // split-K: fp32 partial tile to the workspace

// ---------------------------------------------------------------------------------------------
// gemm2: BM x 256 tile (BM = 128 * WM), 4 * WM waves as WM(M) x 4(N), each wave a 128 x 64 sub-tile
// (8 x 4 accumulators of 16x16, 128 fp32 registers). K advances 32 per LDS tile; 4 LDS tile buffers
// filled by LDS-DMA (global_load_lds_dwordx4, no VGPR staging) run 3 tiles ahead of the MFMAs: at
// the top of each K-tile a wave waits (counted vmcnt, never 0 in steady state) only for ITS part of
// the tile it is about to read, then one raw s_barrier publishes every wave's part and retires the
// reads of the buffer being refilled next (WAR). Both operands are stored fragment-shaped in LDS
// (1 KiB = 16 rows x 32 k, lane-linear), so every ds_read_b128 is conflict-free: the packed weights
// are copied verbatim, x is gathered by per-lane source addresses (16 rows x 64 B per wave-load).
// Workgroups are remapped so consecutive tiles share an XCD (its own L2), M-grouped by 8.
constexpr int G2_BN = 256, G2_NBUF = 4, G2_DIST = 3, G2_GROUP_M = 8;
#ifdef JLA_GEMM_STAMPS
// diagnostic build only (tools/debug/gemm_stamps.hip): per-wave cycles of the ping-pong phases
__device__ unsigned long long g_gemm_stamps[8192 * 8 * 6];
#endif

// tile index (in the M-grouped launch order) -> (m tile, n tile); shared by the data-parallel launch
// and the stream-K tail so both walk the same order
JLA_DEV void g2_tile_coords(int pid, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int in_group = G2_GROUP_M * tiles_n;
  const int first_m = (pid / in_group) * G2_GROUP_M;
  const int gsz = min(tiles_m - first_m, G2_GROUP_M);
  tm = first_m + (pid % in_group) % gsz;
  tn = (pid % in_group) / gsz;
}

// RMS (fused RMSNorm, reference model.py:28-48 with the gain folded into W): the A operand is the
// UNscaled bf16 activation; the waves square-sum the A fragments they already read from LDS (wave wc
// takes m-tiles 2wc, 2wc+1 of its row block, 8 v_dot2 per K-tile) and the epilogue scales each output
// row by rsqrt(mean(x^2) + eps). Split-K: each split stores its partial sums ([split][M] after the
// fp32 slabs) and the reduce kernel finishes the statistic. No rms_scale launch, no scaled copy of x.
// SUB = 2 (ping-pong only): each K-tile runs as two half phases per wave group -- [half the tile's
// LDS-DMA issue + the A/B fragments of m-tiles 0..MT/2-1] -> 16 MFMAs, then [the other half of the issue +
// the remaining A fragments + the vmcnt wait for tile t+1] -> 16 MFMAs -- so the partner group's MFMA
// phase hides a shorter load phase (cdna_hip_programming.md T3+T4: the per-phase interleave is the lever).
// FA (full-line A; 256 x 256 ping-pong only): x is staged in 8-row x 128-B pieces that cover a PAIR of
// K-tiles (lane l of a piece loads row l>>3, 16-B chunk (l&7) ^ swz(row)), instead of 16-row x 64-B
// fragment-shaped loads: half the cache lines per LDS-DMA instruction, so half the TA work for x
// (cdna_hip_programming.md §5 "x through LDS in full 128-B lines"). The LDS image [row][8 chunks] is
// XOR-swizzled (swz = (row & 15) >> 1) so the A-fragment ds_read_b128s stay conflict-free under the
// gfx950 b128 lane groups. x pairs live in a 3-slot ring (96 KiB), weights in the usual 4-slot K-tile
// ring (64 KiB); pair p is issued in two halves with K-tiles 2p-4 and 2p-3 (4 LDS-DMA per wave per
// K-tile, as before), so the vmcnt accounting stays "everything issued two K-tiles back has landed".
template <int MODE, int WM, int NBUF = G2_NBUF, bool LATE_WAIT = false, bool RMS = false, int MT = 8, int NTW = 4,
          int SUB = 1, bool FA = false, int FAM = 0>
__global__ void __launch_bounds__(256 * WM)
    gemm2_kernel(const bf16_t* __restrict__ x, const u32x4* __restrict__ W, void* __restrict__ out, int M, int N,
                 int K, int accumulate, int out_f32, bf16_t* __restrict__ mirror, int kc, int tiles_m, int tiles_n,
                 float rms_eps, float* __restrict__ ssq_ws, QKVArgs qa) {
  // wave tile: MT m-tiles x NTW n-tiles of 16x16 (128 x 64 by default; 64 x 32 for the 128 x 128 tile)
  constexpr int NW = 4 * WM, BM = 16 * MT * WM, BN = 64 * NTW;
  constexpr int RPW = MT / 4;  // RMS: m-tiles whose row statistics each wave accumulates
  constexpr int AF = BM / 16, BF = BN / 16, FR = AF + BF;  // fragments per K-tile
  constexpr int G = FR / NW;                                   // LDS-DMA loads per wave per K-tile
  static_assert(FR % NW == 0, "fragment split");
  constexpr int DIST = NBUF - 1;
  constexpr int A_SLOTS = 3, A_PIECES = BM / 8, A_RING = FA ? A_SLOTS * A_PIECES * 64 : 0;
  static_assert(!FA || (WM == 2 && MT == 8 && NTW == 4 && SUB == 1 && NBUF == 4 && BF == 2 * NW),
                "FA: 256 x 256 ping-pong, 2 weight fragments per wave per K-tile");
  __shared__ u32x4 lds[FA ? A_RING + NBUF * BF * 64 : NBUF * FR * 64];
  u32x4* const bring = lds + A_RING;  // FA: the weight ring follows the x ring

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 2, wc = w & 3;

  // XCD-aware bijective remap, then (split, M-grouped tile) order
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tiles = tiles_m * tiles_n;
  const int split = wgid / tiles;
  const int pid = wgid - split * tiles;
  int tm, tn;
  g2_tile_coords(pid, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;

  const int KS = K >> 5, NTT = N >> 4;
  const int ks0 = split * kc;
  const int KT = min(KS, ks0 + kc) - ks0;  // K-tiles (32 deep) of this split

  // per-wave LDS-DMA sources: fragment f = w + NW*j (A fragments first, then B)
  const char* src[G];
  int step[G];
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const int f = w + NW * j;
    if (f < AF) {
      const int row = min(m0 + 16 * f + (lane & 15), M - 1);
      src[j] = reinterpret_cast<const char*>(x + (size_t)row * K + (size_t)ks0 * 32 + 8 * (lane >> 4));
      step[j] = 64;
    } else {
      const int nt = min((n0 >> 4) + (f - AF), NTT - 1);
      src[j] = reinterpret_cast<const char*>(W + ((size_t)nt * KS + ks0) * 64 + lane);
      step[j] = 1024;
    }
  }
  auto issue = [&](int t) {
    u32x4* buf = lds + (t % NBUF) * FR * 64;
#pragma unroll
    for (int j = 0; j < G; ++j) glds16(src[j] + (size_t)t * step[j], buf + (w + NW * j) * 64);
  };
  // one half of a tile's loads (SUB = 2 issues a tile over two sub-phases)
  auto issue_half = [&](int t, int h) {
    u32x4* buf = lds + (t % NBUF) * FR * 64;
#pragma unroll
    for (int j = h * (G / 2); j < (h + 1) * (G / 2); ++j) glds16(src[j] + (size_t)t * step[j], buf + (w + NW * j) * 64);
  };
  // FA sources, saddr form: one wave-uniform 64-bit base per operand (advanced by scalar adds) plus a
  // 32-bit per-lane byte offset within the tile (< 15 MB for every Llama shape). x piece 16h + wu + 8j
  // of a K-tile pair (h = issue half, a compile-time constant at every call), weight fragments wu + 8j.
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const char* const baseA = reinterpret_cast<const char*>(x + (size_t)m0 * K + (size_t)ks0 * 32);
  const char* const baseB = reinterpret_cast<const char*>(W + ((size_t)(n0 >> 4) * KS + ks0) * 64);
  unsigned offA[2][2], offAt[2][2], offB[2];
  if constexpr (FA) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int P = 16 * h + wu + 8 * j;
        const int row = min(m0 + 8 * P + (lane >> 3), M - 1) - m0;
        const int c = (lane & 7) ^ ((P & 1) * 4 + (lane >> 4));  // the chunk stored at cell lane & 7
        offA[h][j] = (unsigned)row * (unsigned)K * 2u + 16u * (unsigned)c;
        // a pair whose second K-tile is past this split's range: re-read the first K-tile into the
        // unused cells (never past the end of a row)
        offAt[h][j] = offA[h][j] - (c >= 4 ? 64u : 0u);
      }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int nt = min((n0 >> 4) + wu + NW * j, NTT - 1) - (n0 >> 4);
      offB[j] = (unsigned)nt * (unsigned)KS * 1024u + 16u * (unsigned)lane;
    }
  }
  auto issueA1 = [&](int p, auto HC, int j) {  // x pair p (K-tiles 2p, 2p+1), half HC of its pieces
    constexpr int h = decltype(HC)::value;
    glds16(baseA + (size_t)p * 128 + (2 * p + 1 >= KT ? offAt[h][j] : offA[h][j]),
           lds + (p % A_SLOTS) * A_PIECES * 64 + (16 * h + wu + 8 * j) * 64);
  };
  auto issueA = [&](int p, auto HC) {
#pragma unroll
    for (int j = 0; j < 2; ++j) issueA1(p, HC, j);
  };
  auto issueB1 = [&](int t, int j) {
    glds16(baseB + (size_t)t * 1024 + offB[j], bring + (t % NBUF) * BF * 64 + (wu + NW * j) * 64);
  };
  auto issueB = [&](int t) {
#pragma unroll
    for (int j = 0; j < 2; ++j) issueB1(t, j);
  };

  f32x4 acc[MT][NTW];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss0 = 0.f, ss1 = 0.f;  // RMS: partial sums of squares of m-tiles RPW*wc (+1) (row lane & 15)
  // The two fragments are re-read from LDS (2 extra ds_read_b128): selecting them out of a[] by the
  // runtime wc makes hipcc move the fragment array to scratch.
  auto sumsq = [&](const u32x4* buf) {
    if constexpr (RMS) {
      const u32x4 f0 = buf[(wr * MT + RPW * wc) * 64 + lane];
      ss0 = dot8_bf16(f0, f0, ss0);
      if constexpr (RPW == 2) {
        const u32x4 f1 = buf[(wr * MT + RPW * wc + 1) * 64 + lane];
        ss1 = dot8_bf16(f1, f1, ss1);
      }
    }
  };

  if constexpr (FA) {
#pragma unroll
    for (int p = 0; p < 2; ++p)
      if (2 * p < KT) {
        issueA(p, std::integral_constant<int, 0>{});
        issueA(p, std::integral_constant<int, 1>{});
      }
#pragma unroll
    for (int t = 0; t < DIST; ++t)
      if (t < KT) issueB(t);
  } else {
#pragma unroll
    for (int t = 0; t < DIST; ++t)
      if (t < KT) issue(t);
  }

  if constexpr (WM == 2) {
    // Ping-pong: wave rows 0 and 1 (one wave of each per SIMD) run one barrier apart, so while
    // one group issues its LDS-DMA + ds_reads (L phase) the other keeps the SIMD's MFMA pipe busy
    // (M phase). Phase p of a wave: L_p = [issue tile p+3; wait own part of tile p+1; ds_read tile p;
    // lgkmcnt(0)] -> barrier -> M_p (32 MFMAs) -> barrier. Group 0's L_p sits between barrier
    // instances 2p and 2p+1, group 1's between 2p+1 and 2p+2, hence:
    //  RAW: every wave retires its part of tile t in L_{t-1}, before instance 2t; group 0 reads t
    //       after instance 2t, group 1 after 2t+1.
    //  WAR: tile t+3 refills tile t-1's slot in L_t; every wave's reads of t-1 completed
    //       (lgkmcnt(0)) in L_{t-1}, before instance 2t.
    // Both groups call 2*KT + 2 barriers (the stagger and the closing one are balanced).
    if (KT > 0) {
      wait_vmcnt<0>();  // tile 0 (and the rest of the prologue) landed; simple, once per WG
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#ifdef JLA_GEMM_STAMPS
    unsigned long long st_l = 0, st_b1 = 0, st_m = 0, st_b2 = 0, st_iss = 0, st_lds = 0, t0, t1;
#define JLA_STAMP(v)                                                                     \
  __builtin_amdgcn_sched_barrier(0);                                                     \
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");              \
  __builtin_amdgcn_sched_barrier(0);
#else
#define JLA_STAMP(v)
#endif
    if constexpr (SUB == 2) {
      // Barrier instances per K-tile t (group 0 / group 1 = one instance later): L0 | b | M0 | b | L1 | b | M1 | b.
      //  RAW: each wave waits for its part of tile t+1 in L1(t) (group 0 before instance 4t+3, group 1 before
      //       4t+4); tile t+1 is first read in L0(t+1), after instance 4t+4 (group 0) / 4t+5 (group 1).
      //  WAR: tile t+3 refills tile t-1's buffer from L0(t) on (after instance 4t); the last reads of t-1
      //       (group 1's L1(t-1)) retired with lgkmcnt(0) before its call of instance 4t.
      static_assert(MT % 2 == 0 && G % 2 == 0, "SUB=2 splits the m-tiles and the loads in halves");
      constexpr int MH = MT / 2;
      for (int t = 0; t < KT; ++t) {
        const u32x4* buf = lds + (t % NBUF) * FR * 64;
        u32x4 a[MT], b[NTW];
        // ---- L0: first half of tile t+3's loads; B fragments and the first half of A
        if (t + DIST < KT) issue_half(t + DIST, 0);
#pragma unroll
        for (int j = 0; j < NTW; ++j) b[j] = buf[(AF + wc * NTW + j) * 64 + lane];
#pragma unroll
        for (int i = 0; i < MH; ++i) a[i] = buf[(wr * MT + i) * 64 + lane];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < MH; ++i)
#pragma unroll
          for (int j = 0; j < NTW; ++j) acc[i][j] = mfma16x16x32(a[i], b[j], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        // ---- L1: second half of the loads; the rest of A; wait for this wave's part of tile t+1
        if (t + DIST < KT) issue_half(t + DIST, 1);
#pragma unroll
        for (int i = MH; i < MT; ++i) a[i] = buf[(wr * MT + i) * 64 + lane];
        sumsq(buf);
        {
          const int after = min(KT - 1, t + DIST) - (t + 1);  // tiles issued after t+1
          if (after >= 3)
            wait_vmcnt<3 * G>();
          else if (after == 2)
            wait_vmcnt<2 * G>();
          else if (after == 1)
            wait_vmcnt<G>();
          else
            wait_vmcnt<0>();
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = MH; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NTW; ++j) acc[i][j] = mfma16x16x32(a[i], b[j], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
    } else if constexpr (FA) {
      // FA main loop, unrolled by K-tile pairs so each step's x issue half (and its LDS read chunk) is a
      // compile-time constant. Same phase/barrier structure as the loop below.
      // vmcnt: every load of K-tile t+1 (its weights and both halves of its x pair) was issued at K-tile
      // t-2 or earlier (or in the drained prologue); this wave's issues of K-tiles t-1 and t may stay in
      // flight: 2 weight + 2 x loads per K-tile while there is something left to issue.
      // FAM (0..4): that many of a K-tile's 4 loads (weights first, then x) are issued from its M phase,
      // spread between the MFMAs, instead of at the head of its L phase (the stamps put the L phase --
      // issue + reads + wait -- above the M phase); at the wait of K-tile t only the L-phase part of
      // K-tile t's loads has been issued.
      constexpr int MB = FAM < 2 ? FAM : 2, MA = FAM - MB;  // moved weight / x loads
      auto fa_cnt = [&](int s, bool l_only) {
        return s < 0 ? 0
                     : (s + DIST < KT ? (l_only ? 2 - MB : 2) : 0) +
                           (2 * ((s >> 1) + 2) < KT ? (l_only ? 2 - MA : 2) : 0);
      };
      auto fa_step = [&](int t, auto HC) {
        constexpr int h = decltype(HC)::value;  // == t & 1
#ifdef JLA_GEMM_STAMPS
        unsigned long long t0, t1;
        JLA_STAMP(t0)
#endif
        const bool more_b = t + DIST < KT, more_a = 2 * ((t >> 1) + 2) < KT;
        if (more_b) {
#pragma unroll
          for (int j = 0; j < 2 - MB; ++j) issueB1(t + DIST, j);
        }
        if (more_a) {
#pragma unroll
          for (int j = 0; j < 2 - MA; ++j) issueA1((t >> 1) + 2, HC, j);
        }
#ifdef JLA_GEMM_STAMPS
        JLA_STAMP(t1) st_iss += t1 - t0; t0 = t1;
#endif
        // row r of the tile, chunk c of its 64-deep pair sits at u32x4 r * 8 + (c ^ ((r & 15) >> 1))
        const u32x4* abuf = lds + ((t >> 1) % A_SLOTS) * A_PIECES * 64;
        const u32x4* bbuf = bring + (t % NBUF) * BF * 64;
        const int ab = (wr * MT * 16 + (lane & 15)) * 8 + ((4 * h + (lane >> 4)) ^ ((lane >> 1) & 7));
        u32x4 a[MT], b[NTW];
#pragma unroll
        for (int j = 0; j < NTW; ++j) b[j] = bbuf[(wc * NTW + j) * 64 + lane];
#pragma unroll
        for (int i = 0; i < MT; ++i) a[i] = abuf[ab + i * 128];
        if constexpr (RMS) {
          const u32x4 f0 = abuf[ab + RPW * wc * 128];
          ss0 = dot8_bf16(f0, f0, ss0);
          if constexpr (RPW == 2) {
            const u32x4 f1 = abuf[ab + (RPW * wc + 1) * 128];
            ss1 = dot8_bf16(f1, f1, ss1);
          }
        }
#ifdef JLA_GEMM_STAMPS
        JLA_STAMP(t1) st_lds += t1 - t0; t0 = t1;
#endif
        if (t >= 1 && t + 4 < KT) {  // steady state: K-tiles t-1 and t issued 2 + 2 loads (t: its L part)
          wait_vmcnt<8 - FAM>();
        } else {
          const int n = fa_cnt(t - 1, false) + fa_cnt(t, true);
          if (n >= 8)
            wait_vmcnt<8>();
          else if (n == 7)
            wait_vmcnt<7>();
          else if (n == 6)
            wait_vmcnt<6>();
          else if (n == 5)
            wait_vmcnt<5>();
          else if (n == 4)
            wait_vmcnt<4>();
          else if (n == 3)
            wait_vmcnt<3>();
          else if (n == 2)
            wait_vmcnt<2>();
          else if (n == 1)
            wait_vmcnt<1>();
          else
            wait_vmcnt<0>();
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#ifdef JLA_GEMM_STAMPS
        JLA_STAMP(t1) st_l += t1 - t0; t0 = t1;
#endif
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
#ifdef JLA_GEMM_STAMPS
        JLA_STAMP(t1) st_b1 += t1 - t0; t0 = t1;
#endif
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < MT; ++i) {
#pragma unroll
          for (int j = 0; j < NTW; ++j) acc[i][j] = mfma16x16x32(a[i], b[j], acc[i][j]);
          // moved load m (0..FAM-1) goes after m-tile (2m + 1) * MT / (2 FAM): weights j = 2-MB.., then x
#pragma unroll
          for (int m = 0; m < FAM; ++m) {
            if (i == (2 * m + 1) * MT / (2 * FAM)) {
              if (m < MB) {
                if (more_b) {
                  __builtin_amdgcn_sched_barrier(0);
                  issueB1(t + DIST, 2 - MB + m);
                  __builtin_amdgcn_sched_barrier(0);
                }
              } else if (more_a) {
                __builtin_amdgcn_sched_barrier(0);
                issueA1((t >> 1) + 2, HC, 2 - MA + (m - MB));
                __builtin_amdgcn_sched_barrier(0);
              }
            }
          }
        }
        __builtin_amdgcn_s_setprio(0);
        asm volatile("" ::: "memory");
#ifdef JLA_GEMM_STAMPS
        JLA_STAMP(t1) st_m += t1 - t0; t0 = t1;
#endif
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
#ifdef JLA_GEMM_STAMPS
        JLA_STAMP(t1) st_b2 += t1 - t0;
#endif
      };
      for (int t = 0; t < KT; t += 2) {
        fa_step(t, std::integral_constant<int, 0>{});
        if (t + 1 < KT) fa_step(t + 1, std::integral_constant<int, 1>{});
      }
    } else
    for (int t = 0; t < KT; ++t) {
      JLA_STAMP(t0)
      if (t + DIST < KT) issue(t + DIST);
      const int after = min(KT - 1, t + DIST) - (t + 1);  // tiles issued after t+1
      auto wait_next = [&]() {
        if (after >= 3)
          wait_vmcnt<3 * G>();
        else if (after == 2)
          wait_vmcnt<2 * G>();
        else if (after == 1)
          wait_vmcnt<G>();
        else
          wait_vmcnt<0>();
      };
      if constexpr (!LATE_WAIT) wait_next();
#ifdef JLA_GEMM_STAMPS
      JLA_STAMP(t1) st_iss += t1 - t0; t0 = t1;
#endif
      const u32x4* buf = lds + (t % NBUF) * FR * 64;
      u32x4 a[MT], b[NTW];
#pragma unroll
      for (int j = 0; j < NTW; ++j) b[j] = buf[(AF + wc * NTW + j) * 64 + lane];
#pragma unroll
      for (int i = 0; i < MT; ++i) a[i] = buf[(wr * MT + i) * 64 + lane];
      sumsq(buf);
#ifdef JLA_GEMM_STAMPS
      JLA_STAMP(t1) st_lds += t1 - t0; t0 = t1;
#endif
      // LATE_WAIT: tile t+1 only has to land before this phase's barrier, not before tile t's reads
      if constexpr (LATE_WAIT) wait_next();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#ifdef JLA_GEMM_STAMPS
      JLA_STAMP(t1) st_l += t1 - t0; t0 = t1;
#endif
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
#ifdef JLA_GEMM_STAMPS
      JLA_STAMP(t1) st_b1 += t1 - t0; t0 = t1;
#endif
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTW; ++j) acc[i][j] = mfma16x16x32(a[i], b[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
      asm volatile("" ::: "memory");
#ifdef JLA_GEMM_STAMPS
      JLA_STAMP(t1) st_m += t1 - t0; t0 = t1;
#endif
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
#ifdef JLA_GEMM_STAMPS
      JLA_STAMP(t1) st_b2 += t1 - t0;
#endif
    }
    if (wr == 0) __builtin_amdgcn_s_barrier();
#ifdef JLA_GEMM_STAMPS
    if (lane == 0 && MODE == MODE_STORE) {
      unsigned long long* d = g_gemm_stamps + ((size_t)blockIdx.x * NW + w) * 6;
      d[0] = st_l;
      d[1] = st_b1;
      d[2] = st_m;
      d[3] = st_b2;
      d[4] = st_iss;
      d[5] = st_lds;
    }
#endif
  } else
  for (int t = 0; t < KT; ++t) {
    const int ahead = min(KT - 1 - t, DIST - 1);  // tiles issued after t
    if (ahead >= 3)
      wait_vmcnt<3 * G>();
    else if (ahead == 2)
      wait_vmcnt<2 * G>();
    else if (ahead == 1)
      wait_vmcnt<G>();
    else
      wait_vmcnt<0>();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + DIST < KT) issue(t + DIST);  // refills the buffer read at t-1 (retired by the barrier)
    const u32x4* buf = lds + (t % NBUF) * FR * 64;
    u32x4 a[MT], b[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) b[j] = buf[(AF + wc * NTW + j) * 64 + lane];
#pragma unroll
    for (int i = 0; i < MT; ++i) a[i] = buf[(wr * MT + i) * 64 + lane];
    sumsq(buf);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NTW; ++j) acc[i][j] = mfma16x16x32(a[i], b[j], acc[i][j]);
  }

  if constexpr (RMS) {
    // complete each row's sum over the 4 lanes that hold its k-chunks (lane >> 4)
    ss0 += __shfl_xor(ss0, 16, 64);
    ss0 += __shfl_xor(ss0, 32, 64);
    ss1 += __shfl_xor(ss1, 16, 64);
    ss1 += __shfl_xor(ss1, 32, 64);
  }
  if constexpr (RMS) {
    const int rA = m0 + (wr * MT + RPW * wc) * 16 + (lane & 15), rB = rA + 16;
    if constexpr (MODE == MODE_PARTIAL) {
      if (lane < 16) {
        if (rA < M) ssq_ws[(size_t)split * M + rA] = ss0;
        if (RPW == 2 && rB < M) ssq_ws[(size_t)split * M + rB] = ss1;
      }
    } else {
      // publish the row statistics through LDS (the tile buffers are free once every wave is past
      // its last ds_read), then scale every accumulator row
      float* rs = reinterpret_cast<float*>(lds);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __syncthreads();
      if (lane < 16) {
        // (t / K exactly as gemm_reduce_kernel: split and unsplit plans agree bit for bit)
        const float fk = (float)K;
        rs[(wr * MT + RPW * wc) * 16 + lane] = 1.f / sqrtf(ss0 / fk + rms_eps);
        if constexpr (RPW == 2) rs[(wr * MT + RPW * wc + 1) * 16 + lane] = 1.f / sqrtf(ss1 / fk + rms_eps);
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float sc = rs[(wr * MT + i) * 16 + 4 * (lane >> 4) + r];
#pragma unroll
          for (int j = 0; j < NTW; ++j) acc[i][j][r] *= sc;
        }
    }
  }

  const int c = lane & 15;
  if constexpr (MODE == MODE_SWIGLU) {
    const int F = N >> 1;
    bf16_t* o = static_cast<bf16_t*>(out);
#pragma unroll
    for (int j = 0; j < NTW; j += 2) {
      const int gtile = (n0 >> 4) + wc * NTW + j;  // even: gate tile, gtile + 1: its up tile
      if (gtile >= NTT) continue;
      const int col = (gtile >> 1) * 16 + c;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + (wr * MT + i) * 16 + 4 * (lane >> 4) + r;
          if (row < M) o[(size_t)row * F + col] = f2bf(silu(acc[i][j][r]) * acc[i][j + 1][r]);
        }
    }
  } else if constexpr (MODE == MODE_ARGMAX) {
    // greedy lm_head: the logits never leave the registers. Per row, the first maximum over this
    // wave's 64 columns (lane: its 4 columns in ascending order, strict >; then the 16 lanes of the
    // row, ties to the smaller index) -> one (value, index) partial at [row][n0 / 64 + wc] of `out`;
    // argmax_partials_kernel finishes the row (same result as argmax over the stored fp32 logits).
    float2* o = static_cast<float2*>(out);
    const int P = tiles_n * (BN / (16 * NTW)), slot = (n0 >> 6) + wc;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float bv = -INFINITY;
        int bi = 0x7fffffff;
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
          const int tile = (n0 >> 4) + wc * NTW + j;
          const float v = acc[i][j][r];
          if (tile < NTT && v > bv) {
            bv = v;
            bi = tile * 16 + c;
          }
        }
#pragma unroll
        for (int sh = 1; sh < 16; sh <<= 1) {
          const float ov = __shfl_xor(bv, sh, 64);
          const int oi = __shfl_xor(bi, sh, 64);
          if (ov > bv || (ov == bv && oi < bi)) {
            bv = ov;
            bi = oi;
          }
        }
        const int row = m0 + (wr * MT + i) * 16 + 4 * (lane >> 4) + r;
        if (c == 0 && row < M) o[(size_t)row * P + slot] = make_float2(bv, __int_as_float(bi));
      }
  } else if constexpr (MODE == MODE_QKV) {
    // fused qkv projection without a K split (decode B = 2048, prefill): the (norm-scaled) accumulators are staged
    // through LDS one wave row (128 x 256 fp32) at a time, then every thread takes 4 consecutive columns of a row --
    // two RoPE pairs -- rotates the q / k heads and writes q, or the k / v cache row at slot[0] + (position in the
    // sequence), 8 bytes per store; replaces the bf16 store + rope_kv_kernel round trip (same arithmetic as
    // gemm_reduce_kernel<MODE_QKV>; reference model.py:58-92, :169-199)
    static_assert(WM == 2 && MT == 8 && NTW == 4, "QKV epilogue: 256 x 256 tiles");
    float* ep = reinterpret_cast<float*>(lds);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();  // every wave is past its last read of the tile buffers
#pragma unroll 1
    for (int half = 0; half < 2; ++half) {
      if (wr == half) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NTW; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = i * 16 + 4 * (lane >> 4) + r;
              const int col = ((wc * NTW + j) * 16 + c) ^ (((row >> 2) & 3) << 4);
              ep[row * BN + col] = acc[i][j][r];
            }
      }
      __syncthreads();
#pragma unroll 2
      for (int qq = 0; qq < 16; ++qq) {
        const int e = threadIdx.x + 512 * qq;
        const int row = e >> 6, c4 = (e & 63) * 4;
        const int grow = m0 + half * 128 + row, gcol = n0 + c4;
        const float4 v = *reinterpret_cast<const float4*>(ep + row * BN + (c4 ^ (((row >> 2) & 3) << 4)));
        if (grow >= M || gcol >= N) continue;
        float v0 = v.x, v1 = v.y, v2 = v.z, v3 = v.w;
        const int head = gcol / qa.Dh, d0 = gcol - head * qa.Dh;
        const int b = grow / qa.S, sq = grow - b * qa.S;
        if (head < qa.H + qa.Hkv) {
          int pos = qa.positions[grow];
          if (pos < 0 || pos >= qa.table_len) JLA_FLAG(JLA_BOUNDS_ROPE_POS);
          pos = pos < 0 ? 0 : (pos >= qa.table_len ? qa.table_len - 1 : pos);
          const float4 cs = *reinterpret_cast<const float4*>(qa.table + (size_t)pos * (qa.Dh >> 1) + (d0 >> 1));
          const float r0 = v0 * cs.x - v1 * cs.y, r1 = v0 * cs.y + v1 * cs.x;
          const float r2 = v2 * cs.z - v3 * cs.w, r3 = v2 * cs.w + v3 * cs.z;
          v0 = r0;
          v1 = r1;
          v2 = r2;
          v3 = r3;
        }
        const uint2 packed = make_uint2(pack2bf(v0, v1), pack2bf(v2, v3));
        if (head < qa.H) {
          *reinterpret_cast<uint2*>(qa.q + ((size_t)grow * qa.H + head) * qa.Dh + d0) = packed;
        } else {
          const int cslot = qa.slot[0] + sq;
          if (cslot < qa.T) {
            const bool is_k = head < qa.H + qa.Hkv;
            const int kh = is_k ? head - qa.H : head - qa.H - qa.Hkv;
            bf16_t* cache = is_k ? qa.kc : qa.vc;
            *reinterpret_cast<uint2*>(cache + (((size_t)b * qa.Hkv + kh) * qa.T + cslot) * qa.Dh + d0) = packed;
          } else {
            JLA_FLAG(JLA_BOUNDS_KV_SLOT);
          }
        }
      }
      __syncthreads();  // the half-tile is consumed before the other wave row overwrites it
    }
  } else {
    // rows outer, n-tiles inner: a row's adjacent 64-byte pieces back to back (as gemm4's fp32 epilogue; 2-4 % on the
    // split qkv / gate_up slabs and the residual o, profiles/r6_g2_epilogue_order_ab.jsonl); residual: the m-tile's h
    // values loaded before any is used (one round trip per m-tile, not per value)
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      float hv[4][NTW];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < NTW; ++j) hv[r][j] = 0.f;
      if constexpr (MODE == MODE_RESIDUAL) {
        if (accumulate) {  // (unconditional loads at clamped addresses: no per-load branch and join wait)
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < NTW; ++j) {
              const int tile = min((n0 >> 4) + wc * NTW + j, NTT - 1);
              const int row = min(m0 + (wr * MT + i) * 16 + 4 * (lane >> 4) + r, M - 1);
              hv[r][j] = static_cast<const float*>(out)[(size_t)row * N + tile * 16 + c];
            }
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
          const int tile = (n0 >> 4) + wc * NTW + j;
          const int row = m0 + (wr * MT + i) * 16 + 4 * (lane >> 4) + r;
          if (tile >= NTT || row >= M) continue;
          const size_t idx = (size_t)row * N + tile * 16 + c;
          const float v = acc[i][j][r];
          if constexpr (MODE == MODE_PARTIAL) {
            static_cast<float*>(out)[(size_t)split * M * N + idx] = v;
          } else if constexpr (MODE == MODE_RESIDUAL) {
            const float nv = hv[r][j] + v;
            static_cast<float*>(out)[idx] = nv;
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


// ---------------------------------------------------------------------------------------------
// gemm4: the 4-wave 256 x 256 main loop of gemm4w.h (one wave per SIMD, 128 x 128 per wave, 64-deep K-tiles)
// with every epilogue of gemm2. The accumulators are C^T fragments: lane (c = lane & 15, q = lane >> 4) holds,
// per (n-tile j, m-tile i) of its wave block, output row m0 + wr*128 + 16i + c at the 4 consecutive columns
// n0 + wc*128 + 16j + 4q + 0..3 -- so SwiGLU gate/up pairs (adjacent n-tiles), RoPE pairs (adjacent columns) and
// the fp32 residual (one float4) are all in-lane, and every store is 8 or 16 bytes. Split-K: MODE_PARTIAL slabs
// [split][M][N] (+ the fused-RMS partial sums [split][M]) summed by gemm_reduce_kernel, as gemm2's.
// RMSM (fused RMSNorm statistic): 0 none; 1 summed inside the main loop from the x fragments (split-K partial
// slabs: per-split sums to ssq_ws); 2 read from rms_inv[M], computed ahead of the GEMM by rms_rowinv_kernel.
// The epilogue of one gemm4 output tile (every mode; see gemm4_kernel), shared by the data-parallel and the
// stream-K launches. acc: this wave's finished C^T accumulators; ss: the in-loop RMS partial sums (RMSM 1).
struct G4Epi {
  void* out;
  int M, N, K, accumulate, out_f32;
  bf16_t* mirror;
  int tiles_n;
  float rms_eps;
  float* ssq_ws;
  const float* rms_inv;
};
template <int MODE, int RMSM, typename Acc, int NJ = 8>
JLA_DEV void g4_epilogue(Acc& acc, float* ss, u32x4* lds, int wu, int lane, int m0, int n0, int split,
                         const G4Epi& ep, const QKVArgs& qa) {
  constexpr bool RMS = RMSM == 1;
  static_assert(NJ == 8 || (RMSM != 1 && MODE != MODE_ARGMAX),
                "the 256 x 128 / 192 tiles: precomputed norm statistic; no argmax epilogue");
  constexpr int WN = 16 * NJ;  // output columns of a wave block
  constexpr int PJ = NJ == 6 ? 8 : NJ;  // staged row width in n-tiles (a power of two; NJ = 6 leaves the rest unused)
  const int wr = wu >> 1, wc = wu & 1;
  void* const out = ep.out;
  const int M = ep.M, N = ep.N, K = ep.K, accumulate = ep.accumulate, out_f32 = ep.out_f32;
  bf16_t* const mirror = ep.mirror;
  const int tiles_n = ep.tiles_n;
  const float rms_eps = ep.rms_eps;
  float* const ssq_ws = ep.ssq_ws;
  const float* const rms_inv = ep.rms_inv;
  (void)K, (void)tiles_n, (void)rms_eps, (void)ssq_ws, (void)rms_inv, (void)split, (void)accumulate, (void)out_f32,
      (void)mirror, (void)wc;
  const int c = lane & 15, q = lane >> 4, NTT = N >> 4;
  const int rbase = m0 + wr * 128 + c;  // + 16 i: this lane's output row in m-tile i
  float sc[8];                           // RMS: per m-tile row scale
  if constexpr (RMSM == 2) {
#pragma unroll
    for (int i = 0; i < 8; ++i) sc[i] = rms_inv[min(rbase + 16 * i, M - 1)];
  }
  if constexpr (RMS) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // complete each row's sum over the 4 lanes holding its k-chunks
      ss[i] += __shfl_xor(ss[i], 16, 64);
      ss[i] += __shfl_xor(ss[i], 32, 64);
    }
    if constexpr (MODE == MODE_PARTIAL) {
      if (q == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + wr * 128 + (4 * wc + i) * 16 + c;
          if (row < M) ssq_ws[(size_t)split * M + row] = ss[i];
        }
      }
    } else {
      float* rs = reinterpret_cast<float*>(lds + 8192);  // beside the 128 KiB staging space
      __syncthreads();  // every wave is past its last fragment read
      if (q == 0) {
        const float fk = (float)K;  // (t / K exactly as gemm_reduce_kernel and gemm2)
#pragma unroll
        for (int i = 0; i < 4; ++i) rs[wr * 128 + (4 * wc + i) * 16 + c] = 1.f / sqrtf(ss[i] / fk + rms_eps);
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 8; ++i) sc[i] = rs[wr * 128 + 16 * i + c];
    }
  }
  // one accumulator tile at a time, scaled by its row's norm: g4_take keeps hipcc from copying all 256 AGPRs to
  // VGPRs at once (which spilled)
  auto tile_val = [&](int j, int i) -> f32x4 {
    f32x4 v = g4_take(acc[j][i]);
    if constexpr (RMSM != 0 && MODE != MODE_PARTIAL) v *= sc[i];
    return v;
  };

  // bf16 outputs go through the wave's 32 KiB of LDS (g4_stage_put / g4_stage_rows); every wave must be past its
  // last fragment read first (the RMS path above already synchronised)
  char* const wl = reinterpret_cast<char*>(lds) + wu * 32768;
  constexpr bool STAGED = MODE == MODE_SWIGLU || MODE == MODE_QKV || MODE == MODE_STORE;
  if constexpr (STAGED && !(RMS && MODE != MODE_PARTIAL)) __syncthreads();
  const int mrow0 = m0 + wr * 128;  // first output row of the wave block
  if constexpr (MODE == MODE_SWIGLU) {
    // gate tile j (even) and up tile j + 1 -> 16 activation columns; the wave block's 64 columns = 128-byte rows
    const int F = N >> 1;
    bf16_t* o = static_cast<bf16_t*>(out);
#pragma unroll
    for (int j = 0; j < NJ; j += 2) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const f32x4 gv = tile_val(j, i), uv = tile_val(j + 1, i);
        const u32x2 p = {pack2bf(silu(gv[0]) * uv[0], silu(gv[1]) * uv[1]),
                         pack2bf(silu(gv[2]) * uv[2], silu(gv[3]) * uv[3])};
        g4_stage_put<16 * PJ>(wl, 16 * i + c, 16 * j + 8 * q, p);
      }
    }
    const int fcol0 = ((n0 >> 4) + wc * NJ) * 8;  // first activation column of the wave block
    g4_stage_rows<16 * PJ>(wl, lane, [&](int r, int ch, u32x4 v) {
      const int row = mrow0 + r, col = fcol0 + 8 * ch;
      if (row < M && col < F && ch < NJ) *reinterpret_cast<u32x4*>(o + (size_t)row * F + col) = v;
    });
  } else if constexpr (MODE == MODE_ARGMAX) {
    // per row: the first maximum over this wave's 128 columns -> one (value, index) partial at
    // [row][n0 / 128 + wc] (P = 2 tiles_n slots per row); argmax_partials_kernel finishes the row
    float2* o = static_cast<float2*>(out);
    const int P = tiles_n * 2, slot = (n0 >> 7) + wc;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int tile = (n0 >> 4) + wc * 8 + j;
        const f32x4 tv = tile_val(j, i);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = tv[r];
          if (tile < NTT && v > bv) {  // ascending columns in-lane, strict >: the first max
            bv = v;
            bi = tile * 16 + 4 * q + r;
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
      const int row = rbase + 16 * i;
      if (q == 0 && row < M) o[(size_t)row * P + slot] = make_float2(bv, __int_as_float(bi));
    }
  } else if constexpr (MODE == MODE_QKV) {
    // RoPE on the two (even, odd) pairs of the lane's 4 columns in fp32, then staged: 16-byte pieces of a row go to
    // q or to the k / v cache row at slot[0] + (position in the sequence); same arithmetic as gemm2's /
    // gemm_reduce_kernel's QKV epilogue (reference model.py:58-92, :169-199)
    // the positions of this lane's 8 rows, then per n-tile the 8 rows' RoPE factors, each batch loaded before any
    // value is used (loaded where used, behind the staged stores, they went one memory round trip at a time)
    int posr[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) posr[i] = qa.positions[min(rbase + 16 * i, M - 1)];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (posr[i] < 0 || posr[i] >= qa.table_len) JLA_FLAG(JLA_BOUNDS_ROPE_POS);
      posr[i] = posr[i] < 0 ? 0 : (posr[i] >= qa.table_len ? qa.table_len - 1 : posr[i]);
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int gcol = n0 + wc * WN + 16 * j + 4 * q;
      const int head = gcol / qa.Dh, d0 = gcol - head * qa.Dh;
      float4 cs[8];  // (loaded for every head; used for q and k)
#pragma unroll
      for (int i = 0; i < 8; ++i)
        cs[i] = *reinterpret_cast<const float4*>(qa.table + (size_t)posr[i] * (qa.Dh >> 1) + (d0 >> 1));
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const f32x4 tv = tile_val(j, i);
        float v0 = tv[0], v1 = tv[1], v2 = tv[2], v3 = tv[3];
        if (head < qa.H + qa.Hkv) {
          const float r0 = v0 * cs[i].x - v1 * cs[i].y, r1 = v0 * cs[i].y + v1 * cs[i].x;
          const float r2 = v2 * cs[i].z - v3 * cs[i].w, r3 = v2 * cs[i].w + v3 * cs[i].z;
          v0 = r0;
          v1 = r1;
          v2 = r2;
          v3 = r3;
        }
        g4_stage_put<256>(wl, 16 * i + c, 32 * j + 8 * q, u32x2{pack2bf(v0, v1), pack2bf(v2, v3)});
      }
    }
    g4_stage_rows<256>(wl, lane, [&](int r, int ch, u32x4 v) {
      const int grow = mrow0 + r, gcol = n0 + wc * WN + 8 * ch;
      if (grow >= M || gcol >= N || 8 * ch >= WN) return;
      const int head = gcol / qa.Dh, d0 = gcol - head * qa.Dh;
      if (head < qa.H) {
        *reinterpret_cast<u32x4*>(qa.q + ((size_t)grow * qa.H + head) * qa.Dh + d0) = v;
      } else {
        const int b = grow / qa.S, sq = grow - b * qa.S;
        const int cslot = qa.slot[0] + sq;
        if (cslot < qa.T) {
          const bool is_k = head < qa.H + qa.Hkv;
          const int kh = is_k ? head - qa.H : head - qa.H - qa.Hkv;
          bf16_t* cache = is_k ? qa.kc : qa.vc;
          *reinterpret_cast<u32x4*>(cache + (((size_t)b * qa.Hkv + kh) * qa.T + cslot) * qa.Dh + d0) = v;
        } else {
          JLA_FLAG(JLA_BOUNDS_KV_SLOT);
        }
      }
    });
  } else if constexpr (MODE == MODE_STORE) {
    if (out_f32) {  // fp32 logits (16-byte pieces, direct)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int tile = (n0 >> 4) + wc * NJ + j;
        if (tile >= NTT) continue;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int row = rbase + 16 * i;
          const f32x4 v = tile_val(j, i);
          if (row < M) *reinterpret_cast<f32x4*>(static_cast<float*>(out) + (size_t)row * N + tile * 16 + 4 * q) = v;
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const f32x4 v = tile_val(j, i);
          g4_stage_put<32 * PJ>(wl, 16 * i + c, 32 * j + 8 * q, u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])});
        }
      bf16_t* o = static_cast<bf16_t*>(out);
      g4_stage_rows<32 * PJ>(wl, lane, [&](int r, int ch, u32x4 v) {
        const int row = mrow0 + r, col = n0 + wc * WN + 8 * ch;
        if (row < M && col < N && 8 * ch < WN) *reinterpret_cast<u32x4*>(o + (size_t)row * N + col) = v;
      });
    }
  } else {  // PARTIAL / RESIDUAL: fp32, one 16-byte piece per lane per tile
    // rows outer, tiles inner: consecutive instructions take the two 64-byte halves of each 128-byte line of h (and the
    // adjacent 32-byte pieces of the mirror's line) back to back -- 4-7 % faster than tiles outer on the o projection,
    // 1.5-3.5 % on down, M = 4096 and 32768 (profiles/r6_g4_epilogue_order_ab.jsonl)
    // residual: a row's h pieces of every tile are loaded before any is used -- with the stores in between (which may
    // alias h as far as hipcc knows) the loads were issued one at a time, a full memory round trip per 16-byte piece
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = rbase + 16 * i;
      f32x4 hv[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) hv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (MODE == MODE_RESIDUAL) {
        if (accumulate) {  // (unconditional loads at clamped addresses: a per-load branch made hipcc wait at each join)
          const float* hrow = static_cast<const float*>(out) + (size_t)min(row, M - 1) * N + 4 * q;
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            hv[j] = *reinterpret_cast<const f32x4*>(hrow + min((n0 >> 4) + wc * NJ + j, NTT - 1) * 16);
        }
      }
      // every result of the row first, then the stores (a store between two uses made hipcc wait for the store too)
#pragma unroll
      for (int j = 0; j < NJ; ++j) hv[j] += tile_val(j, i);  // (accumulate 0 / partial: hv is zero, 0 + v = v exactly)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int tile = (n0 >> 4) + wc * NJ + j;
        if (tile >= NTT || row >= M) continue;
        const size_t idx = (size_t)row * N + tile * 16 + 4 * q;
        if constexpr (MODE == MODE_PARTIAL) {
          *reinterpret_cast<f32x4*>(static_cast<float*>(out) + (size_t)split * M * N + idx) = hv[j];
        } else {
          *reinterpret_cast<f32x4*>(static_cast<float*>(out) + idx) = hv[j];
          if (mirror)
            *reinterpret_cast<u32x2*>(mirror + idx) = u32x2{pack2bf(hv[j][0], hv[j][1]), pack2bf(hv[j][2], hv[j][3])};
        }
      }
    }
  }
}

template <int MODE, int RMSM, int NJ = 8, int DIAG = 0, bool W3 = false>
__global__ void __launch_bounds__(256, 1)
    gemm4_kernel(const bf16_t* __restrict__ x, const u32x4* __restrict__ W, void* __restrict__ out, int M, int N,
                 int K, int accumulate, int out_f32, bf16_t* __restrict__ mirror, int kc, int tiles_m, int tiles_n,
                 float rms_eps, float* __restrict__ ssq_ws, QKVArgs qa, const float* __restrict__ rms_inv,
                 int group_m) {
  constexpr bool RMS = RMSM == 1;
  // the two K-tile slots (W3: two x + three W slots, all 160 KiB); after the loop: the epilogue's staging (128 KiB)
  // + 1 KiB of row scales
  __shared__ u32x4 lds[W3 ? 2 * G4_A_U4 + 3 * G4_B_U4 : 2 * G4_SLOT_U4 + 64];
  const int lane = threadIdx.x & 63;
  const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wu >> 1, wc = wu & 1;
  // XCD-aware bijective remap, then (split, M-grouped tile) order (as gemm2)
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tiles = tiles_m * tiles_n;
  const int split = wgid / tiles, pid = wgid - split * tiles;
  int tm, tn;
  g4_tile_coords(pid, tiles_m, tiles_n, tm, tn, group_m);
  const int m0 = tm * G4_BM, n0 = tn * (32 * NJ);
  const int t0 = split * kc, KT = min(K >> 6, t0 + kc) - t0;

  f32x4 acc[NJ][8];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[4] = {0.f, 0.f, 0.f, 0.f};
  const G4Args g{x, W, out, M, N, K, kc, tiles_m, tiles_n};
  if constexpr (NJ != 8) {
    static_assert(!RMS, "the 256 x 128 tile: precomputed statistic");
    g4n_mainloop<NJ, decltype(acc), W3>(g, lds, m0, n0, t0, KT, wu, lane, acc);
  } else {
    g4_mainloop<RMS, decltype(acc), DIAG, W3>(g, lds, m0, n0, t0, KT, wu, lane, acc, ss);
  }
  g4_epilogue<MODE, RMSM, decltype(acc), NJ>(
      acc, ss, lds, wu, lane, m0, n0, split,
      G4Epi{out, M, N, K, accumulate, out_f32, mirror, tiles_n, rms_eps, ssq_ws, rms_inv}, qa);
}

// Persistent gemm4 (tile config 13): one workgroup per CU walks the launch order round by round (tile wg, wg + CUs,
// ...), so a CU's next tile starts without a workgroup teardown and relaunch, and the CUs drift apart over the rounds:
// their epilogues (the residual's fp32 read-modify-write above all) stop arriving at HBM as one chip-wide burst.
template <int MODE, int RMSM>
__global__ void __launch_bounds__(256, 1)
    gemm4p_kernel(const bf16_t* __restrict__ x, const u32x4* __restrict__ W, void* __restrict__ out, int M, int N,
                  int K, int accumulate, int out_f32, bf16_t* __restrict__ mirror, int tiles_m, int tiles_n,
                  float rms_eps, QKVArgs qa, const float* __restrict__ rms_inv, int group_m) {
  constexpr bool RMS = RMSM == 1;
  __shared__ u32x4 lds[2 * G4_SLOT_U4 + 64];
  const int lane0 = threadIdx.x & 63;
  const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tiles = tiles_m * tiles_n;
  const G4Args g{x, W, out, M, N, K, K >> 6, tiles_m, tiles_n};
  const G4Epi ep{out, M, N, K, accumulate, out_f32, mirror, tiles_n, rms_eps, nullptr, rms_inv};
  for (int pid = wg; pid < tiles; pid += nwg) {
    int tm, tn;
    g4_tile_coords(pid, tiles_m, tiles_n, tm, tn, group_m);
    const int m0 = tm * G4_BM, n0 = tn * G4_BN;
    // the lane index laundered once per tile: the lane-dependent address math of the main loop and the unrolled
    // epilogue would otherwise be hoisted out of the tile loop and kept live (spills)
    int lane;
    asm volatile("v_mov_b32 %0, %1" : "=v"(lane) : "v"(lane0));
    f32x4 acc[8][8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float ss[4] = {0.f, 0.f, 0.f, 0.f};
    g4_mainloop<RMS>(g, lds, m0, n0, 0, K >> 6, wu, lane, acc, ss);
    g4_epilogue<MODE, RMSM>(acc, ss, lds, wu, lane, m0, n0, 0, ep, qa);
    __syncthreads();  // the epilogue's staging / row scales are done with LDS before the next tile's DMA
  }
}

// Sum of the ksplit fp32 slabs at float4 e4 in split order: the loads of up to 8 splits are issued before the first
// add (the round-4 loop waited on each split in turn: 12 dependent L2/HBM round trips for the 70B shard's qkv at M =
// 256, 9 us for 1.3 MB of output). Same addition order as before, so bit for bit the same sums.
__device__ __forceinline__ float4 sum_splits(const float* __restrict__ ws, int ksplit, size_t slab4, size_t e4) {
  const float4* p = reinterpret_cast<const float4*>(ws) + e4;
  float4 v = p[0];
  for (int s0 = 1; s0 < ksplit; s0 += 8) {
    float4 q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (s0 + j < ksplit) q[j] = p[(size_t)(s0 + j) * slab4];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (s0 + j < ksplit) {
        v.x += q[j].x;
        v.y += q[j].y;
        v.z += q[j].z;
        v.w += q[j].w;
      }
  }
  return v;
}

// Sum the split-K partials (fixed order) and apply the epilogue. One thread = 4 consecutive columns of one row (two
// RoPE pairs; a 16-column tile never straddles a float4); SwiGLU: 4 consecutive output columns, i.e. the gate float4
// and the up float4 16 columns to its right (the launch covers M * N / 8 threads there).
template <int MODE>
__global__ void __launch_bounds__(256)
    gemm_reduce_kernel(const float* __restrict__ ws, int ksplit, void* __restrict__ out, int M, int N,
                       int accumulate, int out_f32, bf16_t* __restrict__ mirror, QKVArgs qa,
                       const float* __restrict__ ssq, int K, float rms_eps) {
  const size_t t4 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t slab4 = (size_t)M * N / 4;
  if (t4 >= (MODE == MODE_SWIGLU ? slab4 >> 1 : slab4)) return;
  size_t e4 = t4;
  if constexpr (MODE == MODE_SWIGLU) {  // output float4 t4 -> the gate float4 of its 32-column (gate, up) tile pair
    const size_t oq = (size_t)N >> 3, mo = t4 / oq, c = (t4 - mo * oq) * 4;
    e4 = (mo * N + (c >> 4) * 32 + (c & 15)) >> 2;
  }
  const size_t idx = e4 * 4;
  const int m = (int)(idx / N), col = (int)(idx - (size_t)m * N);
  float4 v = sum_splits(ws, ksplit, slab4, e4);
  float rs = 1.f;  // fused RMSNorm: the splits' partial sums of squares of row m (fixed order)
  if (ssq) {
    float t = 0.f;
    for (int s = 0; s < ksplit; ++s) t += ssq[(size_t)s * M + m];
    rs = 1.f / sqrtf(t / (float)K + rms_eps);
    v.x *= rs;
    v.y *= rs;
    v.z *= rs;
    v.w *= rs;
  }
  float vv[4] = {v.x, v.y, v.z, v.w};
  if constexpr (MODE == MODE_SWIGLU) {
    // gate tile t = 2p holds columns [32p, 32p+16), the up tile the next 16: pair the two halves
    const int tile = col >> 4, c0 = col & 15;  // tile is even: the gate half of the pair
    float4 u = sum_splits(ws, ksplit, slab4, e4 + 4);
    u.x *= rs;
    u.y *= rs;
    u.z *= rs;
    u.w *= rs;
    const float uu[4] = {u.x, u.y, u.z, u.w};
    bf16_t* o = static_cast<bf16_t*>(out) + (size_t)m * (N >> 1) + (tile >> 1) * 16 + c0;
    const uint2 pk = make_uint2(pack2bf(silu(vv[0]) * uu[0], silu(vv[1]) * uu[1]),
                                pack2bf(silu(vv[2]) * uu[2], silu(vv[3]) * uu[3]));
    *reinterpret_cast<uint2*>(o) = pk;
    // decode M: also the packed copy (common.h pack_off) the next projection's packed-x GEMV reads
    if (qa.pack) *reinterpret_cast<uint2*>(qa.pack + pack_off(m, (tile >> 1) * 16 + c0, N >> 1)) = pk;
  } else if constexpr (MODE == MODE_RESIDUAL) {
    float4* o = reinterpret_cast<float4*>(static_cast<float*>(out) + idx);
    float4 r = *o;
    if (accumulate) {
      r.x += vv[0];
      r.y += vv[1];
      r.z += vv[2];
      r.w += vv[3];
    } else {
      r = make_float4(vv[0], vv[1], vv[2], vv[3]);
    }
    *o = r;
    if (mirror) {
      const uint2 pk = make_uint2(pack2bf(r.x, r.y), pack2bf(r.z, r.w));
      *reinterpret_cast<uint2*>(mirror + idx) = pk;
      if (qa.pack) *reinterpret_cast<uint2*>(qa.pack + pack_off(m, col, N)) = pk;  // packed copy of the mirror
    }
  } else if constexpr (MODE == MODE_QKV) {
    const int head = col / qa.Dh, d0 = col - head * qa.Dh;
    const int b = m / qa.S, sq = m - b * qa.S;
    if (head < qa.H + qa.Hkv) {
      int pos = qa.positions[m];
      if (pos < 0 || pos >= qa.table_len) JLA_FLAG(JLA_BOUNDS_ROPE_POS);
      pos = pos < 0 ? 0 : (pos >= qa.table_len ? qa.table_len - 1 : pos);
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const float2 cs = qa.table[(size_t)pos * (qa.Dh >> 1) + (d0 >> 1) + p];
        const float xr = vv[2 * p], xi = vv[2 * p + 1];
        vv[2 * p] = xr * cs.x - xi * cs.y;
        vv[2 * p + 1] = xr * cs.y + xi * cs.x;
      }
    }
    const uint2 packed = make_uint2(pack2bf(vv[0], vv[1]), pack2bf(vv[2], vv[3]));
    if (head < qa.H) {
      *reinterpret_cast<uint2*>(qa.q + ((size_t)m * qa.H + head) * qa.Dh + d0) = packed;
    } else {
      const int slot = qa.slot[0] + sq;
      if (slot < qa.T) {
        const bool is_k = head < qa.H + qa.Hkv;
        const int kh = is_k ? head - qa.H : head - qa.H - qa.Hkv;
        bf16_t* cache = is_k ? qa.kc : qa.vc;
        *reinterpret_cast<uint2*>(cache + (((size_t)b * qa.Hkv + kh) * qa.T + slot) * qa.Dh + d0) = packed;
      } else {
        JLA_FLAG(JLA_BOUNDS_KV_SLOT);
      }
    }
  } else {
    if (out_f32)
      *reinterpret_cast<float4*>(static_cast<float*>(out) + idx) = make_float4(vv[0], vv[1], vv[2], vv[3]);
    else
      *reinterpret_cast<uint2*>(static_cast<bf16_t*>(out) + idx) =
          make_uint2(pack2bf(vv[0], vv[1]), pack2bf(vv[2], vv[3]));
  }
}

// Split-K reduce of a row-parallel projection with the tensor-parallel all-reduce and the residual add in its epilogue
// (MODE_TPRESID: the tiled GEMM's counterpart of gemv.hip's fused epilogue, for decode batches past the GEMV's 64 rows;
// reference partition.py:67,70 -- the psum of the row-sharded wo / w2). Workgroup w sums the splits of elements
// [4096 w, 4096 (w + 1)) of the M x N output, rounds each pair to bf16 (the partial the unfused reduce stores) and
// pushes it as {2 x bf16, tag} granules into region w of every rank's buffer -- the GEMV workgroup w's TPRES_REGION and
// call counter, so every call that touches region w is ordered by one counter and allreduce.hip's parity argument
// holds -- then gathers the ranks' granules from its own buffer, sums them in rank order in fp32 and adds into h (and
// the bf16 mirror). Bit-identical to the bf16 partial + car_reduce_kernel; one launch and one HBM round trip of the
// partial fewer.
constexpr int TPR_ELEMS = 4096;  // elements per workgroup: 2048 granules of 8 bytes = one TPRES_REGION
static_assert(TPR_ELEMS / 2 * 8 == TPRES_REGION, "one fused-exchange region per workgroup");
__global__ void __launch_bounds__(256)
    gemm_reduce_tp_kernel(const float* __restrict__ ws, int ksplit, float* __restrict__ h, bf16_t* __restrict__ hb,
                          int M, int N, const CarDevice* __restrict__ dev) {
  const CarDevice& d = *dev;  // by reference (a by-value copy indexed with runtime p would live in scratch)
  const int w = blockIdx.x;
  const size_t slab4 = (size_t)M * N / 4;
  __shared__ int s_calls;
  if (threadIdx.x == 0) s_calls = __hip_atomic_load(d.wg_ctr + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  // this thread's 4 float4 groups (coalesced: group j covers threads' consecutive float4s); h loaded now, its round trip
  // behind the exchange
  u32x2 gq[4];
  f32x4 hv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const size_t e4 = (size_t)w * (TPR_ELEMS / 4) + j * 256 + threadIdx.x;
    gq[j] = u32x2{0u, 0u};
    hv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (e4 < slab4) {
      const float4 v = sum_splits(ws, ksplit, slab4, e4);
      gq[j] = u32x2{pack2bf(v.x, v.y), pack2bf(v.z, v.w)};
      hv[j] = *reinterpret_cast<const f32x4*>(h + e4 * 4);
    }
  }
  __syncthreads();
  const int calls = s_calls;
  const unsigned tag = gran_tag_fused(calls);
  const long long wg_base = (long long)w * TPRES_REGION;
  const long long par_base = (long long)(calls & 1) * d.world * d.max_bytes;
  // granule (j, thread, half) at wg_base + ((j * 256 + thread) * 2 + half) * 8
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const size_t e4 = (size_t)w * (TPR_ELEMS / 4) + j * 256 + threadIdx.x;
    if (e4 >= slab4) continue;
    const long long g = wg_base + (long long)(j * 256 + threadIdx.x) * 16;
    for (int p = 0; p < d.world; ++p) {  // (8-byte stores: the unit the protocol relies on landing whole)
      const __amdgpu_buffer_rsrc_t rp = rsrc(d.buf[p]);
      const long long o = par_base + (long long)d.rank * d.max_bytes + g;
      st_sys8(rp, o, u32x2{gq[j][0], tag});
      st_sys8(rp, o + 8, u32x2{gq[j][1], tag});
    }
  }
  const bool give_up = __hip_atomic_load(d.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
  const __amdgpu_buffer_rsrc_t mine = rsrc(d.buf[d.rank]);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const size_t e4 = (size_t)w * (TPR_ELEMS / 4) + j * 256 + threadIdx.x;
    if (e4 >= slab4) continue;
    const long long g = wg_base + (long long)(j * 256 + threadIdx.x) * 16;
    float sm[4] = {0.f, 0.f, 0.f, 0.f};
    u32x4 r[CAR_MAX_WORLD];
    car_gather16(d, mine, par_base + g, d.max_bytes, tag, give_up, r);
#pragma unroll
    for (int p = 0; p < CAR_MAX_WORLD; ++p) {
      if (p < d.world) {
        sm[0] += __uint_as_float(r[p][0] << 16);
        sm[1] += __uint_as_float(r[p][0] & 0xffff0000u);
        sm[2] += __uint_as_float(r[p][2] << 16);
        sm[3] += __uint_as_float(r[p][2] & 0xffff0000u);
      }
    }
    f32x4 n;
#pragma unroll
    for (int i = 0; i < 4; ++i) n[i] = hv[j][i] + sm[i];
    *reinterpret_cast<f32x4*>(h + e4 * 4) = n;
    *reinterpret_cast<u32x2*>(hb + e4 * 4) = u32x2{pack2bf(n[0], n[1]), pack2bf(n[2], n[3])};
  }
  if (threadIdx.x == 0) __hip_atomic_store(d.wg_ctr + w, calls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
int gemm_tp_groups(int M, int N) { return (int)(((size_t)M * N + TPR_ELEMS - 1) / TPR_ELEMS); }

// The 256 x 256 gemm2 runs the full-line x staging pipeline (FA) with each K-tile's weight loads issued between the
// MFMAs (FAM = 2): 6-21 % faster than fragment-shaped x and 1-8 % faster than issuing the loads up front on the
// Llama-3-8B projections (profiles/r1_gemm2_fullline_x_ab.jsonl, r1_gemm2_fam_ab.jsonl). The other pipeline forms
// (early / late waits, 5 LDS buffers, two half phases, loads up front) and the 128 x 128 register-staged v1 kernel were
// never picked and were removed in round 4 (profiles/r4_variant_pruning.md).

static int g2_wm(int M) { return M <= 128 ? 1 : 2; }  // default tile rows / 128

// split-K plan: fill the chip with workgroups while keeping >= 4 K-tiles (gemm2: 1 WG per CU,
// target ~256 WGs) / >= 8 k-steps (gemm v1: ~512 WGs) per split.
int gemm_ksplit(int M, int N, int K) {
  const int KS = K >> 5;
  const int bm = 128 * g2_wm(M);
  const int tiles = ((N + G2_BN - 1) / G2_BN) * ((M + bm - 1) / bm);
  // one WG per CU, and the fp32 partial slabs (ks * M * N * 8 bytes written + read) kept within
  // ~2x the weight bytes (N * K * 2): measured optimum at M = 128..512 (profiles/README.md)
  int ks = min(256 / tiles, max(1, K / (2 * M)));
  ks = ks < 1 ? 1 : (ks > 16 ? 16 : ks);
  while (ks > 1 && KS / ks < 4) --ks;
  const int kc = (KS + ks - 1) / ks;
  return (KS + kc - 1) / kc;
}

static int num_cus();
size_t gemm_workspace_floats(int M, int N, int K) {
  const int ks = gemm_ksplit(M, N, K);
  return ks > 1 ? (size_t)ks * M * (N + 1) : 0;  // slabs + fused-RMS partial sums
}

// gemm2 tile configurations (the `tile` argument of gemm(); 0 = by M):
//   1: 256 x 256, 8 waves (two ping-pong rows) of 128 x 64;   2: 128 x 256, 4 waves of 128 x 64;
//   3: 128 x 128, 8 waves (two ping-pong rows) of 64 x 32 -- 64 KiB of LDS, so two workgroups can share a CU;
//      for decode shapes with few 256-wide tiles (o / qkv projections) it replaces split-K partial slabs.
static int tile_cfg(int tile, int M) { return tile >= 1 && tile <= 3 ? tile : (M <= 128 ? 2 : 1); }
static bool use_g4(int tile, int M, int K);
// gemm4 on narrower tiles, both with the weights three K-tiles deep (W3; the two-slot forms, tiles 10 / 15, were
// never picked by the tuner at a bench shape and were removed in round 6):
constexpr int G4N6D_TILE = 16;  // 256 x 192 tiles (g4n_mainloop<6, W3>)
constexpr int G4ND_TILE = 17;   // 256 x 128 tiles (g4n_mainloop<4, W3>)
int gemm_qkv_direct_ok(int M, int tile, int K) {
  return ((tile == 0 || tile == 1) && tile_cfg(tile, M) == 1) || use_g4(tile, M, K) ||
         (tile == G4N6D_TILE && (K & 63) == 0);
}

// gemm4 (tile config 7; the default for tile 0 once g_g4_default is set): the 4-wave 256 x 256 kernel of gemm4w.h.
// Needs K % 64 == 0; data-parallel or plain split-K (MODE_PARTIAL + reduce kernel) only -- the stream-K tail,
// hybrid and in-kernel fixup plans stay on gemm2.
constexpr int G4_TILE = 7;
static bool g_g4_default = true;
void gemm_set_g4_default(int on) { g_g4_default = on != 0; }
constexpr int G4P_TILE = 13;  // persistent gemm4 (gemm4p_kernel)
// tile config 14: gemm4 with the weight operand three K-tiles deep (g4_mainloop W3, 160 KiB of LDS) -- for the small-M
// plans whose weights stream from HBM with few tiles sharing them
constexpr int G4D_TILE = 14;
static bool use_g4(int tile, int M, int K) {
  return (K & 63) == 0 &&
         (tile == G4_TILE || tile == G4P_TILE || tile == G4D_TILE || (tile == 0 && g_g4_default && M > 128));
}

// Tile rasterisation: the launch order walks groups of gm m-tiles across every n-tile (g4_tile_coords), so the 32
// workgroups an XCD runs at once cover gm m-tiles x 32 / gm n-tiles. gm = 4 (4 x 8 tiles per XCD) beat 8 (the
// round-4 order), 1, 2 and 16 on every Llama-3-8B projection at M = 2048 and 32768: qkv -7 / -9 %, o -3 / -8 %,
// gate_up -5 / 0 %, down -5 / -6 % (profiles/r5_gemm4_group_m.jsonl). gemm_set_g4_group pins another (tools).
static int g_g4_group = 0;
void gemm_set_g4_group(int gm) { g_g4_group = gm; }
static int g4_group_m(int tiles_m, int tiles_n, int K) {
  (void)tiles_n, (void)K;
  const int gm = g_g4_group > 0 ? g_g4_group : 4;
  return gm < tiles_m ? gm : tiles_m;
}
static int g_g5_diag = 0;  // tools only (gemm5ws.h diag bits 1-16; gemm4 store ablations 64 / 128: wrong results)
template <int MODE, int NJ = 8>
static void launch_g4(const bf16_t* x, const u32x4* w, void* out, int M, int N, int K, int accumulate, int out_f32,
                      bf16_t* mirror, int ksplit, float rms_eps, float* ssq, hipStream_t s, const QKVArgs& qa,
                      float* rms_ws = nullptr, bool persistent = false, bool deep = false) {
  const int tm = (M + G4_BM - 1) / G4_BM, tn = (N + 32 * NJ - 1) / (32 * NJ);
  const int KS64 = K >> 6, kc = (KS64 + ksplit - 1) / ksplit;  // splits past the end run no K-tile (zero slabs)
  const bool rms = MODE != MODE_RESIDUAL && rms_eps >= 0.f;
  const int grid = tm * tn * ksplit;
  const int gm = g4_group_m(tm, tn, K);
  if constexpr (NJ == 8 && MODE != MODE_PARTIAL && MODE != MODE_ARGMAX) {
    if (persistent && ksplit == 1) {  // tile config 13: one workgroup per CU over every tile
      const int pg = min(grid, num_cus());
      if (rms && rms_ws != nullptr) {
        if (rms_rowinv(x, rms_ws, M, K, rms_eps, s) != 0) return;
        gemm4p_kernel<MODE, 2><<<pg, 256, 0, s>>>(x, w, out, M, N, K, accumulate, out_f32, mirror, tm, tn, rms_eps, qa,
                                                  rms_ws, gm);
      } else if (rms) {
        gemm4p_kernel<MODE, 1><<<pg, 256, 0, s>>>(x, w, out, M, N, K, accumulate, out_f32, mirror, tm, tn, rms_eps, qa,
                                                  nullptr, gm);
      } else {
        gemm4p_kernel<MODE, 0><<<pg, 256, 0, s>>>(x, w, out, M, N, K, accumulate, out_f32, mirror, tm, tn, rms_eps, qa,
                                                  nullptr, gm);
      }
      return;
    }
  }
  if constexpr (NJ != 8) {  // 256 x 128 / 192 tiles (deep W only): the statistic precomputed (callers guarantee rms_ws,
    //                         no K split)
    if (rms && rms_ws != nullptr && ksplit == 1 && MODE != MODE_PARTIAL) {
      if (rms_rowinv(x, rms_ws, M, K, rms_eps, s) != 0) return;
      gemm4_kernel<MODE, 2, NJ, 0, true><<<grid, 256, 0, s>>>(x, w, out, M, N, K, accumulate, out_f32, mirror, kc, tm,
                                                              tn, rms_eps, ssq, qa, rms_ws, gm);
    } else if (!rms) {
      gemm4_kernel<MODE, 0, NJ, 0, true><<<grid, 256, 0, s>>>(x, w, out, M, N, K, accumulate, out_f32, mirror, kc, tm,
                                                              tn, rms_eps, ssq, qa, nullptr, gm);
    }
    return;
  }
  if constexpr (MODE == MODE_STORE) {  // ablation instances (tools only; wrong results)
    if (!rms && (g_g5_diag & 192)) {
      if ((g_g5_diag & 192) == 64)
        gemm4_kernel<MODE, 0, 8, 1><<<grid, 256, 0, s>>>(x, w, out, M, N, K, accumulate, out_f32, mirror, kc, tm, tn,
                                                        rms_eps, ssq, qa, nullptr, gm);
      else if ((g_g5_diag & 192) == 128)
        gemm4_kernel<MODE, 0, 8, 2><<<grid, 256, 0, s>>>(x, w, out, M, N, K, accumulate, out_f32, mirror, kc, tm, tn,
                                                        rms_eps, ssq, qa, nullptr, gm);
      else
        gemm4_kernel<MODE, 0, 8, 3><<<grid, 256, 0, s>>>(x, w, out, M, N, K, accumulate, out_f32, mirror, kc, tm, tn,
                                                        rms_eps, ssq, qa, nullptr, gm);
      return;
    }
  }
#define JLA_G4(R, INV)                                                                                             \
  if (deep)                                                                                                         \
    gemm4_kernel<MODE, R, 8, 0, true><<<grid, 256, 0, s>>>(x, w, out, M, N, K, accumulate, out_f32, mirror, kc, tm, \
                                                           tn, rms_eps, ssq, qa, INV, gm);                          \
  else                                                                                                              \
    gemm4_kernel<MODE, R><<<grid, 256, 0, s>>>(x, w, out, M, N, K, accumulate, out_f32, mirror, kc, tm, tn, rms_eps, \
                                               ssq, qa, INV, gm)
  if (rms && rms_ws != nullptr && ksplit == 1 && MODE != MODE_PARTIAL) {
    if (rms_rowinv(x, rms_ws, M, K, rms_eps, s) != 0) return;  // (K % 8 == 0 always holds here)
    JLA_G4(2, rms_ws);
  } else if (rms) {
    JLA_G4(1, nullptr);
  } else {
    JLA_G4(0, nullptr);
  }
#undef JLA_G4
}

template <int MODE>
static void launch_g2(const bf16_t* x, const u32x4* w, void* out, int M, int N, int K, int accumulate, int out_f32,
                      bf16_t* mirror, int kc, int ksplit, float rms_eps, float* ssq, int tile, hipStream_t s,
                      const QKVArgs& qa = QKVArgs{}, float* rms_ws = nullptr) {
  if constexpr (MODE != MODE_QKV && MODE != MODE_ARGMAX) {
    if (tile == G4ND_TILE && (K & 63) == 0) {
      launch_g4<MODE, 4>(x, w, out, M, N, K, accumulate, out_f32, mirror, ksplit, rms_eps, ssq, s, qa, rms_ws, false,
                         true);
      return;
    }
  }
  // tile config 16: 256 x 192 tiles -- Llama-3-8B qkv (N = 6144) at M = 2048 is 8 x 32 = 256 tiles, one per CU, where
  // the 256 x 256 grid has 192 (0.75 of a wave); the QKV epilogue included
  if constexpr (MODE != MODE_ARGMAX) {
    if (tile == G4N6D_TILE && (K & 63) == 0) {
      launch_g4<MODE, 6>(x, w, out, M, N, K, accumulate, out_f32, mirror, ksplit, rms_eps, ssq, s, qa, rms_ws, false,
                         true);
      return;
    }
  }
  if (use_g4(tile, M, K)) {
    // persistent for the residual epilogue at prefill sizes: o / down at M = 32768 3.5 / 2.4 % faster (the CUs'
    // fp32 read-modify-write bursts desynchronise); the store / SwiGLU / QKV epilogues lose 1.5-3.6 % that way
    // (profiles/r5_gemm4_persistent_ab.jsonl)
    const bool persist = tile == G4P_TILE || (MODE == MODE_RESIDUAL && tile == 0 && ksplit == 1 && M >= 4096);
    launch_g4<MODE>(x, w, out, M, N, K, accumulate, out_f32, mirror, ksplit, rms_eps, ssq, s, qa, rms_ws, persist,
                    tile == G4D_TILE);
    return;
  }
  const int cfg = tile_cfg(tile, M);
  const int bm = cfg == 1 ? 256 : 128, bn = cfg == 3 ? 128 : 256;
  const int tm = (M + bm - 1) / bm, tn = (N + bn - 1) / bn;
  const int grid = tm * tn * ksplit;
#define JLA_G2S(WMV, NB, LATE, R, MTV, NTV, SB)                                                             \
  gemm2_kernel<MODE, WMV, NB, LATE, R, MTV, NTV, SB><<<grid, 256 * WMV, 0, s>>>(                            \
      x, w, out, M, N, K, accumulate, out_f32, mirror, kc, tm, tn, rms_eps, ssq, qa)
#define JLA_G2(WMV, NB, LATE, R, MTV, NTV) JLA_G2S(WMV, NB, LATE, R, MTV, NTV, 1)
#define JLA_G2FA(R, FM)                                                                                      \
  gemm2_kernel<MODE, 2, 4, true, R, 8, 4, 1, true, FM><<<grid, 512, 0, s>>>(x, w, out, M, N, K, accumulate,     \
                                                                           out_f32, mirror, kc, tm, tn, rms_eps, ssq, qa)
  if constexpr (MODE == MODE_QKV) {  // the direct RoPE / KV-write epilogue: the default 256 x 256 FA pipeline only
    JLA_G2FA(true, 2);
  } else {
  const bool rms = MODE != MODE_RESIDUAL && rms_eps >= 0.f;
  if constexpr (MODE != MODE_RESIDUAL) {
    if (rms) {  // fused RMSNorm statistic (default pipeline variant only)
      if (cfg == 2)
        JLA_G2(1, 4, false, true, 8, 4);
      else if (cfg == 3)
        JLA_G2(2, 4, true, true, 4, 2);
      else
        JLA_G2FA(true, 2);
      return;
    }
  }
  if (cfg == 2)
    JLA_G2(1, 4, false, false, 8, 4);
  else if (cfg == 3)
    JLA_G2(2, 4, true, false, 4, 2);
  else
    JLA_G2FA(false, 2);
  }
#undef JLA_G2FA
#undef JLA_G2
#undef JLA_G2S
}

template <int MODE>
static void launch_tiled(const bf16_t* x, const u32x4* w, void* out, int M, int N, int K, int accumulate,
                         int out_f32, bf16_t* mirror, int kc, int ksplit, float rms_eps, float* ssq, int tile,
                         hipStream_t s, float* rms_ws = nullptr) {
  launch_g2<MODE>(x, w, out, M, N, K, accumulate, out_f32, mirror, kc, ksplit, rms_eps, ssq, tile, s, QKVArgs{},
                  rms_ws);
}

static int g_num_cus = 0;
static int num_cus() {
  if (g_num_cus == 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      g_num_cus = prop.multiProcessorCount;
    if (g_num_cus <= 0) g_num_cus = 256;
  }
  return g_num_cus;
}

// the split-K reduce + epilogue launch over [ksplit][M][N] partial slabs (+ [ksplit][M] sums of squares, fused norm)
static int launch_reduce(const float* ws, int ksplit, void* out, int M, int N, int K, int mode, int accumulate,
                         int out_f32, bf16_t* mirror, const QKVArgs* qkv, const float* ssq, float rms_eps,
                         hipStream_t s) {
  const size_t total4 = (size_t)M * N / (mode == MODE_SWIGLU ? 8 : 4);
  const int rgrid = (int)((total4 + 255) / 256);
  QKVArgs qa{};
  if (qkv) qa = *qkv;
  const float eps = ssq ? rms_eps : 0.f;
  switch (mode) {
    case MODE_STORE:
      gemm_reduce_kernel<MODE_STORE><<<rgrid, 256, 0, s>>>(ws, ksplit, out, M, N, accumulate, out_f32, nullptr, qa,
                                                           ssq, K, eps);
      break;
    case MODE_RESIDUAL:
      gemm_reduce_kernel<MODE_RESIDUAL><<<rgrid, 256, 0, s>>>(ws, ksplit, out, M, N, accumulate, 1, mirror, qa,
                                                              nullptr, K, eps);
      break;
    case MODE_SWIGLU:
      gemm_reduce_kernel<MODE_SWIGLU><<<rgrid, 256, 0, s>>>(ws, ksplit, out, M, N, accumulate, 0, nullptr, qa, ssq,
                                                            K, eps);
      break;
    case MODE_QKV:
      gemm_reduce_kernel<MODE_QKV><<<rgrid, 256, 0, s>>>(ws, ksplit, out, M, N, accumulate, 0, nullptr, qa, ssq, K,
                                                         eps);
      break;
    case MODE_TPRESID:  // out = h (fp32 residual), mirror = hb, qkv->tp = the TP group's CarDevice
      if (!qkv || !qa.tp || !mirror || ssq || (N & 3)) return -1;
      gemm_reduce_tp_kernel<<<gemm_tp_groups(M, N), 256, 0, s>>>(ws, ksplit, static_cast<float*>(out), mirror, M, N,
                                                                 static_cast<const CarDevice*>(qa.tp));
      break;
    default: return -1;
  }
  JLA_CHECK_LAUNCH();
  return 0;
}

// gemm5 (tile 11: 4 n-tiles per wave, 256-column workgroups; tile 12: 2 n-tiles, 128 columns): the weight-streaming
// split-K main loop (gemm5ws.h), then the reduce kernel runs the epilogue (even without a K split)
void gemm5_set_diag(int d) { g_g5_diag = d; }
int gemm5_ksplit(int K, int ksplit) {  // the effective split count over 64-deep K-stages
  const int KS64 = K >> 6;
  if (ksplit < 1) ksplit = 1;
  const int kc = (KS64 + ksplit - 1) / ksplit;
  return (KS64 + kc - 1) / kc;
}
static int launch_g5(const bf16_t* x, const u32x4* w, void* out, int M, int N, int K, int mode, int accumulate,
                     int out_f32, bf16_t* mirror, const QKVArgs* qkv, float* ws, size_t ws_floats, int ksplit,
                     float rms_eps, int tile, hipStream_t s) {
  if ((K & 63) || (N & 15) || M <= 0) return -1;
  if (mode == MODE_SWIGLU && (N & 31)) return -1;
  if (mode == MODE_QKV && !qkv) return -1;
  const bool rms = rms_eps >= 0.f && mode != MODE_RESIDUAL;
  const int KS64 = K >> 6;
  ksplit = gemm5_ksplit(K, ksplit);
  const int kc = (KS64 + ksplit - 1) / ksplit;
  const size_t need = (size_t)ksplit * M * N + (rms ? (size_t)ksplit * M : 0);
  if (ws == nullptr || ws_floats < need) return -3;
  float* ssq = rms ? ws + (size_t)ksplit * M * N : nullptr;
  const int mt = M <= 128 ? 8 : 16, rows = 16 * mt;
  const int ntw = tile == G5_TILE ? 4 : 2;
  const int tiles_m = (M + rows - 1) / rows, tiles_n = (N + 64 * ntw - 1) / (64 * ntw);
  const int grid = tiles_m * tiles_n * ksplit;
  if (mt == 8 && ntw == 4)
    gemm5_partial_kernel<8, 4><<<grid, 256, 0, s>>>(x, w, ws, M, N, K, kc, tiles_m, tiles_n, ssq, g_g5_diag);
  else if (mt == 8)
    gemm5_partial_kernel<8, 2><<<grid, 256, 0, s>>>(x, w, ws, M, N, K, kc, tiles_m, tiles_n, ssq, g_g5_diag);
  else if (ntw == 4)
    gemm5_partial_kernel<16, 4><<<grid, 256, 0, s>>>(x, w, ws, M, N, K, kc, tiles_m, tiles_n, ssq, g_g5_diag);
  else
    gemm5_partial_kernel<16, 2><<<grid, 256, 0, s>>>(x, w, ws, M, N, K, kc, tiles_m, tiles_n, ssq, g_g5_diag);
  JLA_CHECK_LAUNCH();
  return launch_reduce(ws, ksplit, out, M, N, K, mode, accumulate, out_f32, mirror, qkv, ssq, rms_eps, s);
}

int gemm(const bf16_t* x, const void* W, void* out, int M, int N, int K, int mode, int accumulate, int out_f32,
         bf16_t* mirror, const QKVArgs* qkv, float* ws, size_t ws_floats, int ksplit, hipStream_t s,
         float rms_eps, int tile, float* rms_ws, size_t rms_ws_floats) {
  if (tile == G5_TILE || tile == G5_TILE + 1) {
    if (mode == MODE_ARGMAX || (rms_eps >= 0.f && (mode == MODE_RESIDUAL || mode == MODE_TPRESID))) return -1;
    return launch_g5(x, static_cast<const u32x4*>(W), out, M, N, K, mode, accumulate, out_f32, mirror, qkv, ws,
                     ws_floats, ksplit, rms_eps, tile, s);
  }
  if (rms_ws != nullptr && rms_ws_floats < (size_t)M) rms_ws = nullptr;  // too small: the in-loop statistic
  if (tile == G4ND_TILE &&
      ((K & 63) || (mode == MODE_QKV && ksplit <= 1) || mode == MODE_ARGMAX ||
       (rms_eps >= 0.f && mode != MODE_RESIDUAL && (ksplit > 1 || rms_ws == nullptr))))
    return -1;  // the 256 x 128 plan: no QKV / argmax epilogue, the fused norm only precomputed without a K split
  if (M <= 0) return 0;
  if ((N & 15) || (K & 31)) return -1;
  if (mode == MODE_SWIGLU && (N & 31)) return -1;
  const bool rms = rms_eps >= 0.f;
  if (rms && mode == MODE_RESIDUAL) return -5;  // caller pre-scales x instead
  if (mode == MODE_QKV && !qkv) return -1;
  const int KS = K >> 5;
  if (ksplit < 1) ksplit = 1;
  const int kc = (KS + ksplit - 1) / ksplit;
  ksplit = (KS + kc - 1) / kc;
  if (mode == MODE_TPRESID && (ksplit == 1 || rms)) return -1;  // the exchange lives in the split-K reduce
  // qkv without a K split: the RoPE / KV-write epilogue of the default FA pipeline (256 x 256 tiles, fused norm)
  if (mode == MODE_QKV && ksplit == 1 && !(gemm_qkv_direct_ok(M, tile, K) && rms)) return -1;
  // the 256 x 128 / 192 tiles take the fused norm only as the precomputed statistic without a K split (launch_g4
  // would otherwise launch nothing)
  if ((tile == G4ND_TILE || tile == G4N6D_TILE) && rms &&
      (ksplit > 1 || rms_ws == nullptr))
    return -6;
  const u32x4* w = static_cast<const u32x4*>(W);
  if (ksplit == 1) {
    switch (mode) {
      case MODE_QKV:
        launch_g2<MODE_QKV>(x, w, nullptr, M, N, K, 0, 0, nullptr, kc, 1, rms_eps, nullptr, tile, s, *qkv, rms_ws);
        break;
      case MODE_STORE:
        launch_tiled<MODE_STORE>(x, w, out, M, N, K, accumulate, out_f32, nullptr, kc, 1, rms_eps, nullptr, tile, s,
                                 rms_ws);
        break;
      case MODE_RESIDUAL:
        launch_tiled<MODE_RESIDUAL>(x, w, out, M, N, K, accumulate, 1, mirror, kc, 1, -1.f, nullptr, tile, s);
        break;
      case MODE_SWIGLU:
        launch_tiled<MODE_SWIGLU>(x, w, out, M, N, K, accumulate, 0, nullptr, kc, 1, rms_eps, nullptr, tile, s,
                                  rms_ws);
        break;
      default: return -1;
    }
    JLA_CHECK_LAUNCH();
    return 0;
  }
  // workspace: [ksplit][M][N] fp32 partial slabs, then (fused RMS) [ksplit][M] partial sums of squares
  const size_t need = (size_t)ksplit * M * N + (rms ? (size_t)ksplit * M : 0);
  if ((N & 3) || ws == nullptr || ws_floats < need) return -3;
  float* ssq = rms ? ws + (size_t)ksplit * M * N : nullptr;
  launch_tiled<MODE_PARTIAL>(x, w, ws, M, N, K, 0, 1, nullptr, kc, ksplit, rms_eps, ssq, tile, s);
  JLA_CHECK_LAUNCH();
  return launch_reduce(ws, ksplit, out, M, N, K, mode, accumulate, out_f32, mirror, qkv, ssq, rms_eps, s);
}

// ---- greedy lm_head: GEMM with the argmax in its epilogue (no fp32 logits round trip through HBM:
// at M = 2048, V = 128256 that is 1 GB written + 1 GB read per decode step), then the [M][P] partials are
// reduced per row. Ties go to the smaller index, so the result equals argmax_kernel's.
JLA_DEV void amax_merge(float& bv, int& bi, float ov, int oi) {
  if (ov > bv || (ov == bv && oi < bi)) {
    bv = ov;
    bi = oi;
  }
}

// TPR threads per row (64: one wave per row, 4 rows per 256-thread block; 1024: one block per row for the
// decode-sized M, where one wave walking ~8000 partials of a row with one dependent load per step took ~38 us).
// Each thread keeps 4 independent (value, index) candidates so 4 loads are in flight per step.
template <int TPR>
__global__ void __launch_bounds__(TPR == 64 ? 256 : TPR)
    argmax_partials_kernel(const float2* __restrict__ part, int P, int M, int32_t* __restrict__ idx,
                           float* __restrict__ val) {
  __shared__ float s_v[16];
  __shared__ int s_i[16];
  const int row = TPR == 64 ? blockIdx.x * 4 + (threadIdx.x >> 6) : blockIdx.x;
  const int t = TPR == 64 ? (threadIdx.x & 63) : threadIdx.x;
  if (row >= M) return;
  const float2* pr = part + (size_t)row * P;
  float bv[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  int bi[4] = {0x7fffffff, 0x7fffffff, 0x7fffffff, 0x7fffffff};
  for (int k0 = t; k0 < P; k0 += 4 * TPR) {
    float2 e[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + u * TPR;
      e[u] = k < P ? pr[k] : make_float2(-INFINITY, __int_as_float(0x7fffffff));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) amax_merge(bv[u], bi[u], e[u].x, __float_as_int(e[u].y));
  }
#pragma unroll
  for (int u = 1; u < 4; ++u) amax_merge(bv[0], bi[0], bv[u], bi[u]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) amax_merge(bv[0], bi[0], __shfl_xor(bv[0], o, 64), __shfl_xor(bi[0], o, 64));
  if constexpr (TPR > 64) {
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
      s_v[w] = bv[0];
      s_i[w] = bi[0];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int ww = 1; ww < TPR / 64; ++ww) amax_merge(bv[0], bi[0], s_v[ww], s_i[ww]);
      idx[row] = bi[0] == 0x7fffffff ? 0 : bi[0];
      val[row] = bv[0];
    }
  } else if (t == 0) {
    idx[row] = bi[0] == 0x7fffffff ? 0 : bi[0];
    val[row] = bv[0];
  }
}

static void launch_argmax_partials(const float2* part, int P, int M, int32_t* idx, float* val, hipStream_t s) {
  if (M <= 512)
    argmax_partials_kernel<1024><<<M, 1024, 0, s>>>(part, P, M, idx, val);
  else
    argmax_partials_kernel<64><<<(M + 3) / 4, 256, 0, s>>>(part, P, M, idx, val);
}

int argmax_partials(const float* part, int P, int M, int32_t* idx, float* val, hipStream_t s) {
  if (M <= 0) return 0;
  launch_argmax_partials(reinterpret_cast<const float2*>(part), P, M, idx, val, s);
  JLA_CHECK_LAUNCH();
  return 0;
}

size_t gemm_argmax_workspace_floats(int M, int N) { return (size_t)M * ((N + G2_BN - 1) / G2_BN) * 4 * 2; }

int gemm_argmax(const bf16_t* x, const void* W, float* ws, size_t ws_floats, int M, int N, int K, float rms_eps,
                int32_t* idx, float* val, hipStream_t s, float* rms_ws, size_t rms_ws_floats) {
  if (rms_ws != nullptr && rms_ws_floats < (size_t)M) rms_ws = nullptr;
  if (M <= 0) return 0;
  if ((N & 15) || (K & 31)) return -1;
  if (ws == nullptr || ws_floats < gemm_argmax_workspace_floats(M, N)) return -3;
  const int tm = (M + 255) / 256, tn = (N + G2_BN - 1) / G2_BN;
  const u32x4* w = static_cast<const u32x4*>(W);
  if (use_g4(0, M, K)) {  // 2 partials per 256-column tile (one per wave column)
    launch_g4<MODE_ARGMAX>(x, w, ws, M, N, K, 0, 1, nullptr, 1, rms_eps, nullptr, s, QKVArgs{}, rms_ws);
    JLA_CHECK_LAUNCH();
    launch_argmax_partials(reinterpret_cast<const float2*>(ws), tn * 2, M, idx, val, s);
    JLA_CHECK_LAUNCH();
    return 0;
  }
  if (rms_eps >= 0.f)
    gemm2_kernel<MODE_ARGMAX, 2, 4, true, true, 8, 4, 1, true, 2><<<tm * tn, 512, 0, s>>>(
        x, w, ws, M, N, K, 0, 1, nullptr, K >> 5, tm, tn, rms_eps, nullptr, QKVArgs{});
  else
    gemm2_kernel<MODE_ARGMAX, 2, 4, true, false, 8, 4, 1, true, 2><<<tm * tn, 512, 0, s>>>(
        x, w, ws, M, N, K, 0, 1, nullptr, K >> 5, tm, tn, rms_eps, nullptr, QKVArgs{});
  JLA_CHECK_LAUNCH();
  launch_argmax_partials(reinterpret_cast<const float2*>(ws), tn * 4, M, idx, val, s);
  JLA_CHECK_LAUNCH();
  return 0;
}

JLA_BOUNDS_ACCESSOR(gemm)

}  // namespace jla
