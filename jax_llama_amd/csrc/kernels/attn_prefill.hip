// Prefill (multi-query) attention over the KV cache: flash-style online softmax on MFMA.
//
// Reference semantics: model.py:236-291 (causal mask sliced at cache_index, AND padding mask,
// additive finfo.min bias, softmax in fp32, P.V), without ever materialising the (S x T) score
// matrix or the (L x L) causal mask (model.py:154). Query s of row b sits at cache slot slot0 + s
// and attends keys j with kv_start[b] <= j <= slot0 + s (and key_mask[b, j] if given). A query
// with no valid key (a left-pad position) outputs 0, never NaN.
//
// Workgroup = (64-query block, q head, batch row), 4 waves x 16 query rows. Per 32-key tile:
//   K tile [32 x 128] and V^T tile [128 x 32] are staged in LDS (V transposed on the way in so the
//   P.V B operand is a contiguous ds_read_b128); padded rows make every fragment read
//   bank-conflict free;
//   S = Q K^T: 2 key sub-tiles x 4 d-steps of v_mfma_f32_16x16x32_bf16 (Q fragments live in VGPRs);
//   online softmax on the accumulator layout (row stats reduced over 16 lanes);
//   P goes through a small per-wave LDS tile to become the A operand; O += P V: 8 MFMAs.
#include <type_traits>

#include "common.h"
#include "launchers.h"

namespace jla {

constexpr int AP_DH = 128;
constexpr int AP_QB = 64;             // queries per workgroup
constexpr int AP_KT = 32;             // keys per tile
constexpr int AP_KROW = AP_DH + 8;    // K tile row (bf16 elements): 272 B
constexpr int AP_VROW = AP_KT + 8;    // V^T tile row: 80 B
constexpr int AP_PROW = AP_KT + 8;    // P tile row: 80 B

__global__ void __launch_bounds__(256)
    attn_prefill_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                        const int32_t* __restrict__ slot_ptr, const int32_t* __restrict__ kv_start,
                        const uint8_t* __restrict__ key_mask, int mask_len, bf16_t* __restrict__ out, int S, int H,
                        int Hkv, int T, float scale) {
  __shared__ __attribute__((aligned(16))) bf16_t Kt[AP_KT * AP_KROW];
  __shared__ __attribute__((aligned(16))) bf16_t Vt[AP_DH * AP_VROW];
  __shared__ __attribute__((aligned(16))) bf16_t Pt[4][16 * AP_PROW];

  const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int rep = H / Hkv, kvh = h / rep;
  const int slot0 = slot_ptr[0];
  if (slot0 + S > T && threadIdx.x == 0) JLA_FLAG(JLA_BOUNDS_ATTN_T);
  const int lo = kv_start[b];
  const uint8_t* mrow = key_mask ? key_mask + (size_t)b * mask_len : nullptr;

  // Q fragments (A operand): row li of this wave's 16 queries, d = 32*kk + 8*g
  const int qrow_a = min(qb * AP_QB + w * 16 + li, S - 1);
  u32x4 qa[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk)
    qa[kk] = *reinterpret_cast<const u32x4*>(q + (((size_t)b * S + qrow_a) * H + h) * AP_DH + 32 * kk + 8 * g);

  // this lane's 4 accumulator rows
  int qslot[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) qslot[i] = slot0 + qb * AP_QB + w * 16 + 4 * g + i;

  f32x4 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrun[4], lrun[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    mrun[i] = -INFINITY;
    lrun[i] = 0.f;
  }

  const int last_key = min(slot0 + min(S, (qb + 1) * AP_QB) - 1, T - 1);
  const int t_begin = (lo / AP_KT) * AP_KT;
  const bf16_t* kb = kc + ((size_t)b * Hkv + kvh) * T * AP_DH;
  const bf16_t* vb = vc + ((size_t)b * Hkv + kvh) * T * AP_DH;

  for (int t0 = t_begin; t0 <= last_key; t0 += AP_KT) {
    // ---- stage K (row-major) and V (transposed); 512 x 16 B per tile each, 2 per thread
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int idx = tid + r * 256;  // 0..511
      const int key = idx >> 4, d0 = (idx & 15) * 8;
      const int j = min(t0 + key, T - 1);
      const u32x4 kv = *reinterpret_cast<const u32x4*>(kb + (size_t)j * AP_DH + d0);
      const u32x4 vv = *reinterpret_cast<const u32x4*>(vb + (size_t)j * AP_DH + d0);
      *reinterpret_cast<u32x4*>(&Kt[key * AP_KROW + d0]) = kv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        Vt[(d0 + 2 * e) * AP_VROW + key] = (bf16_t)(vv[e] & 0xffffu);
        Vt[(d0 + 2 * e + 1) * AP_VROW + key] = (bf16_t)(vv[e] >> 16);
      }
    }
    __syncthreads();

    // ---- S = Q K^T for two 16-key sub-tiles
    f32x4 s[2];
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      s[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const u32x4 kf = *reinterpret_cast<const u32x4*>(&Kt[(n * 16 + li) * AP_KROW + 32 * kk + 8 * g]);
        s[n] = mfma16x16x32(qa[kk], kf, s[n]);
      }
    }
    // ---- mask + online softmax (row i of this lane = query 4g+i; column = key n*16+li)
    float p[2][4];
    float alpha[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float mt = -INFINITY;
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int j = t0 + n * 16 + li;
        bool valid = j <= qslot[i] && j >= lo && j < T;
        if (mrow && j < mask_len) valid = valid && mrow[j] != 0;
        const float v = valid ? s[n][i] * scale : -INFINITY;
        p[n][i] = v;
        mt = fmaxf(mt, v);
      }
      mt = fmaxf(mt, __shfl_xor(mt, 1, 64));
      mt = fmaxf(mt, __shfl_xor(mt, 2, 64));
      mt = fmaxf(mt, __shfl_xor(mt, 4, 64));
      mt = fmaxf(mt, __shfl_xor(mt, 8, 64));
      const float mn = fmaxf(mrun[i], mt);
      float rs = 0.f;
      if (mn == -INFINITY) {
        alpha[i] = 1.f;
        p[0][i] = 0.f;
        p[1][i] = 0.f;
      } else {
        alpha[i] = __expf(mrun[i] - mn);
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          p[n][i] = (p[n][i] == -INFINITY) ? 0.f : __expf(p[n][i] - mn);
          rs += p[n][i];
        }
      }
      rs += __shfl_xor(rs, 1, 64);
      rs += __shfl_xor(rs, 2, 64);
      rs += __shfl_xor(rs, 4, 64);
      rs += __shfl_xor(rs, 8, 64);
      lrun[i] = lrun[i] * alpha[i] + rs;
      mrun[i] = mn;
    }
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) o[dt][i] *= alpha[i];

    // ---- P (C layout) -> LDS -> A operand
    bf16_t* pw = Pt[w];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) pw[(4 * g + i) * AP_PROW + n * 16 + li] = f2bf(p[n][i]);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's P writes landed
    __builtin_amdgcn_wave_barrier();
    const u32x4 pa = *reinterpret_cast<const u32x4*>(&pw[li * AP_PROW + 8 * g]);
    // ---- O += P V
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      const u32x4 vf = *reinterpret_cast<const u32x4*>(&Vt[(dt * 16 + li) * AP_VROW + 8 * g]);
      o[dt] = mfma16x16x32(pa, vf, o[dt]);
    }
  }

  // ---- epilogue: out[b*S + q][h*Dh + d]
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int qr = qb * AP_QB + w * 16 + 4 * g + i;
    if (qr >= S) continue;
    const float inv = lrun[i] > 0.f ? 1.f / lrun[i] : 0.f;
    bf16_t* dst = out + ((size_t)b * S + qr) * H * AP_DH + (size_t)h * AP_DH;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) dst[dt * 16 + li] = f2bf(o[dt][i] * inv);
  }
}

// ================================================================================================
// v2: GQA-shared flash prefill on v_mfma_f32_32x32x16_bf16.
//
// Workgroup = NW waves = (batch row b, kv head, group of q heads, block of query positions); every wave
// owns 32 query rows of ONE q head, and all NW waves read the SAME K/V tiles from LDS, so a (b, kv head)
// K/V tile is fetched once per rep/hpw workgroups instead of once per q head (rep = H / Hkv).
// Per 64-key tile and wave:
//   S^T = K Q^T   (A = K fragment by ds_read_b128 from an XOR-swizzled image, B = Q^T fragments held in
//                  VGPRs for the whole kernel): 2 key blocks x 8 dk-steps = 16 MFMAs. The C layout puts the
//                  wave's query on the LANE (col = lane & 31) and 32 of the 64 keys in its registers, so the
//                  online softmax is lane-local plus one exchange with lane ^ 32;
//   O^T += V^T P^T (A = V^T by ds_read_b64_tr_b16 transposed reads of the row-major V image, B = the bf16 P
//                  registers used in place with the permuted k order of the accumulator layout): 4 d tiles x
//                  4 key steps = 16 MFMAs. O^T again has the query on the lane, so the rescale by
//                  exp2(m_old - m_new) is lane-local too.
// K/V tiles are register-staged (loads for tile t+1 issued before tile t's MFMAs, written to LDS after
// the barrier that ends tile t). Causal: the workgroup stops at its last query's slot; a wave whose
// queries all precede a tile skips its MFMAs; only tiles that cross the diagonal, kv_start or T are
// masked element-wise. Each workgroup runs a heavy and a light query block (causal balance).
constexpr int FA_KT = 64;  // keys per tile

// byte offset of 16-byte chunk ch (0..15) of row `row` in a [rows][128 bf16] image whose XOR swizzle
// serves both ds_read_b128 row reads and ds_read_b64_tr_b16 transposed reads without bank conflicts
JLA_DEV int fa_off(int row, int ch) { return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3))); }

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

JLA_DEV f32x16 mfma32(const u32x4 a, const u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}
JLA_DEV u32x2 ld_tr(const char* lds, int off) {
  return __builtin_bit_cast(u32x2, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                       (__attribute__((address_space(3))) s16x4*)(lds + off)));
}

// One query block of 32 per wave (a 64-query "QB = 2" form halved the LDS bytes per MFMA but needed ~340 registers,
// one workgroup per CU, and ran 1.4-2x slower: profiles/r2_attn_prefill_qb2_ab.jsonl -- removed).
//
// PIPE: the scores of tile i+1 are issued before the softmax of tile i, so one wave's MFMA pipe works
// through S(i+1) while its VALU runs exp / sum / pack of tile i (independent instructions in one basic block).
// K and V each get a 2-slot LDS ring (64 KiB per workgroup): K(i+1) and V(i) are resident during tile i while
// the registers stage K(i+2) and V(i+1) into the slots freed by tile i-1, so each tile ends with ONE barrier.
// Lazy rescale (every launch): the running max (and with it the O / l rescale) moves only when a lane's tile max
// exceeds it by more than 8 (log2 units): exp2 of the rest stays <= 256, exact in fp32 and bf16-representable for P;
// the 64 O multiplies per tile run only in a wave-uniform branch when some lane needs them (mostly the first tiles).
// (The eager-rescale launches, impls 4 / 5 / 6 / 10, were slower everywhere and removed in round 4:
// profiles/r3_attn_prefill_pipe_ab.jsonl, profiles/r4_variant_pruning.md.)
// PIPE 2: the same loop with the K / V DMA as inline asm (glds16_asm: with the builtin, hipcc put a vmcnt(0) before
// the first V read of every tile, i.e. waited for the DMA of the NEXT tiles it had just issued), and branch-free, with
// the next tile's 16 scores MFMAs spread over the 4 key steps (4 per step, fenced by sched_barrier) beside the exps and
// PV MFMAs instead of sunk into one serial read -> wait -> MFMA chain at the end of the tile.
template <int NW, int PIPE>
__global__ void __launch_bounds__(NW * 64, 2)
    attn_prefill_v2_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                           const int32_t* __restrict__ slot_ptr, const int32_t* __restrict__ kv_start,
                           const uint8_t* __restrict__ key_mask, int mask_len, bf16_t* __restrict__ out, int S, int H,
                           int Hkv, int T, float scale_log2, int npb, int hgroups, int n_qb, int split) {
  constexpr int QB = 1;  // query blocks of 32 per wave
  constexpr int NT = NW * 64;
  constexpr int TILE_BYTES = FA_KT * AP_DH * 2;            // 16 KiB
  constexpr int CH_PER_T = FA_KT * 16 / NT;                 // 16-byte chunks per thread per tile (K or V)
  constexpr int QW = 32 * QB;                               // queries per wave
  __shared__ __attribute__((aligned(16))) char lds[(PIPE ? 4 : 2) * TILE_BYTES];
  char* Ks = lds;
  char* Vs = lds + TILE_BYTES;

  // split = 1 (small grids): the heavy and the light block of a pair are two workgroups of a 1-D grid, all heavy
  // ones first -- ids g and g + items are the same pair, so when the second round of dispatch lands on the CUs in
  // the order of the first, every CU again holds one (heavy, light) pair, now as two resident workgroups
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z, pass_lo = 0, pass_hi = 2;
  if (split) {
    const int P = (n_qb + 1) / 2, Y = Hkv * hgroups;  // 1-D grid of 2 x P x Y x B workgroups
    const int items = (int)gridDim.x / 2;
    int g = blockIdx.x;
    const bool light = g >= items;
    if (light) g -= items;
    bx = g % P;
    by = (g / P) % Y;
    bz = g / (P * Y);
    pass_lo = light ? 1 : 0;
    pass_hi = light ? 2 : 1;
  }
  const int kvh = by / hgroups, hg = by - kvh * hgroups;
  const int b = bz;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int hi = lane >> 5, col = lane & 31;
  const int rep = H / Hkv, hpw = NW / npb;
  const int r = w / npb, pb = w - r * npb;
  const int h = kvh * rep + hg * hpw + r;
  // causal balance: workgroup x runs query block n_qb-1-x (heavy) and then block x (light), so every
  // workgroup streams ~the same number of K/V tiles (with one block per workgroup, S = 2048 at B = 1 ran
  // the heaviest workgroup ~2x longer than the average one)
  for (int pass = pass_lo; pass < pass_hi; ++pass) {
  const int qb = pass == 0 ? n_qb - 1 - bx : bx;
  if (pass == 1 && qb >= n_qb - 1 - bx) break;  // odd n_qb: the middle block runs once
  if (pass == 1) __syncthreads();  // every wave is done with the LDS images of the first block
  const int p0 = qb * QW * npb + QW * pb;   // first query position of this wave
  const int slot0 = slot_ptr[0];
  if (slot0 + S > T && threadIdx.x == 0) JLA_FLAG(JLA_BOUNDS_ATTN_T);
  const int lo = kv_start[b];
  const uint8_t* mrow = key_mask ? key_mask + (size_t)b * mask_len : nullptr;

  // Q^T fragments (B operand) of query block qq: lane holds Q[p0 + 32 qq + col][16 ks + 8 hi .. +7]
  u32x4 qf[QB][8];
#pragma unroll
  for (int qq = 0; qq < QB; ++qq) {
    const int pos = p0 + 32 * qq + col;
    const bf16_t* qrow = q + (((size_t)b * S + min(pos, S - 1)) * H + h) * AP_DH + 8 * hi;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qf[qq][ks] = *reinterpret_cast<const u32x4*>(qrow + 16 * ks);
  }
  f32x16 o[QB][4];
  float m_run[QB], l_run[QB];
#pragma unroll
  for (int qq = 0; qq < QB; ++qq) {
    m_run[qq] = -INFINITY;
    l_run[qq] = 0.f;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) o[qq][dt][i] = 0.f;
  }

  const int wg_last_pos = min(S, (qb + 1) * QW * npb) - 1;
  const int last_key = min(slot0 + wg_last_pos, T - 1);
  const int t_begin = (lo / FA_KT) * FA_KT;
  const int wave_last_slot = slot0 + min(p0 + QW - 1, S - 1);
  const bf16_t* kb = kc + ((size_t)b * Hkv + kvh) * T * AP_DH;
  const bf16_t* vb = vc + ((size_t)b * Hkv + kvh) * T * AP_DH;

  // staging: thread handles chunks c = tid + NT * i (row = c >> 4, ch = c & 15) of each tile
  u32x4 sk[CH_PER_T], sv[CH_PER_T];
  auto load_tile = [&](int t0) {
#pragma unroll
    for (int i = 0; i < CH_PER_T; ++i) {
      const int c = tid + NT * i, row = c >> 4, ch = c & 15;
      const size_t src = (size_t)min(t0 + row, T - 1) * AP_DH + 8 * ch;
      sk[i] = *reinterpret_cast<const u32x4*>(kb + src);
      sv[i] = *reinterpret_cast<const u32x4*>(vb + src);
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < CH_PER_T; ++i) {
      const int c = tid + NT * i, row = c >> 4, ch = c & 15;
      *reinterpret_cast<u32x4*>(Ks + fa_off(row, ch)) = sk[i];
      *reinterpret_cast<u32x4*>(Vs + fa_off(row, ch)) = sv[i];
    }
  };
  // per-lane LDS read offsets: K row reads (key block kb, dk step ks -> chunk 2 ks + hi)
  // V transposed reads: 16-lane group G = lane >> 4 covers d columns 16 (G & 1) .. +15 of a 32-wide d tile,
  // lane 4q + p of the group addresses row q of the 4-key block, columns 4p .. 4p + 3.
  const int gq = (lane & 15) >> 2, gp = lane & 3, G = lane >> 4;
  if constexpr (PIPE) {
    // LDS-DMA staging (no VGPRs held across the tile): wave w fills 1-KiB blocks w, w + NW, ... of a tile
    // image; lane L of block bi writes row 4 bi + L / 16, slot L % 16, so it fetches the source chunk that
    // fa_off's swizzle puts in that slot
    auto Kr = [&](int i) { return lds + i * TILE_BYTES; };
    auto Vr = [&](int i) { return lds + (2 + i) * TILE_BYTES; };
    auto dma = [&](const bf16_t* src, int t0, char* dst) {
#pragma unroll
      for (int i = 0; i < 16 / NW; ++i) {
        const int bi = w + NW * i, row = 4 * bi + (lane >> 4);
        const int ch = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
        if constexpr (PIPE == 2)
          glds16_asm(src + (size_t)min(t0 + row, T - 1) * AP_DH + 8 * ch, dst + 1024 * bi);
        else
          glds16(src + (size_t)min(t0 + row, T - 1) * AP_DH + 8 * ch, dst + 1024 * bi);
      }
    };
    auto scores = [&](const char* Kt, f32x16 (&s)[2]) {
#pragma unroll
      for (int kbk = 0; kbk < 2; ++kbk) {
#pragma unroll
        for (int i = 0; i < 16; ++i) s[kbk][i] = 0.f;
#pragma unroll
        for (int ks = 0; ks < 8; ++ks)
          s[kbk] = mfma32(*reinterpret_cast<const u32x4*>(Kt + fa_off(32 * kbk + col, 2 * ks + hi)), qf[0][ks], s[kbk]);
      }
    };
    const int n_t = t_begin <= last_key ? (last_key - t_begin) / FA_KT + 1 : 0;
    const int qfirst = slot0 + p0, qslot = qfirst + col;
    f32x16 st[2];
    if (n_t > 0) {
      dma(kb, t_begin, Kr(0));
      dma(vb, t_begin, Vr(0));
    }
    if (n_t > 1) dma(kb, t_begin + FA_KT, Kr(1));
    wait_vmcnt<0>();
    __syncthreads();
    if (n_t > 0 && t_begin <= wave_last_slot) scores(Kr(0), st);
    // the first iteration's DMA of K(2) lands in K(0)'s slot: every wave must be done reading it
    if (n_t > 2) __syncthreads();
    for (int it = 0; it < n_t; ++it) {
      const int t0 = t_begin + it * FA_KT, cur = it & 1;
      const bool has1 = it + 1 < n_t, has2 = it + 2 < n_t;
      // K(i+2) into K(i)'s slot and V(i+1) into V(i-1)'s: both last read before the previous barrier
      if (has2) dma(kb, t0 + 2 * FA_KT, Kr(cur));
      if (has1) dma(vb, t0 + FA_KT, Vr(cur ^ 1));
      if (t0 <= wave_last_slot) {  // wave-uniform; every later tile is inactive too
        // masking (wave-uniform branch: only tiles crossing kv_start, the diagonal, T, or a key mask)
        const bool full = !mrow && t0 >= lo && t0 + FA_KT - 1 <= qfirst && t0 + FA_KT - 1 < T;
        if (!full) {
#pragma unroll
          for (int kbk = 0; kbk < 2; ++kbk)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int j = t0 + 32 * kbk + (i & 3) + 8 * (i >> 2) + 4 * hi;
              bool ok = j >= lo && j <= qslot && j < T;
              if (mrow) ok = ok && j < mask_len && mrow[j] != 0;
              st[kbk][i] = ok ? st[kbk][i] : -INFINITY;
            }
        }
        float tmax = -INFINITY;
#pragma unroll
        for (int kbk = 0; kbk < 2; ++kbk)
#pragma unroll
          for (int i = 0; i < 16; ++i) tmax = fmaxf(tmax, st[kbk][i]);
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64)) * scale_log2;  // scale > 0: max of the scaled scores
        if (__ballot(tmax > m_run[0] + 8.f)) {
          const float m_new = fmaxf(m_run[0], tmax);
          const float alpha = __builtin_amdgcn_exp2f(m_run[0] - (m_new == -INFINITY ? 0.f : m_new));
          l_run[0] *= alpha;
          m_run[0] = m_new;
#pragma unroll
          for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int i = 0; i < 16; ++i) o[0][dt][i] *= alpha;
        }
        const float m_use = m_run[0] == -INFINITY ? 0.f : m_run[0];
        // one straight-line block: S(i+1) on the matrix pipe beside exp / sum / pack of tile i (VALU), then
        // O += V(i) P(i); NEXT is a compile-time copy so no branch splits the MFMAs from the VALU work
        auto body = [&](auto NEXT) {
          f32x16 sn[2];
          if constexpr (decltype(NEXT)::value) {
            if constexpr (PIPE == 2) {
#pragma unroll
              for (int i = 0; i < 16; ++i) sn[0][i] = sn[1][i] = 0.f;
            } else {
              scores(Kr(cur ^ 1), sn);
            }
          }
          // key step s: 8 exps -> one P fragment -> its 4 PV MFMAs (one fragment live, exp beside the MFMAs)
          float rs = 0.f;
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            if constexpr (PIPE == 2) {
              // PIPE 2: a quarter of the next tile's scores (dk steps 2s, 2s + 1, both key blocks: 4 MFMAs on two
              // alternating accumulators) in each key step, fenced so the scheduler keeps them beside this step's
              // exps and PV MFMAs instead of sinking all 16 into a serial read -> wait -> MFMA chain at the end
              __builtin_amdgcn_sched_barrier(0);
              if constexpr (decltype(NEXT)::value) {
                const char* Kt = Kr(cur ^ 1);
#pragma unroll
                for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                  for (int kbk = 0; kbk < 2; ++kbk)
                    sn[kbk] = mfma32(*reinterpret_cast<const u32x4*>(Kt + fa_off(32 * kbk + col, 4 * s + 2 * kk + hi)),
                                     qf[0][2 * s + kk], sn[kbk]);
              }
            }
            float e[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              e[j] = __builtin_amdgcn_exp2f(fmaf(st[s >> 1][8 * (s & 1) + j], scale_log2, -m_use));
              rs += e[j];
            }
            const u32x4 pf = pack8(e);
            const int r0 = 16 * s + 4 * (G >> 1) + gq;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
              const int c0 = 4 * dt + 2 * (G & 1) + (gp >> 1);
              const u32x2 lo4 = ld_tr(Vr(cur), fa_off(r0, c0) + 8 * (gp & 1));
              const u32x2 hi4 = ld_tr(Vr(cur), fa_off(r0 + 8, c0) + 8 * (gp & 1));
              const u32x4 vf = {lo4[0], lo4[1], hi4[0], hi4[1]};
              o[0][dt] = mfma32(vf, pf, o[0][dt]);
            }
          }
          rs += __shfl_xor(rs, 32, 64);
          l_run[0] += rs;
          if constexpr (decltype(NEXT)::value) {
            st[0] = sn[0];
            st[1] = sn[1];
          }
        };
        // (the branch lets LLVM hoist the shared exp block above the scores MFMAs; a branch-free variant that always
        // runs the NEXT copy interleaves them but measured neutral: profiles/r3_attn_prefill_branchfree_ab.jsonl)
        // PIPE 2: branch-free (the next tile's scores always run; past the wave's last tile they read a settled stale
        // slot and are never used), so the exps stay in the fenced key steps beside the MFMAs
        if (PIPE == 2 || (has1 && t0 + FA_KT <= wave_last_slot))
          body(std::true_type{});
        else
          body(std::false_type{});
      }
      wait_vmcnt<0>();
      __syncthreads();
    }
  } else {
  if (t_begin <= last_key) {
    load_tile(t_begin);
    store_tile();
  }
  __syncthreads();
  for (int t0 = t_begin; t0 <= last_key; t0 += FA_KT) {
    const bool has_next = t0 + FA_KT <= last_key;
    if (has_next) load_tile(t0 + FA_KT);
    if (t0 <= wave_last_slot) {
      // ---- S^T = K Q^T (each K fragment feeds the QB query blocks)
      f32x16 st[QB][2];
#pragma unroll
      for (int kbk = 0; kbk < 2; ++kbk) {
#pragma unroll
        for (int qq = 0; qq < QB; ++qq)
#pragma unroll
          for (int i = 0; i < 16; ++i) st[qq][kbk][i] = 0.f;
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
          const u32x4 kf = *reinterpret_cast<const u32x4*>(Ks + fa_off(32 * kbk + col, 2 * ks + hi));
#pragma unroll
          for (int qq = 0; qq < QB; ++qq) st[qq][kbk] = mfma32(kf, qf[qq][ks], st[qq][kbk]);
        }
      }
      // ---- online softmax per query block (log2 domain); element (kbk, i) is key
      // t0 + 32 kbk + (i & 3) + 8 (i >> 2) + 4 hi
      u32x4 pf[QB][4];  // B fragments of P^T for the 4 key steps
#pragma unroll
      for (int qq = 0; qq < QB; ++qq) {
        const int qfirst = slot0 + p0 + 32 * qq, qslot = qfirst + col;
        const bool full = !mrow && t0 >= lo && t0 + FA_KT - 1 <= qfirst && t0 + FA_KT - 1 < T;
        float tmax = -INFINITY;
#pragma unroll
        for (int kbk = 0; kbk < 2; ++kbk)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            float v = st[qq][kbk][i] * scale_log2;
            if (!full) {
              const int j = t0 + 32 * kbk + (i & 3) + 8 * (i >> 2) + 4 * hi;
              bool ok = j >= lo && j <= qslot && j < T;
              if (mrow) ok = ok && j < mask_len && mrow[j] != 0;
              v = ok ? v : -INFINITY;
            }
            st[qq][kbk][i] = v;
            tmax = fmaxf(tmax, v);
          }
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        if (__ballot(tmax > m_run[qq] + 8.f)) {
          const float m_new = fmaxf(m_run[qq], tmax);
          const float alpha = __builtin_amdgcn_exp2f(m_run[qq] - (m_new == -INFINITY ? 0.f : m_new));
          l_run[qq] *= alpha;
          m_run[qq] = m_new;
#pragma unroll
          for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int i = 0; i < 16; ++i) o[qq][dt][i] *= alpha;
        }
        const float m_use = m_run[qq] == -INFINITY ? 0.f : m_run[qq];
        float rs = 0.f;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          float e[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            e[j] = __builtin_amdgcn_exp2f(st[qq][s >> 1][8 * (s & 1) + j] - m_use);
            rs += e[j];
          }
          pf[qq][s] = pack8(e);
        }
        rs += __shfl_xor(rs, 32, 64);
        l_run[qq] += rs;
      }
      // ---- O^T += V^T P^T; A element j of lane half hi = V[key 16 s + 8 (j >> 2) + 4 hi + (j & 3)][d]
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int c0 = 4 * dt + 2 * (G & 1) + (gp >> 1);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int r0 = 16 * s + 4 * (G >> 1) + gq;
          const u32x2 lo4 = ld_tr(Vs, fa_off(r0, c0) + 8 * (gp & 1));
          const u32x2 hi4 = ld_tr(Vs, fa_off(r0 + 8, c0) + 8 * (gp & 1));
          const u32x4 vf = {lo4[0], lo4[1], hi4[0], hi4[1]};
#pragma unroll
          for (int qq = 0; qq < QB; ++qq) o[qq][dt] = mfma32(vf, pf[qq][s], o[qq][dt]);
        }
      }
    }
    __syncthreads();  // every wave is done with this tile's LDS images
    if (has_next) {
      store_tile();
      __syncthreads();
    }
  }
  }  // !PIPE

  // ---- epilogue: lane (query pos, half hi) holds d = 32 dt + 8 g + 4 hi + (0..3) in o[dt][4 g .. 4 g + 3]
#pragma unroll
  for (int qq = 0; qq < QB; ++qq) {
    const int pos = p0 + 32 * qq + col;
    if (pos < S) {
      const float inv = l_run[qq] > 0.f ? 1.f / l_run[qq] : 0.f;
      bf16_t* dst = out + ((size_t)b * S + pos) * H * AP_DH + (size_t)h * AP_DH + 4 * hi;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          u32x2 pk;
          pk[0] = pack2bf(o[qq][dt][4 * g] * inv, o[qq][dt][4 * g + 1] * inv);
          pk[1] = pack2bf(o[qq][dt][4 * g + 2] * inv, o[qq][dt][4 * g + 3] * inv);
          *reinterpret_cast<u32x2*>(dst + 32 * dt + 8 * g) = pk;
        }
    }
  }
  }  // pass
}

// v2 launch with NW waves per workgroup: NW / rep position blocks (rep < NW) or NW of the rep q heads (rep >= NW) share
// each K/V tile the workgroup stages; `paired_only`: always the (heavy, light) pair per workgroup
template <int NW, int PIPE>
static void launch_prefill_v2(const bf16_t* q, const bf16_t* kc, const bf16_t* vc, const int32_t* slot,
                              const int32_t* kv_start, const uint8_t* key_mask, int mask_len, bf16_t* out, int B, int S,
                              int H, int Hkv, int T, int rep, bool paired_only, hipStream_t s) {
  const int npb = rep >= NW ? 1 : NW / rep;    // position blocks per workgroup
  const int hpw = NW / npb;                    // q heads per workgroup
  const int hgroups = rep / hpw;
  const float sl2 = 1.4426950408889634f / sqrtf((float)AP_DH);
  const int n_qb = (S + 32 * npb - 1) / (32 * npb);
  const int pairs = (n_qb + 1) / 2 * Hkv * hgroups * B;
  // fewer pairs than two workgroups per CU (B = 1 prefill): each half of a pair is its own workgroup, so a CU
  // holds two resident workgroups instead of one
  const bool split = !paired_only && pairs < 2 * 256;
  if (split) {
    attn_prefill_v2_kernel<NW, PIPE><<<dim3(2 * pairs, 1, 1), NW * 64, 0, s>>>(
        q, kc, vc, slot, kv_start, key_mask, mask_len, out, S, H, Hkv, T, sl2, npb, hgroups, n_qb, 1);
  } else {
    dim3 grid2((n_qb + 1) / 2, Hkv * hgroups, B);  // a (heavy, light) pair of query blocks per workgroup
    attn_prefill_v2_kernel<NW, PIPE><<<grid2, NW * 64, 0, s>>>(q, kc, vc, slot, kv_start, key_mask, mask_len, out, S,
                                                                H, Hkv, T, sl2, npb, hgroups, n_qb, 0);
  }
}

// impl (attn_prefill_set_impl, A/B): 2 = default dispatch; 7 = pipelined 4 waves, 8 = unpipelined 4 waves, 9 =
// pipelined 8 waves (paired), 13 = the same with asm LDS-DMA and the next tile's scores spread over the key steps
// (PIPE 2); 1 = the v1 kernel (also the fallback for a non-power-of-two GQA ratio)
static int g_attn_prefill_impl = 2;
void attn_prefill_set_impl(int impl) { g_attn_prefill_impl = impl; }

int attn_prefill(const bf16_t* q, const bf16_t* kc, const bf16_t* vc, const int32_t* slot, const int32_t* kv_start,
                 const uint8_t* key_mask, int mask_len, bf16_t* out, int B, int S, int H, int Hkv, int Dh, int T,
                 hipStream_t s) {
  if (B <= 0 || S <= 0) return 0;
  if (Dh != AP_DH || H % Hkv) return -1;
  const int rep = H / Hkv;
  const bool pow2rep = rep == 1 || rep == 2 || rep == 4 || rep == 8;
  int impl = g_attn_prefill_impl;
  // default (impl 2): the software-pipelined loop from S = 512 (a query block needs a few tiles to pipeline), with 8
  // waves per workgroup when that paired grid fills the CUs without exceeding ~4 workgroups per CU (256..1023
  // workgroups: twice the queries per staged K/V tile), else 4 waves; up to S = 256 the unpipelined 4-wave loop. Interleaved A/B
  // (profiles/r3_attn_prefill_pipe_ab.jsonl, TFLOP/s, previous default -> now): 8B B = 1 S = 2048 454 -> 509,
  // B = 16 S = 2048 672 -> 746, S = 8192 854 -> 903, B = 2048 S = 128 186 -> 198, 70B S = 2048 698 -> 733.
  // The 8-wave launch is PIPE 2 (impl 13) since round 4: bit-identical to impl 9, +1-5 % on the 8-wave shapes
  // (profiles/r4_attn_prefill_asm_dma_ab.jsonl).
  if (impl == 2 && pow2rep) {
    if (S <= 256) {
      impl = 8;
    } else {
      const int npb8 = rep >= 8 ? 1 : 8 / rep;
      const int n_qb8 = (S + 32 * npb8 - 1) / (32 * npb8);
      const int wg8 = (n_qb8 + 1) / 2 * Hkv * (rep / (8 / npb8)) * B;
      // 8 waves only for mid-sized grids: from 4 paired 8-wave workgroups per CU up, the 4-wave grid (twice the
      // workgroups, 2 resident per CU) measured faster or tied on 4 of 4 boxes (8B B = 16 S = 2048 747-784 vs 731-762
      // TFLOP/s, 7B MHA B = 16 661-687 vs 597-675; profiles/r4_attn_prefill_dispatch_ab.jsonl)
      impl = wg8 >= 256 && wg8 < 1024 ? 13 : 7;
    }
  }
  const int nw_impl = impl == 9 || impl == 13 ? 8 : 4;
  if ((impl == 7 || impl == 8 || impl == 9 || impl == 13) && (rep % nw_impl == 0 || nw_impl % rep == 0)) {
    if (impl == 7)
      launch_prefill_v2<4, 1>(q, kc, vc, slot, kv_start, key_mask, mask_len, out, B, S, H, Hkv, T, rep, false, s);
    else if (impl == 8)
      launch_prefill_v2<4, 0>(q, kc, vc, slot, kv_start, key_mask, mask_len, out, B, S, H, Hkv, T, rep, false, s);
    else if (impl == 9)
      launch_prefill_v2<8, 1>(q, kc, vc, slot, kv_start, key_mask, mask_len, out, B, S, H, Hkv, T, rep, true, s);
    else
      launch_prefill_v2<8, 2>(q, kc, vc, slot, kv_start, key_mask, mask_len, out, B, S, H, Hkv, T, rep, true, s);
    JLA_CHECK_LAUNCH();
    return 0;
  }
  dim3 grid((S + AP_QB - 1) / AP_QB, H, B);
  attn_prefill_kernel<<<grid, 256, 0, s>>>(q, kc, vc, slot, kv_start, key_mask, mask_len, out, S, H, Hkv, T,
                                           1.f / sqrtf((float)Dh));
  JLA_CHECK_LAUNCH();
  return 0;
}

JLA_BOUNDS_ACCESSOR(attn_prefill)

}  // namespace jla
