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

int attn_prefill(const bf16_t* q, const bf16_t* kc, const bf16_t* vc, const int32_t* slot, const int32_t* kv_start,
                 const uint8_t* key_mask, int mask_len, bf16_t* out, int B, int S, int H, int Hkv, int Dh, int T,
                 hipStream_t s) {
  if (B <= 0 || S <= 0) return 0;
  if (Dh != AP_DH || H % Hkv) return -1;
  dim3 grid((S + AP_QB - 1) / AP_QB, H, B);
  attn_prefill_kernel<<<grid, 256, 0, s>>>(q, kc, vc, slot, kv_start, key_mask, mask_len, out, S, H, Hkv, T,
                                           1.f / sqrtf((float)Dh));
  JLA_CHECK_LAUNCH();
  return 0;
}

}  // namespace jla
