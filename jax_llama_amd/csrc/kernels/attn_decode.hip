// Decode attention (one query position per sequence) over the bf16 KV cache, split-KV + combine.
//
// Reference: FlaxLLaMAAttention with a cache (model.py:169-199 cache write/pad mask, :236-267 mask
// + bias, :269-270 repeat_kv, :277-291 softmax(QK^T/sqrt(Dh)) V). Here the mask is computed from
// (kv_start, slot, optional key mask) in-kernel, GQA is pure indexing (the REP query heads that
// share a kv head are processed by one workgroup so K/V are read from HBM once), and only keys
// [kv_start, slot] are touched (the reference attends over the whole cache length).
//
// Kernel 1: workgroup = (split, kv head, batch row), 4 waves, a chunk of CH keys.
//   Each 16-lane group owns one key row (16 lanes x 16 B = 256 B = Dh 128 bf16), so one wave-wide
//   load fetches 4 consecutive cache rows = 1 KiB contiguous. QK^T partial dots are reduced over
//   the 16 lanes, scores go to LDS, softmax stats per head, then P.V with the same row mapping.
//   Output: per (b, h, split) the running max m, the sum l and the unnormalised o[Dh] (fp32).
// Kernel 2: combine the splits (log-sum-exp merge) -> bf16 out[b, h*Dh].
// Rows with no valid key produce 0 (never NaN: -inf maxima are guarded).
#include "common.h"
#include "launchers.h"

namespace jla {

constexpr int AD_DH = 128;
constexpr int AD_WAVES = 4;

template <int REP>
__global__ void __launch_bounds__(AD_WAVES * 64)
    attn_decode_split_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc,
                             const bf16_t* __restrict__ vc, const int32_t* __restrict__ slot_ptr,
                             const int32_t* __restrict__ kv_start, const uint8_t* __restrict__ key_mask,
                             int mask_len, float* __restrict__ ws, int H, int Hkv, int T, int t_cap, int CH,
                             int nsplit, float scale) {
  extern __shared__ float smem[];
  float* sc = smem;                    // [REP][CH]
  float* ored = sc + REP * CH;         // [AD_WAVES][REP][AD_DH]
  float* stats = ored + AD_WAVES * REP * AD_DH;  // [REP][2]

  const int split = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int slot = slot_ptr[0];
  const int lo = kv_start[b];
  const int c0 = split * CH;
  const int c1 = min(c0 + CH, min(t_cap, slot + 1));
  const int h0 = kvh * REP;
  float* out_base = ws + ((size_t)b * H + h0) * nsplit * (AD_DH + 2);
  const size_t hstride = (size_t)nsplit * (AD_DH + 2);

  if (c0 >= c1 || c1 <= lo) {  // chunk entirely outside the valid range
    for (int i = threadIdx.x; i < REP * (AD_DH + 2); i += blockDim.x) {
      const int h = i / (AD_DH + 2), e = i - h * (AD_DH + 2);
      out_base[h * hstride + split * (AD_DH + 2) + e] = (e == 0) ? -INFINITY : 0.f;
    }
    return;
  }

  // q fragment for this lane's 8 dims, all REP heads, pre-scaled
  float qf[REP][8];
#pragma unroll
  for (int h = 0; h < REP; ++h) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(q + ((size_t)b * H + h0 + h) * AD_DH + 8 * li);
    unpack8(v, qf[h]);
#pragma unroll
    for (int e = 0; e < 8; ++e) qf[h][e] *= scale;
  }

  const bf16_t* kbase = kc + ((size_t)b * Hkv + kvh) * T * AD_DH + 8 * li;
  const bf16_t* vbase = vc + ((size_t)b * Hkv + kvh) * T * AD_DH + 8 * li;
  const uint8_t* mrow = key_mask ? key_mask + (size_t)b * mask_len : nullptr;
  const int nkeys = c1 - c0;

  // ---- scores
  for (int jl0 = w * 4; jl0 < nkeys; jl0 += AD_WAVES * 4 * 2) {
    u32x4 kv[2];
    int jj[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      jj[u] = jl0 + u * AD_WAVES * 4 + g;
      const int j = c0 + min(jj[u], nkeys - 1);
      kv[u] = *reinterpret_cast<const u32x4*>(kbase + (size_t)j * AD_DH);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float kf[8];
      unpack8(kv[u], kf);
      const int j = c0 + jj[u];
      bool valid = jj[u] < nkeys && j >= lo;
      if (mrow && j < mask_len) valid = valid && mrow[j] != 0;
#pragma unroll
      for (int h = 0; h < REP; ++h) {
        float d = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) d += qf[h][e] * kf[e];
        d += __shfl_xor(d, 1, 64);
        d += __shfl_xor(d, 2, 64);
        d += __shfl_xor(d, 4, 64);
        d += __shfl_xor(d, 8, 64);
        if (li == 0 && jj[u] < nkeys) sc[h * CH + jj[u]] = valid ? d : -INFINITY;
      }
    }
  }
  __syncthreads();

  // ---- softmax stats per head (wave h handles heads h, h+4, ...)
  for (int h = w; h < REP; h += AD_WAVES) {
    float m = -INFINITY;
    for (int j = lane; j < nkeys; j += 64) m = fmaxf(m, sc[h * CH + j]);
    m = wave_max(m);
    float l = 0.f;
    for (int j = lane; j < nkeys; j += 64) {
      const float s = sc[h * CH + j];
      const float p = (m == -INFINITY) ? 0.f : __expf(s - m);
      sc[h * CH + j] = p;
      l += p;
    }
    l = wave_sum(l);
    if (lane == 0) {
      stats[2 * h] = m;
      stats[2 * h + 1] = l;
    }
  }
  __syncthreads();

  // ---- P.V
  float o[REP][8];
#pragma unroll
  for (int h = 0; h < REP; ++h)
#pragma unroll
    for (int e = 0; e < 8; ++e) o[h][e] = 0.f;
  for (int jl0 = w * 4; jl0 < nkeys; jl0 += AD_WAVES * 4 * 2) {
    u32x4 vv[2];
    int jj[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      jj[u] = jl0 + u * AD_WAVES * 4 + g;
      const int j = c0 + min(jj[u], nkeys - 1);
      vv[u] = *reinterpret_cast<const u32x4*>(vbase + (size_t)j * AD_DH);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (jj[u] < nkeys) {
        float vf[8];
        unpack8(vv[u], vf);
#pragma unroll
        for (int h = 0; h < REP; ++h) {
          const float p = sc[h * CH + jj[u]];
#pragma unroll
          for (int e = 0; e < 8; ++e) o[h][e] += p * vf[e];
        }
      }
    }
  }
#pragma unroll
  for (int h = 0; h < REP; ++h)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = o[h][e];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      o[h][e] = v;
    }
  if (g == 0) {
#pragma unroll
    for (int h = 0; h < REP; ++h)
#pragma unroll
      for (int e = 0; e < 8; ++e) ored[(w * REP + h) * AD_DH + 8 * li + e] = o[h][e];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < REP * AD_DH; i += blockDim.x) {
    const int h = i / AD_DH, d = i - h * AD_DH;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < AD_WAVES; ++ww) v += ored[(ww * REP + h) * AD_DH + d];
    float* dst = out_base + h * hstride + split * (AD_DH + 2);
    dst[2 + d] = v;
    if (d == 0) {
      dst[0] = stats[2 * h];
      dst[1] = stats[2 * h + 1];
    }
  }
}

__global__ void __launch_bounds__(AD_DH)
    attn_decode_combine_kernel(const float* __restrict__ ws, bf16_t* __restrict__ out, int nsplit) {
  const int bh = blockIdx.x, d = threadIdx.x;
  const float* src = ws + (size_t)bh * nsplit * (AD_DH + 2);
  float M = -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, src[s * (AD_DH + 2)]);
  float num = 0.f, den = 0.f;
  if (M != -INFINITY) {
    for (int s = 0; s < nsplit; ++s) {
      const float m = src[s * (AD_DH + 2)];
      if (m == -INFINITY) continue;
      const float f = __expf(m - M);
      den += f * src[s * (AD_DH + 2) + 1];
      num += f * src[s * (AD_DH + 2) + 2 + d];
    }
  }
  out[(size_t)bh * AD_DH + d] = f2bf(den > 0.f ? num / den : 0.f);
}

int attn_decode_chunk(int B, int Hkv, int T) {
  int ch = 64;
  while (ch < 256 && ch < T && (long)B * Hkv * ((T + ch - 1) / ch) > 1024) ch *= 2;
  return ch;
}

int attn_decode_splits(int B, int Hkv, int T) {
  const int ch = attn_decode_chunk(B, Hkv, T);
  return (T + ch - 1) / ch;
}

int attn_decode(const bf16_t* q, const bf16_t* kc, const bf16_t* vc, const int32_t* slot, const int32_t* kv_start,
                const uint8_t* key_mask, int mask_len, bf16_t* out, float* ws, int B, int H, int Hkv, int Dh, int T,
                int t_cap, int nsplit, hipStream_t s) {
  if (B <= 0) return 0;
  if (Dh != AD_DH || H % Hkv) return -1;
  const int rep = H / Hkv;
  const int ch = attn_decode_chunk(B, Hkv, t_cap);
  if ((t_cap + ch - 1) / ch != nsplit) return -2;
  const float scale = 1.f / sqrtf((float)Dh);
  dim3 grid(nsplit, Hkv, B);
  const size_t lds = sizeof(float) * (rep * ch + AD_WAVES * rep * AD_DH + 2 * rep);
#define JLA_AD(R)                                                                                             \
  case R:                                                                                                    \
    attn_decode_split_kernel<R><<<grid, AD_WAVES * 64, lds, s>>>(q, kc, vc, slot, kv_start, key_mask, mask_len, \
                                                                 ws, H, Hkv, T, t_cap, ch, nsplit, scale);       \
    break;
  switch (rep) {
    JLA_AD(1)
    JLA_AD(2)
    JLA_AD(4)
    JLA_AD(8)
    JLA_AD(16)
    default: return -1;
  }
#undef JLA_AD
  JLA_CHECK_LAUNCH();
  attn_decode_combine_kernel<<<B * H, AD_DH, 0, s>>>(ws, out, nsplit);
  JLA_CHECK_LAUNCH();
  return 0;
}

}  // namespace jla
