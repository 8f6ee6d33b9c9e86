// Decode attention (one query position per sequence) over the bf16 KV cache, one pass, split-KV.
//
// Reference: FlaxLLaMAAttention with a cache (model.py:169-199 cache write/pad mask, :236-267 mask
// + bias, :269-270 repeat_kv, :277-291 softmax(QK^T/sqrt(Dh)) V). Here the mask is computed from
// (kv_start, slot, optional key mask) in-kernel, GQA is pure indexing (the REP query heads that
// share a kv head are processed by one workgroup so K/V are read from HBM once), and only keys
// [kv_start, slot] are touched (the reference attends over the whole cache length).
//
// Workgroup = (split, kv head, batch row): 4 waves, CH = 16*KPG keys. Each 16-lane group owns KPG
// key rows (16 lanes x 16 B = one 256 B row of Dh = 128 bf16); rows are interleaved across groups
// so one wave-wide load fetches 4 consecutive cache rows (1 KiB contiguous). ALL K and V rows of
// the chunk are issued up front (one memory round trip per workgroup), then QK^T (16-lane
// reductions), softmax (wave + LDS max/sum), P.V in registers, and a cross-wave LDS reduction.
// With nsplit > 1 each split publishes (m, l, o[Dh]) with write-through stores and bumps a
// per-(b, kv head) ticket; the last arriver merges the splits (log-sum-exp) and writes bf16 out,
// so decode attention is ONE launch (release/acquire recipe: cdna_hip_programming.md Guideline 16,
// sc1-store / sc1-load form; the last arriver resets the ticket for the next replay).
// Rows with no valid key produce 0 (never NaN: -inf maxima are guarded).
#include "common.h"
#include "launchers.h"

namespace jla {

constexpr int AD_DH = 128;
constexpr int AD_WAVES = 4;

JLA_DEV void st_wt(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
JLA_DEV float ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int REP, int KPG>
__global__ void __launch_bounds__(AD_WAVES * 64)
    attn_decode_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                       const int32_t* __restrict__ slot_ptr, const int32_t* __restrict__ kv_start,
                       const uint8_t* __restrict__ key_mask, int mask_len, bf16_t* __restrict__ out,
                       float* __restrict__ ws, int32_t* __restrict__ tickets, int H, int Hkv, int T, int t_cap,
                       int nsplit, float scale) {
  constexpr int CH = 16 * KPG;
  __shared__ float red_m[AD_WAVES][REP];
  __shared__ float red_l[AD_WAVES][REP];
  __shared__ float red_o[AD_WAVES][REP][AD_DH];
  __shared__ int last_flag;

  const int split = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int slot = slot_ptr[0];
  const int lo = kv_start[b];
  const int c0 = split * CH;
  const int c1 = min(c0 + CH, min(t_cap, slot + 1));  // keys [c0, c1) of this split
  const int h0 = kvh * REP;
  const uint8_t* mrow = key_mask ? key_mask + (size_t)b * mask_len : nullptr;
  const bool any = c0 < c1 && c1 > lo;

  float m_h[REP], l_h[REP];
  float o[REP][8];
#pragma unroll
  for (int h = 0; h < REP; ++h) {
    m_h[h] = -INFINITY;
    l_h[h] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[h][e] = 0.f;
  }

  if (any) {
    // ---- issue every K and V row of the chunk (clamped rows for keys past the end: masked)
    const size_t head_off = ((size_t)b * Hkv + kvh) * T * AD_DH + 8 * li;
    u32x4 kr[KPG], vr[KPG];
    int jv[KPG];
#pragma unroll
    for (int r = 0; r < KPG; ++r) {
      const int j = c0 + w * 4 + g + 16 * r;
      jv[r] = j;
      const int jc = min(j, c1 - 1);
      kr[r] = *reinterpret_cast<const u32x4*>(kc + head_off + (size_t)jc * AD_DH);
    }
#pragma unroll
    for (int r = 0; r < KPG; ++r) {
      const int jc = min(jv[r], c1 - 1);
      vr[r] = *reinterpret_cast<const u32x4*>(vc + head_off + (size_t)jc * AD_DH);
    }
    // q for this lane's 8 dims (pre-scaled by 1/sqrt(Dh))
    float qf[REP][8];
#pragma unroll
    for (int h = 0; h < REP; ++h) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(q + ((size_t)b * H + h0 + h) * AD_DH + 8 * li);
      unpack8(v, qf[h]);
#pragma unroll
      for (int e = 0; e < 8; ++e) qf[h][e] *= scale;
    }
    // ---- scores (every lane of a 16-lane group ends with the full dot product)
    float sc[REP][KPG];
#pragma unroll
    for (int r = 0; r < KPG; ++r) {
      float kf[8];
      unpack8(kr[r], kf);
      const int j = jv[r];
      bool valid = j < c1 && j >= lo;
      if (mrow && j < mask_len) valid = valid && mrow[j] != 0;
#pragma unroll
      for (int h = 0; h < REP; ++h) {
        float d = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) d += qf[h][e] * kf[e];
        d = row16_sum(d);  // DPP: every lane of the 16-lane row gets the full dot product
        sc[h][r] = valid ? d : -INFINITY;
      }
    }
    // ---- per-head max over the chunk: registers -> 4 groups (xor 16, 32) -> 4 waves (LDS)
#pragma unroll
    for (int h = 0; h < REP; ++h) {
      float mx = sc[h][0];
#pragma unroll
      for (int r = 1; r < KPG; ++r) mx = fmaxf(mx, sc[h][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      m_h[h] = mx;
    }
    if (lane == 0) {
#pragma unroll
      for (int h = 0; h < REP; ++h) red_m[w][h] = m_h[h];
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < REP; ++h) {
      float mx = red_m[0][h];
#pragma unroll
      for (int ww = 1; ww < AD_WAVES; ++ww) mx = fmaxf(mx, red_m[ww][h]);
      m_h[h] = mx;
    }
    // ---- p = exp(s - m); P.V into this lane's 8 dims
#pragma unroll
    for (int r = 0; r < KPG; ++r) {
      float vf[8];
      unpack8(vr[r], vf);
#pragma unroll
      for (int h = 0; h < REP; ++h) {
        const float p = (sc[h][r] == -INFINITY) ? 0.f : __expf(sc[h][r] - m_h[h]);
        l_h[h] += p;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[h][e] += p * vf[e];
      }
    }
    // l: each key's p was added by all 16 lanes of its group -> sum over groups, count once
#pragma unroll
    for (int h = 0; h < REP; ++h) {
      float l = l_h[h];
      l += __shfl_xor(l, 16, 64);
      l += __shfl_xor(l, 32, 64);
      l_h[h] = l;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float v = o[h][e];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        o[h][e] = v;
      }
    }
    if (g == 0) {
#pragma unroll
      for (int h = 0; h < REP; ++h) {
#pragma unroll
        for (int e = 0; e < 8; ++e) red_o[w][h][8 * li + e] = o[h][e];
        if (li == 0) red_l[w][h] = l_h[h];
      }
    }
    __syncthreads();
  }

  // ---- this split's (m, l, o) per head: thread t -> (head, d)
  float* part = ws + (((size_t)b * Hkv + kvh) * nsplit + split) * REP * (AD_DH + 2);
  for (int i = threadIdx.x; i < REP * AD_DH; i += AD_WAVES * 64) {
    const int h = i / AD_DH, d = i - h * AD_DH;
    float ov = 0.f, lv = 0.f, mv = -INFINITY;
    if (any) {
#pragma unroll
      for (int ww = 0; ww < AD_WAVES; ++ww) {
        ov += red_o[ww][h][d];
        lv += red_l[ww][h];
      }
      mv = m_h[h];
    }
    if (nsplit == 1) {
      out[((size_t)b * H + h0 + h) * AD_DH + d] = f2bf(lv > 0.f ? ov / lv : 0.f);
    } else {
      st_wt(part + h * (AD_DH + 2) + 2 + d, ov);
      if (d == 0) {
        st_wt(part + h * (AD_DH + 2), mv);
        st_wt(part + h * (AD_DH + 2) + 1, lv);
      }
    }
  }
  if (nsplit == 1) return;

  // ---- publish: every storing wave drains its write-through stores, then one ticket add
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t* tk = tickets + (size_t)b * Hkv + kvh;
    const int prev = __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == nsplit - 1;
    if (last) __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // reset for next replay
    last_flag = last;
  }
  __syncthreads();
  if (!last_flag) return;

  // ---- last arriver: merge all splits of this (b, kv head) with sc1 loads, in parallel:
  // (1) every (split, head) max/sum loaded by its own thread, (2) per-head weights in LDS,
  // (3) each (head, d) thread sums the splits' o with independent loads (8 in flight).
  const float* base = ws + ((size_t)b * Hkv + kvh) * nsplit * REP * (AD_DH + 2);
  float* wsh = &red_o[0][0][0];  // reuse: [nsplit][REP] weights (nsplit * REP <= 4 * REP * 128)
  for (int i = threadIdx.x; i < nsplit * REP; i += AD_WAVES * 64) wsh[i] = ld_wt(base + (size_t)i * (AD_DH + 2));
  __syncthreads();
  if (threadIdx.x < REP) {
    const int h = threadIdx.x;
    float M = -INFINITY;
    for (int s = 0; s < nsplit; ++s) M = fmaxf(M, wsh[s * REP + h]);
    red_m[0][h] = M;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nsplit * REP; i += AD_WAVES * 64) {
    const float M = red_m[0][i % REP], m = wsh[i];
    wsh[i] = (m == -INFINITY || M == -INFINITY) ? 0.f : __expf(m - M);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < REP * AD_DH; i += AD_WAVES * 64) {
    const int h = i / AD_DH, d = i - h * AD_DH;
    float num = 0.f, den = 0.f;
    int s = 0;
    for (; s + 8 <= nsplit; s += 8) {
      float ov[8], lv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float* ps = base + ((size_t)(s + q) * REP + h) * (AD_DH + 2);
        lv[q] = ld_wt(ps + 1);
        ov[q] = ld_wt(ps + 2 + d);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float f = wsh[(s + q) * REP + h];
        den += f * lv[q];
        num += f * ov[q];
      }
    }
    for (; s < nsplit; ++s) {
      const float* ps = base + ((size_t)s * REP + h) * (AD_DH + 2);
      const float f = wsh[s * REP + h];
      den += f * ld_wt(ps + 1);
      num += f * ld_wt(ps + 2 + d);
    }
    out[((size_t)b * H + h0 + h) * AD_DH + d] = f2bf(den > 0.f ? num / den : 0.f);
  }
}

static int kpg_for(int rep) { return rep <= 4 ? 8 : (rep == 8 ? 4 : 2); }

int attn_decode_chunk(int B, int Hkv, int T, int rep) { return 16 * kpg_for(rep); }

int attn_decode_splits(int B, int Hkv, int T, int rep) {
  const int ch = attn_decode_chunk(B, Hkv, T, rep);
  return (T + ch - 1) / ch;
}

int attn_decode(const bf16_t* q, const bf16_t* kc, const bf16_t* vc, const int32_t* slot, const int32_t* kv_start,
                const uint8_t* key_mask, int mask_len, bf16_t* out, float* ws, int32_t* tickets, int B, int H,
                int Hkv, int Dh, int T, int t_cap, int nsplit, hipStream_t s) {
  if (B <= 0) return 0;
  if (Dh != AD_DH || H % Hkv) return -1;
  const int rep = H / Hkv;
  if (attn_decode_splits(B, Hkv, t_cap, rep) != nsplit) return -2;
  const float scale = 1.f / sqrtf((float)Dh);
  dim3 grid(nsplit, Hkv, B);
#define JLA_AD(R)                                                                                              \
  case R:                                                                                                     \
    attn_decode_kernel<R, (R <= 4 ? 8 : (R == 8 ? 4 : 2))><<<grid, AD_WAVES * 64, 0, s>>>(                     \
        q, kc, vc, slot, kv_start, key_mask, mask_len, out, ws, tickets, H, Hkv, T, t_cap, nsplit, scale);     \
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
  return 0;
}

}  // namespace jla
