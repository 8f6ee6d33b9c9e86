// Decode attention (one query position per sequence) over the bf16 KV cache, one pass.
//
// Reference: FlaxLLaMAAttention with a cache (model.py:169-199 cache write/pad mask, :236-267 mask
// + bias, :269-270 repeat_kv, :277-291 softmax(QK^T/sqrt(Dh)) V). Here the mask is computed from
// (kv_start, slot, optional key mask) in-kernel, GQA is pure indexing (the REP query heads that
// share a kv head are processed together so K/V are read from HBM once), and only keys
// [kv_start, slot] are touched (the reference attends over the whole cache length).
//
// One kernel per regime (attn_decode below picks by (row, kv head) pairs and query heads per kv head, REP):
//   v5  split small batch, <= 64 pairs (<= 256 at REP >= 8)   -- the latency-bound B = 1..8 steps
//   v6  matrix-core scores / P.V, REP >= 8 and 8..2047 pairs  -- the 70B tensor-parallel shard (attn_decode_mma.hip)
//   v3  one workgroup per pair, up to 4096 pairs (REP <= 8)    -- mid batches
//   v4  one wave per pair, register ring, one split, no key mask -- large batches (the B = 2048 headline)
//   v2  one wave per (pair, key split), LDS ring, optional key mask -- large batches with a padding mask, and the
//       fallback for every other shape (REP 16 mid batches)
// With splits, each split publishes (m, l, o[Dh]) with write-through stores and bumps a per-pair ticket; the last
// arriver merges the splits (log-sum-exp), so decode attention is ONE launch (cdna_hip_programming.md Guideline 16,
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

// ---------------------------------------------------------------------------------------------
// v3 (small batch): ONE workgroup per (batch row, kv head) and no cross-workgroup merge.
//
// At B <= 64 the decode attention moves well under a MiB and a split kernel's critical path is latency: load ->
// score -> publish partials -> ticket -> last arriver reloads every split -> merge (~10 us at B = 1
// whatever the split count: profiles/r2_attn_decode_small_batch_ab.jsonl). Here 8 waves split the
// valid keys [kv_start, slot] into interleaved 16-lane rows (chunk of 32 * KPG keys per step, the next
// chunk's K/V loads issued before the current chunk is scored), every wave keeps its own running
// (max, sum, o) per query head (online softmax, no barrier in the loop), and the 8 waves merge once
// through LDS. Rows with no valid key output 0.
constexpr int AD3_WAVES = 8;

template <int REP, int KPG>
__global__ void __launch_bounds__(AD3_WAVES * 64)
    attn_decode_v3_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                          const int32_t* __restrict__ slot_ptr, const int32_t* __restrict__ kv_start,
                          const uint8_t* __restrict__ key_mask, int mask_len, bf16_t* __restrict__ out, int H,
                          int Hkv, int T, int t_cap, float scale, bf16_t* __restrict__ out_pack) {
  constexpr int CH = AD3_WAVES * 4 * KPG;  // keys per chunk (8 waves x 4 groups x KPG rows)
  __shared__ float sm_m[AD3_WAVES][REP];
  __shared__ float sm_l[AD3_WAVES][REP];
  __shared__ float sm_o[AD3_WAVES][REP][AD_DH];

  const int kvh = blockIdx.x, b = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int slot = slot_ptr[0];
  if (slot >= T && threadIdx.x == 0) JLA_FLAG(JLA_BOUNDS_ATTN_T);  // keys past the cache are never read
  const int lo = kv_start[b];
  const int hi_key = min(slot + 1, t_cap);  // keys [lo, hi_key)
  const int h0 = kvh * REP;
  const uint8_t* mrow = key_mask ? key_mask + (size_t)b * mask_len : nullptr;
  const size_t head_off = ((size_t)b * Hkv + kvh) * T * AD_DH + 8 * li;

  float qf[REP][8];
#pragma unroll
  for (int h = 0; h < REP; ++h) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(q + ((size_t)b * H + h0 + h) * AD_DH + 8 * li);
    unpack8(v, qf[h]);
#pragma unroll
    for (int e = 0; e < 8; ++e) qf[h][e] *= scale;
  }
  float m_h[REP], l_h[REP], o[REP][8];
#pragma unroll
  for (int h = 0; h < REP; ++h) {
    m_h[h] = -INFINITY;
    l_h[h] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[h][e] = 0.f;
  }

  const int c_begin = lo - (lo % CH);
  // row r of this lane's group in chunk c0: key c0 + 32 r + 4 w + g (one wave load = 4 consecutive rows)
  u32x4 kr[KPG], vr[KPG];
  auto load = [&](int c0) {
#pragma unroll
    for (int r = 0; r < KPG; ++r) {
      const int j = min(max(c0 + 32 * r + 4 * w + g, 0), hi_key - 1);
      kr[r] = *reinterpret_cast<const u32x4*>(kc + head_off + (size_t)j * AD_DH);
      vr[r] = *reinterpret_cast<const u32x4*>(vc + head_off + (size_t)j * AD_DH);
    }
  };
  if (c_begin < hi_key && lo < hi_key) load(c_begin);
  for (int c0 = c_begin; c0 < hi_key && lo < hi_key; c0 += CH) {
    u32x4 kcur[KPG], vcur[KPG];
#pragma unroll
    for (int r = 0; r < KPG; ++r) {
      kcur[r] = kr[r];
      vcur[r] = vr[r];
    }
    if (c0 + CH < hi_key) load(c0 + CH);  // next chunk in flight while this one is scored
    float sc[REP][KPG];
#pragma unroll
    for (int r = 0; r < KPG; ++r) {
      const int j = c0 + 32 * r + 4 * w + g;
      bool valid = j >= lo && j < hi_key;
      if (mrow) valid = valid && j < mask_len && mrow[j] != 0;
      float kf[8];
      unpack8(kcur[r], kf);
#pragma unroll
      for (int h = 0; h < REP; ++h) {
        float d = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) d += qf[h][e] * kf[e];
        d = row16_sum(d);
        sc[h][r] = valid ? d : -INFINITY;
      }
    }
#pragma unroll
    for (int h = 0; h < REP; ++h) {
      float mx = sc[h][0];
#pragma unroll
      for (int r = 1; r < KPG; ++r) mx = fmaxf(mx, sc[h][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m_h[h], mx);
      if (mn == -INFINITY) continue;  // nothing valid for this wave yet (wave-uniform)
      const float alpha = __expf(m_h[h] - mn);  // m_h = -inf -> 0
      l_h[h] *= alpha;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[h][e] *= alpha;
      m_h[h] = mn;
#pragma unroll
      for (int r = 0; r < KPG; ++r) {
        const float p = sc[h][r] == -INFINITY ? 0.f : __expf(sc[h][r] - mn);
        l_h[h] += p;  // the 16 lanes of a group hold the same p (and the same running sum)
        float vf[8];
        unpack8(vcur[r], vf);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[h][e] += p * vf[e];
      }
    }
  }
  // ---- per wave: sum the 4 groups (same max), then merge the 8 waves through LDS
#pragma unroll
  for (int h = 0; h < REP; ++h) {
    float l = l_h[h];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = o[h][e];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      o[h][e] = v;
    }
    if (g == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) sm_o[w][h][8 * li + e] = o[h][e];
      if (li == 0) {
        sm_m[w][h] = m_h[h];
        sm_l[w][h] = l;  // sum over the 4 groups (lanes li, li + 16, li + 32, li + 48)
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < REP * AD_DH; i += AD3_WAVES * 64) {
    const int h = i / AD_DH, d = i - h * AD_DH;
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < AD3_WAVES; ++ww) M = fmaxf(M, sm_m[ww][h]);
    float num = 0.f, den = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int ww = 0; ww < AD3_WAVES; ++ww) {
        const float mw = sm_m[ww][h];
        const float f = mw == -INFINITY ? 0.f : __expf(mw - M);
        num += f * sm_o[ww][h][d];
        den += f * sm_l[ww][h];
      }
    }
    const bf16_t r = f2bf(den > 0.f ? num / den : 0.f);
    out[((size_t)b * H + h0 + h) * AD_DH + d] = r;
    if (out_pack) out_pack[pack_off(b, (h0 + h) * AD_DH + d, H * AD_DH)] = r;  // the o projection's packed x
  }
}

// ---------------------------------------------------------------------------------------------
// v5 (small batch, split over keys): v3 runs a whole (row, kv head) pair on ONE workgroup, so at B x Hkv << CUs the
// pair's scoring is compute-bound on one CU (Llama-3-70B at MP 8, B = 1: 8 q heads x ~200 keys on a single CU,
// 13 us per layer in the decode trace). Here the valid keys [kv_start, slot] are cut into CH-key splits, one
// 4-wave workgroup each (every K / V row of the split issued at once: one memory round trip), scores by v_dot2,
// a per-wave online softmax, one LDS merge of the 4 waves; a split publishes its (m, l, o) with write-through (sc1)
// 16-B stores and takes the pair's agent-scope ticket, and the last arriver merges the splits in split order
// (sc1 loads; cdna_hip_programming.md Guideline 16 R1 form) and writes the output (+ the packed copy for the o
// projection). Splits outside the valid key range exit at once (the grid covers the whole cache, the valid range is
// device state), so the ticket counts only the active splits; a pair with one active split writes directly.
constexpr int AD5_WAVES = 4;
// splits the last arriver merges per round (all of a round's partial loads in flight together): 4 or 12; by default
// 12 from 16 (row, kv head) pairs on (70B MP 8 B = 32 T = 384: 13.9 -> 12.8 us) and 4 below (B = 1: 8.8 vs 9.4 us;
// profiles/r3_attn_decode_v5_fold_ab.jsonl). attn_set_v5_fold(4 / 12) pins one (A/B), 0 = by pairs.
static int g_attn_v5_fold = 0;
void attn_set_v5_fold(int n) { g_attn_v5_fold = (n == 4 || n == 12) ? n : 0; }
static int g_attn_v5_max_pairs = 64;  // v5 up to this many (row, kv head) pairs (0: off)
void attn_set_v5_max_pairs(int n) { g_attn_v5_max_pairs = n < 0 ? 64 : n; }
static int kpg5(int rep) { return rep >= 16 ? 1 : (rep == 8 ? 2 : (rep == 4 ? 4 : 8)); }

template <int REP, int KPG, int AD5_FOLD>
__global__ void __launch_bounds__(AD5_WAVES * 64)
    attn_decode_v5_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                          const int32_t* __restrict__ slot_ptr, const int32_t* __restrict__ kv_start,
                          const uint8_t* __restrict__ key_mask, int mask_len, bf16_t* __restrict__ out,
                          float* __restrict__ ws, int32_t* __restrict__ tickets, int H, int Hkv, int T, int t_cap,
                          int nsplit, float scale, bf16_t* __restrict__ out_pack) {
  constexpr int CH = AD5_WAVES * 4 * KPG;     // keys per split
  constexpr int HS = AD_DH + 4;               // floats per head of a partial: [m, l, 0, 0, o[128]]
  constexpr int PS = REP * HS;                // floats per split partial
  __shared__ float sm_m[AD5_WAVES][REP];
  __shared__ float sm_l[AD5_WAVES][REP];
  __shared__ float sm_o[AD5_WAVES][REP][AD_DH];
  __shared__ int last_flag;

  const int split = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int slot = slot_ptr[0];
  if (slot >= T && threadIdx.x == 0) JLA_FLAG(JLA_BOUNDS_ATTN_T);  // keys past the cache are never read
  const int lo = kv_start[b];
  const int hi = min(slot + 1, t_cap);  // valid keys [lo, hi)
  const int s_lo = lo / CH, s_hi = hi > lo ? (hi + CH - 1) / CH : s_lo;
  const int n_act = s_hi - s_lo;
  const int h0 = kvh * REP;
  const int HD = H * AD_DH;
  auto store_out = [&](int h, int d, const float* v) {  // 4 consecutive dims of head h
    bf16_t* o = out + ((size_t)b * H + h0 + h) * AD_DH + d;
    u32x2 pk;
    pk[0] = pack2bf(v[0], v[1]);
    pk[1] = pack2bf(v[2], v[3]);
    *reinterpret_cast<u32x2*>(o) = pk;
    if (out_pack) *reinterpret_cast<u32x2*>(out_pack + pack_off(b, (h0 + h) * AD_DH + d, HD)) = pk;
  };
  if (n_act <= 0) {  // no valid key for this row: 0 (never NaN), written once
    if (split == 0)
      for (int it = threadIdx.x; it < REP * 32; it += AD5_WAVES * 64) {
        const float z[4] = {0.f, 0.f, 0.f, 0.f};
        store_out(it >> 5, 4 * (it & 31), z);
      }
    return;
  }
  if (split < s_lo || split >= s_hi) return;

  // ---- every K and V row of the split, then q (rows past the valid range re-read a valid one: masked)
  const int c0 = split * CH;
  const size_t head_off = ((size_t)b * Hkv + kvh) * T * AD_DH + 8 * li;
  u32x4 kr[KPG], vr[KPG], qv[REP];
#pragma unroll
  for (int r = 0; r < KPG; ++r) {
    const int jc = min(max(c0 + 16 * r + 4 * w + g, lo), hi - 1);
    kr[r] = *reinterpret_cast<const u32x4*>(kc + head_off + (size_t)jc * AD_DH);
  }
#pragma unroll
  for (int r = 0; r < KPG; ++r) {
    const int jc = min(max(c0 + 16 * r + 4 * w + g, lo), hi - 1);
    vr[r] = *reinterpret_cast<const u32x4*>(vc + head_off + (size_t)jc * AD_DH);
  }
#pragma unroll
  for (int h = 0; h < REP; ++h) qv[h] = *reinterpret_cast<const u32x4*>(q + ((size_t)b * H + h0 + h) * AD_DH + 8 * li);
  const uint8_t* mrow = key_mask ? key_mask + (size_t)b * mask_len : nullptr;

  // ---- scores (v_dot2 over the lane's 8 dims, 16-lane DPP sum: every lane of the group gets the score)
  float sc[REP][KPG];
#pragma unroll
  for (int r = 0; r < KPG; ++r) {
    const int j = c0 + 16 * r + 4 * w + g;
    bool valid = j >= lo && j < hi;
    if (mrow) valid = valid && j < mask_len && mrow[j] != 0;
#pragma unroll
    for (int h = 0; h < REP; ++h) {
      const float d = row16_sum(dot8_bf16(qv[h], kr[r], 0.f)) * scale;
      sc[h][r] = valid ? d : -INFINITY;
    }
  }
  // ---- per wave: max, p = exp(s - m), l, o = P.V over the lane's 8 dims; the 4 groups summed by shuffles
#pragma unroll
  for (int h = 0; h < REP; ++h) {
    float mx = sc[h][0];
#pragma unroll
    for (int r = 1; r < KPG; ++r) mx = fmaxf(mx, sc[h][r]);
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float l = 0.f, o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (mx != -INFINITY) {  // wave-uniform
#pragma unroll
      for (int r = 0; r < KPG; ++r) {
        const float p = sc[h][r] == -INFINITY ? 0.f : __expf(sc[h][r] - mx);
        l += p;  // the 16 lanes of a group hold the same p
        float vf[8];
        unpack8(vr[r], vf);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += p * vf[e];
      }
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] += __shfl_xor(o[e], 16, 64);
      o[e] += __shfl_xor(o[e], 32, 64);
    }
    if (g == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) sm_o[w][h][8 * li + e] = o[e];
      if (li == 0) {
        sm_m[w][h] = mx;
        sm_l[w][h] = l;
      }
    }
  }
  __syncthreads();

  // ---- the workgroup's (m, l, o) per head: thread -> (head, 4 dims)
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(ws + ((size_t)b * Hkv + kvh) * nsplit * PS, 0, nsplit * PS * 4, 0x00020000);
  for (int it = threadIdx.x; it < REP * 32; it += AD5_WAVES * 64) {
    const int h = it >> 5, d = 4 * (it & 31);
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < AD5_WAVES; ++ww) M = fmaxf(M, sm_m[ww][h]);
    float num[4] = {0.f, 0.f, 0.f, 0.f}, den = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int ww = 0; ww < AD5_WAVES; ++ww) {
        const float mw = sm_m[ww][h];
        const float f = mw == -INFINITY ? 0.f : __expf(mw - M);
        den += f * sm_l[ww][h];
#pragma unroll
        for (int e = 0; e < 4; ++e) num[e] += f * sm_o[ww][h][d + e];
      }
    }
    if (n_act == 1) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = den > 0.f ? num[e] / den : 0.f;
      store_out(h, d, v);
    } else {
      const int off = (split * PS + h * HS) * 4;
      __builtin_amdgcn_raw_buffer_store_b128(
          u32x4{__float_as_uint(num[0]), __float_as_uint(num[1]), __float_as_uint(num[2]), __float_as_uint(num[3])},
          rs, off + (4 + d) * 4, 0, 16);
      if (d == 0)
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(M), __float_as_uint(den), 0u, 0u}, rs, off, 0, 16);
    }
  }
  if (n_act == 1) return;

  // ---- publish: every storing wave drains its write-through stores, then one ticket add per workgroup
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t* tk = tickets + (size_t)b * Hkv + kvh;
    const int prev = __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == n_act - 1;
    if (last) __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // reset for the next call
    last_flag = last;
  }
  __syncthreads();
  if (!last_flag) return;

  // ---- last arriver: online merge of the active splits in split order (sc1 loads, 4 splits in flight)
  for (int it = threadIdx.x; it < REP * 32; it += AD5_WAVES * 64) {
    const int h = it >> 5, d = 4 * (it & 31);
    float Mr = -INFINITY, Lr = 0.f, Or[4] = {0.f, 0.f, 0.f, 0.f};
    auto fold = [&](const u32x4 ml, const u32x4 ov) {
      const float ms = __uint_as_float(ml[0]);
      if (ms == -INFINITY) return;
      const float mn = fmaxf(Mr, ms);
      const float a = Mr == -INFINITY ? 0.f : __expf(Mr - mn), f = __expf(ms - mn);
      Lr = Lr * a + f * __uint_as_float(ml[1]);
#pragma unroll
      for (int e = 0; e < 4; ++e) Or[e] = Or[e] * a + f * __uint_as_float(ov[e]);
      Mr = mn;
    };
    // AD5_FOLD splits per round, all loads of a round in flight together (one dependent L2 round trip per round,
    // not one per 4 splits: T = 384 at rep 8 is 12 splits); past the end the last split is re-read, never folded
    for (int s = s_lo; s < s_hi; s += AD5_FOLD) {
      u32x4 ml[AD5_FOLD], ov[AD5_FOLD];
#pragma unroll
      for (int u = 0; u < AD5_FOLD; ++u) {
        const int off = (min(s + u, s_hi - 1) * PS + h * HS) * 4;
        ml[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
        ov[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, off + (4 + d) * 4, 0, 16);
      }
#pragma unroll
      for (int u = 0; u < AD5_FOLD; ++u)
        if (s + u < s_hi) fold(ml[u], ov[u]);
    }
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = Lr > 0.f ? Or[e] / Lr : 0.f;
    store_out(h, d, v);
  }
}

// ---------------------------------------------------------------------------------------------
// v2 (default): streaming decode attention, one WAVE per work item (batch row, kv head, key split).
//
// The round-1 kernel (v1, removed in round 6) gave every 128-key chunk its own workgroup (load everything, compute,
// merge), so a CU's HBM queue drained between a workgroup's load burst and its compute/merge phases and every chunk
// paid a merge; it held ~3-3.8 TB/s. Here each wave streams its item's keys in chunks of 4*KPG rows
// through two register buffers (chunk c+1 in flight while chunk c is scored), keeps a running
// (max, sum, o) per query head (online softmax), and needs no workgroup barrier at all. Splits are
// only used when B*Hkv alone cannot fill the chip (small batch / long context): the split count
// targets >= `waves_target` waves, and the last-arriving wave of a (b, kv head) merges the splits'
// (m, l, o) (sc1 stores -> vmcnt(0) -> one agent-scope ticket add per wave).
//
// Lane layout per chunk: lane = 16*g + li; row r of lane group g is key k0 + CK*c + 4*r + g, and
// the lane holds dims [8*li, 8*li + 8) of it, so one wave load instruction covers 4 consecutive
// cache rows (1 KiB contiguous). QK^T: 8 FMAs + a 16-lane DPP sum; P.V: lane-local over the group's
// rows, summed across the 4 groups once per item.
static int g_attn_waves_target = 2048;
static int g_attn_v2_min_pairs = 4096;
static int g_attn_diag = 0;  // tools only: 1 = v2 / v4 stream K/V without the math (wrong results)
// register-ring streaming kernel (v4) for one-split large batches without a key mask: 5-12 % faster than v2 at
// B = 512-2048 (profiles/r2_attn_decode_v4_vs_v2.jsonl); impl 2 (default) uses it, impl 4 pins v2 (KPG 4, 2 slots)
static bool g_attn_v4 = true;
void attn_set_diag(int d) { g_attn_diag = d; }
void attn_set_impl(int impl, int waves_target);

template <int REP, int KPG, int NS, bool MASK>
__global__ void __launch_bounds__(64)
    attn_decode_v2_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                          const int32_t* __restrict__ slot_ptr, const int32_t* __restrict__ kv_start,
                          const uint8_t* __restrict__ key_mask, int mask_len, bf16_t* __restrict__ out,
                          float* __restrict__ ws, int32_t* __restrict__ tickets, int B, int H, int Hkv, int T,
                          int t_cap, int nsplit, int split_len, float scale, int diag) {
  constexpr int CK = 4 * KPG;        // keys per chunk
  constexpr int SLOT = 2 * KPG * 64;  // u32x4 per ring slot: KPG K-row loads then KPG V-row loads
  constexpr int QL = (REP + 3) / 4;  // q LDS-DMA loads (4 heads of 256 B per wave load)
  __shared__ u32x4 ring[NS * SLOT + QL * 64];
  u32x4* qbuf = ring + NS * SLOT;
  const int lane = threadIdx.x;
  const int item = blockIdx.x;
  const int pair = item / nsplit, split = item - pair * nsplit;
  const int kvh = pair % Hkv, b = pair / Hkv;
  const int g = lane >> 4, li = lane & 15;
  const int slot = slot_ptr[0];
  if (slot >= T && threadIdx.x == 0) JLA_FLAG(JLA_BOUNDS_ATTN_T);  // keys past the cache are never read
  const int lo = kv_start[b];
  const int s0 = split * split_len;
  const int k0 = max(s0, lo);
  const int k1 = min(min(s0 + split_len, t_cap), slot + 1);  // keys [k0, k1)
  const int h0 = kvh * REP;

  float m_h[REP], l_h[REP];
  f32x2_t o[REP][4];  // dims 8*li + 2i, 8*li + 2i + 1
#pragma unroll
  for (int h = 0; h < REP; ++h) {
    m_h[h] = -INFINITY;
    l_h[h] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[h][i] = f32x2_t{0.f, 0.f};
  }

  if (k0 < k1) {
    const size_t head_off = ((size_t)b * Hkv + kvh) * T * AD_DH + 8 * li;
    const bf16_t* kbase = kc + head_off;
    const bf16_t* vbase = vc + head_off;
    const uint8_t* mrow = MASK ? key_mask + (size_t)b * mask_len : nullptr;
    // q rides the same LDS-DMA queue as K/V (an ordinary load beside glds makes hipcc wait
    // vmcnt(0) at its first use, draining the ring): 16 lanes per head, 16 B each
    const bf16_t* qrow = q + ((size_t)b * H + h0) * AD_DH;
#pragma unroll
    for (int i = 0; i < QL; ++i)
      glds16(qrow + (size_t)min(4 * i + g, REP - 1) * AD_DH + 8 * li, qbuf + i * 64);
    const int nc = (k1 - k0 + CK - 1) / CK;
    u32x4 qp[REP];  // this lane's 8 dims of each query head, packed bf16 (v_dot2 operand)

    // LDS-DMA: chunk c -> ring slot c % NS; lane l of K-row load r lands at slot + r*64 + l, i.e.
    // exactly where the same lane reads it back (no other wave touches this ring).
    auto issue = [&](int c) __attribute__((always_inline)) {
      u32x4* sl = ring + (c % NS) * SLOT;
      const int jb = k0 + c * CK + g;
#pragma unroll
      for (int r = 0; r < KPG; ++r) glds16(kbase + (size_t)min(jb + 4 * r, k1 - 1) * AD_DH, sl + r * 64);
#pragma unroll
      for (int r = 0; r < KPG; ++r) glds16(vbase + (size_t)min(jb + 4 * r, k1 - 1) * AD_DH, sl + (KPG + r) * 64);
    };
    auto compute = [&](const u32x4* kr, const u32x4* vr, int c) __attribute__((always_inline)) {
      const int jb = k0 + c * CK + g;
      float sc[REP][KPG];
#pragma unroll
      for (int r = 0; r < KPG; ++r) {
        const int j = jb + 4 * r;
        bool valid = j < k1;
        if constexpr (MASK) valid = valid && (j >= mask_len || mrow[j] != 0);
#pragma unroll
        for (int h = 0; h < REP; ++h) {
          float d = dot8_bf16(kr[r], qp[h], 0.f);
          d = row16_sum(d) * scale;
          sc[h][r] = valid ? d : -INFINITY;
        }
      }
#pragma unroll
      for (int h = 0; h < REP; ++h) {
        float cm = sc[h][0];
#pragma unroll
        for (int r = 1; r < KPG; ++r) cm = fmaxf(cm, sc[h][r]);
        cm = fmaxf(cm, __shfl_xor(cm, 16, 64));
        cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
        const float mn = fmaxf(m_h[h], cm);
        const float alpha = (m_h[h] == -INFINITY) ? 0.f : __expf(m_h[h] - mn);
        m_h[h] = mn;
        l_h[h] *= alpha;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[h][i] *= alpha;
      }
#pragma unroll
      for (int r = 0; r < KPG; ++r) {
        f32x2_t vf[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          vf[i] = f32x2_t{__uint_as_float(vr[r][i] << 16), __uint_as_float(vr[r][i] & 0xffff0000u)};
#pragma unroll
        for (int h = 0; h < REP; ++h) {
          const float p = (sc[h][r] == -INFINITY) ? 0.f : __expf(sc[h][r] - m_h[h]);
          l_h[h] += p;
          const f32x2_t pp = {p, p};
#pragma unroll
          for (int i = 0; i < 4; ++i) o[h][i] = __builtin_elementwise_fma(pp, vf[i], o[h][i]);
        }
      }
    };

    // ring: NS-1 chunks in flight ahead of the one being scored; waits counted by hand (the loop has
    // no compiler-visible global loads, so hipcc inserts no vmcnt of its own)
#pragma unroll
    for (int c = 0; c < NS - 1; ++c)
      if (c < nc) issue(c);
    {  // q landed once chunk 0 has (issued before it)
      const int ahead = min(nc - 1, NS - 2);
      if (ahead >= 2)
        wait_vmcnt<2 * 2 * KPG>();
      else if (ahead == 1)
        wait_vmcnt<2 * KPG>();
      else
        wait_vmcnt<0>();
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int h = 0; h < REP; ++h) qp[h] = qbuf[(h >> 2) * 64 + (h & 3) * 16 + li];
    for (int c = 0; c < nc; ++c) {
      if (c + NS - 1 < nc) issue(c + NS - 1);
      const int ahead = min(nc - 1 - c, NS - 1);  // chunks issued after c
      if (ahead >= 3)
        wait_vmcnt<3 * 2 * KPG>();
      else if (ahead == 2)
        wait_vmcnt<2 * 2 * KPG>();
      else if (ahead == 1)
        wait_vmcnt<2 * KPG>();
      else
        wait_vmcnt<0>();
      asm volatile("" ::: "memory");
      const u32x4* sl = ring + (c % NS) * SLOT;
      u32x4 kr[KPG], vr[KPG];
#pragma unroll
      for (int r = 0; r < KPG; ++r) kr[r] = sl[r * 64 + lane];
#pragma unroll
      for (int r = 0; r < KPG; ++r) vr[r] = sl[(KPG + r) * 64 + lane];
      if (diag) {  // DIAGNOSTIC (wrong results): stream only, keep the chunk live, skip the math
#pragma unroll
        for (int r = 0; r < KPG; ++r) asm volatile("" ::"v"(kr[r]), "v"(vr[r]));
      } else {
        compute(kr, vr, c);
      }
      // WAR: slot c % NS is refilled by the issue at the top of iteration c + 1; its ds_reads above
      // were consumed by compute (lgkmcnt waited before use), so they have completed.
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    // across the 4 lane groups: each group summed its own rows (l is the same in its 16 lanes)
#pragma unroll
    for (int h = 0; h < REP; ++h) {
      l_h[h] += __shfl_xor(l_h[h], 16, 64);
      l_h[h] += __shfl_xor(l_h[h], 32, 64);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          o[h][i][e] += __shfl_xor(o[h][i][e], 16, 64);
          o[h][i][e] += __shfl_xor(o[h][i][e], 32, 64);
        }
    }
  }

  if (nsplit == 1) {
    if (g == 0) {
#pragma unroll
      for (int h = 0; h < REP; ++h) {
        const float inv = l_h[h] > 0.f ? 1.f / l_h[h] : 0.f;
        float r8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) r8[e] = o[h][e >> 1][e & 1] * inv;
        *reinterpret_cast<u32x4*>(out + ((size_t)b * H + h0 + h) * AD_DH + 8 * li) = pack8(r8);
      }
    }
    return;
  }

  // ---- publish this split's (m, l, o) with write-through stores, then one ticket add per wave
  float* part = ws + (size_t)item * REP * (AD_DH + 2);
  if (g == 0) {
#pragma unroll
    for (int h = 0; h < REP; ++h) {
#pragma unroll
      for (int e = 0; e < 8; ++e) st_wt(part + h * (AD_DH + 2) + 2 + 8 * li + e, o[h][e >> 1][e & 1]);
      if (li == 0) {
        st_wt(part + h * (AD_DH + 2), m_h[h]);
        st_wt(part + h * (AD_DH + 2) + 1, l_h[h]);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int last = 0;
  if (lane == 0) {
    int32_t* tk = tickets + pair;
    const int prev = __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == nsplit - 1;
    if (last) __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // reset for next replay
  }
  last = __shfl(last, 0, 64);
  if (!last) return;

  // ---- last arriver (one wave): log-sum-exp merge of the pair's splits with sc1 loads
  const float* base = ws + (size_t)pair * nsplit * REP * (AD_DH + 2);
#pragma unroll 1
  for (int h = 0; h < REP; ++h) {
    float M = -INFINITY;
    for (int s = 0; s < nsplit; ++s) M = fmaxf(M, ld_wt(base + ((size_t)s * REP + h) * (AD_DH + 2)));
    float num0 = 0.f, num1 = 0.f, den = 0.f;
    for (int s = 0; s < nsplit; ++s) {
      const float* ps = base + ((size_t)s * REP + h) * (AD_DH + 2);
      const float ms = ld_wt(ps), ls = ld_wt(ps + 1);
      const float a = ld_wt(ps + 2 + lane), c = ld_wt(ps + 2 + 64 + lane);
      const float wgt = (ms == -INFINITY || M == -INFINITY) ? 0.f : __expf(ms - M);
      den += wgt * ls;
      num0 += wgt * a;
      num1 += wgt * c;
    }
    const float inv = den > 0.f ? 1.f / den : 0.f;
    bf16_t* op = out + ((size_t)b * H + h0 + h) * AD_DH;
    op[lane] = f2bf(num0 * inv);
    op[64 + lane] = f2bf(num1 * inv);
  }
}

// ---------------------------------------------------------------------------------------------
// v4 (large batch, one split): v2's one-wave-per-(row, kv head) stream with the K/V rows loaded straight into
// registers instead of through an LDS-DMA ring. v2 holds one 8-KiB chunk in flight per wave and its 17-33 KiB
// LDS ring caps a CU at 4-9 waves: its stream-only diagnostic build (no math) tops out at 5.5-5.8 TB/s
// (profiles/r2_attn_decode_b2048_geometry.jsonl). Here a U-slot register ring keeps U-1 chunks of 16 keys
// (U-1 x 8 KiB) in flight per wave with no LDS, so occupancy is set by registers alone.
// The loads are inline asm with hand-counted waits (the GEMV recipe, gemv.hip: hipcc's own waitcnt pass
// would drain the ring at the loop back-edge); every ring slot is a "+v"-tied variable pinned behind its
// wait, and build.py checks the assembly with tools/check_asm_ring.py. Chunks past the end re-load the last
// valid row (never scored), so every iteration issues exactly L loads and the wait count is a constant.
JLA_DEV void ad_load_nt(u32x4& r, const void* p) {
  asm volatile("global_load_dwordx4 %0, %1, off nt" : "+v"(r) : "v"(p) : "memory");
}
JLA_DEV void ad_load(u32x4& r, const void* p) { asm volatile("global_load_dwordx4 %0, %1, off" : "+v"(r) : "v"(p) : "memory"); }
JLA_DEV void ad_pin(u32x4& r) { asm volatile("" : "+v"(r)); }
template <int N>
JLA_DEV void ad_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

template <int REP, int KPG, int U, bool DIAG = false>
__global__ void __launch_bounds__(64)
    attn_decode_v4_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                          const int32_t* __restrict__ slot_ptr, const int32_t* __restrict__ kv_start,
                          bf16_t* __restrict__ out, int H, int Hkv, int T, int t_cap, float scale,
                          bf16_t* __restrict__ out_pack) {
  constexpr int CK = 4 * KPG;  // keys per chunk
  constexpr int L = 2 * KPG;   // loads per chunk and lane: KPG K rows + KPG V rows (16 B each)
  const int lane = threadIdx.x;
  const int item = blockIdx.x;
  const int kvh = item % Hkv, b = item / Hkv;
  const int g = lane >> 4, li = lane & 15;
  const int slot = slot_ptr[0];
  if (slot >= T && lane == 0) JLA_FLAG(JLA_BOUNDS_ATTN_T);  // keys past the cache are never read
  const int k0 = kv_start[b];
  const int k1 = min(t_cap, slot + 1);  // keys [k0, k1)
  const int h0 = kvh * REP;

  float m_h[REP], l_h[REP];
  f32x2_t o[REP][4];  // dims 8*li + 2i, 8*li + 2i + 1
#pragma unroll
  for (int h = 0; h < REP; ++h) {
    m_h[h] = -INFINITY;
    l_h[h] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[h][i] = f32x2_t{0.f, 0.f};
  }

  const int nc = k1 > k0 ? (k1 - k0 + CK - 1) / CK : 0;
  if (nc > 0) {
    const size_t head_off = ((size_t)b * Hkv + kvh) * T * AD_DH + 8 * li;
    const bf16_t* kbase = kc + head_off;
    const bf16_t* vbase = vc + head_off;
    // this lane's 8 dims of each query head (packed bf16: the v_dot2 operand), counted in the same queue
    u32x4 qp[REP] = {};
#pragma unroll
    for (int h = 0; h < REP; ++h) ad_load(qp[h], q + ((size_t)b * H + h0 + h) * AD_DH + 8 * li);
    u32x4 ring[U][L] = {};
    auto issue = [&](int c, u32x4* sl) __attribute__((always_inline)) {
      const int jb = k0 + c * CK + g;
#pragma unroll
      for (int r = 0; r < KPG; ++r) ad_load_nt(sl[r], kbase + (size_t)min(jb + 4 * r, k1 - 1) * AD_DH);
#pragma unroll
      for (int r = 0; r < KPG; ++r) ad_load_nt(sl[KPG + r], vbase + (size_t)min(jb + 4 * r, k1 - 1) * AD_DH);
    };
    // base-2 softmax (scale pre-multiplied by log2 e, v_exp_f32 directly). Chunk 0 always holds key k0, so after it
    // every running max is finite: exp2(-inf - max) = 0 for masked keys and for the first rescale (m = -inf) without
    // selects; only the last chunk (keys past k1) masks scores, behind a wave-uniform branch.
    const float scale2 = scale * 1.4426950408889634f;
    auto compute = [&](const u32x4* kr, const u32x4* vr, int c) __attribute__((always_inline)) {
      const int jb = k0 + c * CK + g;
      const bool full = k0 + (c + 1) * CK <= k1;
      float sc[REP][KPG];
#pragma unroll
      for (int r = 0; r < KPG; ++r) {
#pragma unroll
        for (int h = 0; h < REP; ++h) {
          const float d = dot8_bf16(kr[r], qp[h], 0.f);
          sc[h][r] = row16_sum(d) * scale2;
        }
      }
      if (!full) {
#pragma unroll
        for (int r = 0; r < KPG; ++r) {
          const bool valid = jb + 4 * r < k1;
#pragma unroll
          for (int h = 0; h < REP; ++h) sc[h][r] = valid ? sc[h][r] : -INFINITY;
        }
      }
#pragma unroll
      for (int h = 0; h < REP; ++h) {
        float cm = sc[h][0];
#pragma unroll
        for (int r = 1; r < KPG; ++r) cm = fmaxf(cm, sc[h][r]);
        cm = fmaxf(cm, __shfl_xor(cm, 16, 64));
        cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
        const float mn = fmaxf(m_h[h], cm);
        const float alpha = __builtin_amdgcn_exp2f(m_h[h] - mn);
        m_h[h] = mn;
        l_h[h] *= alpha;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[h][i] *= alpha;
      }
#pragma unroll
      for (int r = 0; r < KPG; ++r) {
        f32x2_t vf[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          vf[i] = f32x2_t{__uint_as_float(vr[r][i] << 16), __uint_as_float(vr[r][i] & 0xffff0000u)};
#pragma unroll
        for (int h = 0; h < REP; ++h) {
          const float pr = __builtin_amdgcn_exp2f(sc[h][r] - m_h[h]);
          l_h[h] += pr;
          const f32x2_t pp = {pr, pr};
#pragma unroll
          for (int i = 0; i < 4; ++i) o[h][i] = __builtin_elementwise_fma(pp, vf[i], o[h][i]);
        }
      }
    };

    // prologue: chunks 0 .. U-2 in flight (the q loads before them)
#pragma unroll
    for (int c = 0; c < U - 1; ++c) issue(c, ring[c]);
    for (int c0 = 0; c0 < nc; c0 += U) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int c = c0 + u;
        issue(c + U - 1, ring[(u + U - 1) % U]);  // refills the slot chunk c-1 was scored from
        ad_vmcnt<L * (U - 1)>();                  // chunk c (and q) landed: U-1 newer chunks may be in flight
#pragma unroll
        for (int e = 0; e < L; ++e) ad_pin(ring[u][e]);
#pragma unroll
        for (int h = 0; h < REP; ++h) ad_pin(qp[h]);
        if constexpr (DIAG) {  // tools only (attn_set_diag): the stream without the math (the pins keep it live)
          (void)c;
        } else {
          if (c < nc) compute(ring[u], ring[u] + KPG, c);
        }
      }
    }
    // retire the past-the-end refills, keeping every ring register live until then
    ad_vmcnt<0>();
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < L; ++e) ad_pin(ring[u][e]);
    // across the 4 lane groups: each group summed its own rows
#pragma unroll
    for (int h = 0; h < REP; ++h) {
      l_h[h] += __shfl_xor(l_h[h], 16, 64);
      l_h[h] += __shfl_xor(l_h[h], 32, 64);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          o[h][i][e] += __shfl_xor(o[h][i][e], 16, 64);
          o[h][i][e] += __shfl_xor(o[h][i][e], 32, 64);
        }
    }
  }
  if (g == 0) {
#pragma unroll
    for (int h = 0; h < REP; ++h) {
      const float inv = l_h[h] > 0.f ? 1.f / l_h[h] : 0.f;
      float r8[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) r8[e] = o[h][e >> 1][e & 1] * inv;
      const u32x4 pk = pack8(r8);
      *reinterpret_cast<u32x4*>(out + ((size_t)b * H + h0 + h) * AD_DH + 8 * li) = pk;
      // decode rows <= 64: also the packed copy (common.h pack_off) the o projection's packed-x GEMV reads
      if (out_pack) *reinterpret_cast<u32x4*>(out_pack + pack_off(b, (h0 + h) * AD_DH + 8 * li, H * AD_DH)) = pk;
    }
  }
}

static int g_kpg_small = 8;  // v2 ring geometry for REP <= 4 below 16384 pairs (impl 4: 4)
// the geometry by size: at >= 16384 (row, kv head) pairs (B >= 2048 at 8 kv heads) the 17-KiB (KPG 4, 2 slots) ring --
// 9 waves per CU instead of 4 -- streams 5.4-5.8 TB/s against 4.0-5.6 for (KPG 8, 2 slots), which stays best at
// B = 1024 (profiles/r2_attn_decode_b2048_geometry.jsonl)
static bool g_geo_auto = true;
static int kpg_v2(int rep, int pairs) {
  if (rep <= 4) return (g_geo_auto && pairs >= 16384) ? 4 : g_kpg_small;
  return rep == 8 ? 2 : 1;
}

// impl 2 = default dispatch; 4 = v2 with the (KPG 4, 2 slots) ring and no v4 (tests / A/B).
// waves_target > 0: v2's split count target; < 0: v2 (or v4) down to -waves_target pairs
void attn_set_impl(int impl, int waves_target) {
  g_kpg_small = impl == 4 ? 4 : 8;
  g_geo_auto = impl != 4;
  g_attn_v4 = impl != 4;
  if (waves_target > 0) g_attn_waves_target = waves_target;
  g_attn_v2_min_pairs = waves_target < 0 ? -waves_target : 4096;  // < 0: force v2 down to -target pairs
}

// v2 streams whole (b, kv head) pairs from ~4096 pairs (B = 512 at 8 kv heads) up.
// The one-split register-ring stream (v4) also serves batches above the decode GEMV's rows (B > 64) below the v2
// threshold: at rep <= 4 from there on, at rep 8 from 2048 (row, kv head) pairs. Graph-timed with cold K/V
// (profiles/r3_attn_decode_v4_midbatch.jsonl): Llama-3-8B B = 128 / 256 (T 384) 71.9 / 129 us (v3) -> 57.9 / 70.5;
// Llama-3-70B B = 256 (T 256 / 384) 158 / 206 -> 87 / 125; v3 stays ahead at B <= 64 (where it also writes the
// packed copy the o projection's GEMV reads) and at rep 8 below 2048 pairs.
static bool v4_midbatch(int B, int Hkv, int rep) {
  return g_attn_v4 && g_attn_v2_min_pairs == 4096 && rep <= 8 &&
         ((rep <= 4 && B > 32) || (rep == 8 && B * Hkv >= 2048));
}
static bool use_v2(int B, int Hkv, int rep) { return B * Hkv >= g_attn_v2_min_pairs || v4_midbatch(B, Hkv, rep); }

// v3 (one workgroup per (row, kv head), no split merge) below this many (row, kv head) pairs
static int g_attn_v3_max_pairs = 4096;  // up to the v2 threshold: faster than the split kernels at B = 1..256 (8 kv heads)
void attn_set_v3_max_pairs(int n) { g_attn_v3_max_pairs = n; }
static bool use_v3(int B, int Hkv, int rep) {
  return rep <= 8 && !use_v2(B, Hkv, rep) && B * Hkv <= g_attn_v3_max_pairs;
}
// v3 keys per lane-group row per chunk = base KPG (REP * KPG = 8) x this multiplier (1, 2, 4; capped at 8 rows):
// fewer, larger chunks = fewer dependent load round trips on the latency-bound small-batch path
// 0 = by size: x2 up to 128 (row, kv head) pairs (B <= 16 at 8 kv heads: B = 1 T = 384 12.4 -> 11.0 us, B = 8
// 12.8 -> 11.3, B = 1 T = 1024 25.2 -> 22.1), x1 above (B = 32 / 64 slightly faster at x1;
// profiles/r2_attn_decode_v3_kpg_ab.jsonl)
static int g_v3_kpg_mult = 0;
void attn_set_v3_kpg(int mult) { g_v3_kpg_mult = mult >= 4 ? 4 : (mult >= 2 ? 2 : (mult == 1 ? 1 : 0)); }
// v5 (split small-batch kernel) below g_attn_v5_max_pairs (row, kv head) pairs, ahead of v3
// (measured with tools/bench_attn_decode.py, profiles/r3_attn_decode_v5_vs_v3.jsonl: at rep 8 -- Llama-3-70B at MP 8 --
// v3 is compute-bound on one CU per pair, so v5 wins 1.5-2x up to 32 pairs and further; at rep 4 -- Llama-3-8B -- the
// two tie at 64 pairs and v3 wins at 128)
static bool use_v5(int B, int Hkv, int rep) {
  const int pairs = B * Hkv;
  return rep <= 16 && (rep & (rep - 1)) == 0 &&
         (pairs <= g_attn_v5_max_pairs || (rep >= 8 && pairs <= 4 * g_attn_v5_max_pairs));
}
// v6 (attn_decode_mma.hip: scores and P.V on the matrix cores, one workgroup per pair, no workspace): 0 off,
// 1 where it wins (by shape), 2 every decode shape it supports (A/B, tests)
// By shape (graph-timed with cold K/V, profiles/r5_attn_decode_v6_ab.jsonl): at rep 8 from 8 up to (not including)
// 2048 (row, kv head) pairs -- Llama-3-70B at MP 8, B = 32 / 256: 12.9 / 28.8 -> 10.2 / 14.1 us; MP 1, B = 32: 39.0 ->
// 18.7 -- the VALU kernels there are compute-bound on the 8 q heads of a pair; v4 keeps rep 8 from 2048 pairs (MP 1,
// B = 256: 80 vs 94 us) and every rep <= 4 shape (v4 / v3 / v5 stream those faster).
static int g_attn_v6 = 1;
void attn_set_v6(int mode) { g_attn_v6 = mode < 0 ? 0 : (mode > 2 ? 2 : mode); }
static bool use_v6(int B, int Hkv, int rep) {
  if (g_attn_v6 == 0 || rep > 16 || (rep & (rep - 1))) return false;
  if (g_attn_v6 == 2) return true;
  return rep >= 8 && B * Hkv >= 8 && B * Hkv < 2048;
}
// the kernels that also write the packed output copy: v6, v5, v3, and v4 at decode rows <= 64 (mid-batch)
int attn_decode_packs(int B, int Hkv, int rep) {
  return (use_v6(B, Hkv, rep) || use_v5(B, Hkv, rep) || use_v3(B, Hkv, rep) || (B <= SKINNY_MAX_M && v4_midbatch(B, Hkv, rep))) ? 1 : 0;
}

int attn_decode_chunk(int B, int Hkv, int T, int rep) {
  if (use_v6(B, Hkv, rep)) return T;
  if (use_v5(B, Hkv, rep)) return 16 * kpg5(rep);
  if (use_v3(B, Hkv, rep)) return T;
  return 4 * kpg_v2(rep, B * Hkv);
}

int attn_decode_splits(int B, int Hkv, int T, int rep) {
  if (use_v6(B, Hkv, rep)) return 1;
  if (use_v5(B, Hkv, rep)) return (T + 16 * kpg5(rep) - 1) / (16 * kpg5(rep));
  if (use_v3(B, Hkv, rep)) return 1;
  if (v4_midbatch(B, Hkv, rep)) return 1;  // one split: the v4 stream (v2 with a key mask)
  const int pairs = B * Hkv;
  const int max_split = T > 64 ? (T + 63) / 64 : 1;  // >= 64 keys per split
  int ns = (g_attn_waves_target + pairs - 1) / pairs;
  ns = ns < 1 ? 1 : (ns > max_split ? max_split : ns);
  return ns;
}

int attn_decode(const bf16_t* q, const bf16_t* kc, const bf16_t* vc, const int32_t* slot, const int32_t* kv_start,
                const uint8_t* key_mask, int mask_len, bf16_t* out, float* ws, int32_t* tickets, int B, int H,
                int Hkv, int Dh, int T, int t_cap, int nsplit, hipStream_t s, bf16_t* out_pack) {
  if (B <= 0) return 0;
  if (out_pack && !attn_decode_packs(B, Hkv, H / Hkv)) return -3;  // only the small-batch kernels write the packed copy
  // (a key mask sends the mid-batch rows to v2, which does not write it)
  if (out_pack && key_mask && !use_v6(B, Hkv, H / Hkv) && !use_v5(B, Hkv, H / Hkv) && !use_v3(B, Hkv, H / Hkv))
    return -3;
  if (Dh != AD_DH || H % Hkv) return -1;
  const int rep = H / Hkv;
  if (attn_decode_splits(B, Hkv, t_cap, rep) != nsplit) return -2;
  if (use_v6(B, Hkv, rep))
    return attn_decode_v6(q, kc, vc, slot, kv_start, key_mask, mask_len, out, B, H, Hkv, T, t_cap, s, out_pack);
  const float scale = 1.f / sqrtf((float)Dh);
  if (use_v5(B, Hkv, rep)) {
    dim3 grid5(nsplit, Hkv, B);
#define JLA_AD5(R, K)                                                                                          \
  if (rep == R) {                                                                                              \
    if (g_attn_v5_fold == 4 || (g_attn_v5_fold == 0 && B * Hkv < 16))                                          \
      attn_decode_v5_kernel<R, K, 4><<<grid5, AD5_WAVES * 64, 0, s>>>(q, kc, vc, slot, kv_start, key_mask,     \
                                                                      mask_len, out, ws, tickets, H, Hkv, T,   \
                                                                      t_cap, nsplit, scale, out_pack);         \
    else                                                                                                       \
      attn_decode_v5_kernel<R, K, 12><<<grid5, AD5_WAVES * 64, 0, s>>>(q, kc, vc, slot, kv_start, key_mask,    \
                                                                       mask_len, out, ws, tickets, H, Hkv, T,  \
                                                                       t_cap, nsplit, scale, out_pack);        \
    JLA_CHECK_LAUNCH();                                                                                        \
    return 0;                                                                                                  \
  }
    JLA_AD5(1, 8) JLA_AD5(2, 8) JLA_AD5(4, 4) JLA_AD5(8, 2) JLA_AD5(16, 1)
#undef JLA_AD5
    return -1;
  }
  if (use_v3(B, Hkv, rep)) {
    dim3 grid3(Hkv, B);
#define JLA_AD3(R, K)                                                                                          \
  if (rep == R) {                                                                                              \
    attn_decode_v3_kernel<R, K><<<grid3, AD3_WAVES * 64, 0, s>>>(q, kc, vc, slot, kv_start, key_mask, mask_len, \
                                                                 out, H, Hkv, T, t_cap, scale, out_pack);      \
    JLA_CHECK_LAUNCH();                                                                                        \
    return 0;                                                                                                  \
  }
    const int mult = g_v3_kpg_mult ? g_v3_kpg_mult : (B * Hkv <= 128 ? 2 : 1);
    const int kpg3 = min(min(8, 16 / rep), (8 / rep) * mult);  // REP * KPG <= 16: no spills
#define JLA_AD3K(R, K) \
  if (kpg3 == K) {     \
    JLA_AD3(R, K)      \
  }
    JLA_AD3K(1, 8) JLA_AD3K(2, 4) JLA_AD3K(2, 8) JLA_AD3K(4, 2) JLA_AD3K(4, 4) JLA_AD3K(8, 1) JLA_AD3K(8, 2)
#undef JLA_AD3K
#undef JLA_AD3
    return -1;
  }
  const int items = B * Hkv * nsplit;
  if (g_attn_v4 && nsplit == 1 && !key_mask && rep <= 8) {
#define JLA_AD4(R, K, U)                                                                                         \
  if (rep == R) {                                                                                                \
    attn_decode_v4_kernel<R, K, U><<<items, 64, 0, s>>>(q, kc, vc, slot, kv_start, out, H, Hkv, T, t_cap, scale,   \
                                                        out_pack);                                               \
    JLA_CHECK_LAUNCH();                                                                                          \
    return 0;                                                                                                    \
  }
    if (g_attn_diag && rep == 4) {  // tools only: stream-only build of the rep-4 kernel (wrong results)
      attn_decode_v4_kernel<4, 4, 3, true><<<items, 64, 0, s>>>(q, kc, vc, slot, kv_start, out, H, Hkv, T, t_cap, scale,
                                                                nullptr);
      JLA_CHECK_LAUNCH();
      return 0;
    }
    JLA_AD4(1, 4, 3) JLA_AD4(2, 4, 3) JLA_AD4(4, 4, 3)
    // rep 8 (Llama-3-70B: 8 q heads per kv head): twice the q / o registers of rep 4, so 8-key chunks, 3 in flight
    // (16-key chunks x 3 slots at rep 8 fail the ring check: the compiler reuses in-flight ring registers)
    JLA_AD4(8, 2, 4)
#undef JLA_AD4
  }
  int split_len = (t_cap + nsplit - 1) / nsplit;
  split_len = (split_len + 31) / 32 * 32;
#define JLA_AD2(R, KPG, NS)                                                                                          \
  if (key_mask)                                                                                                     \
    attn_decode_v2_kernel<R, KPG, NS, true><<<items, 64, 0, s>>>(q, kc, vc, slot, kv_start, key_mask, mask_len, out, \
                                                                 ws, tickets, B, H, Hkv, T, t_cap, nsplit, split_len, \
                                                                 scale, g_attn_diag);                              \
  else                                                                                                              \
    attn_decode_v2_kernel<R, KPG, NS, false><<<items, 64, 0, s>>>(q, kc, vc, slot, kv_start, key_mask, mask_len, out, \
                                                                  ws, tickets, B, H, Hkv, T, t_cap, nsplit,          \
                                                                  split_len, scale, g_attn_diag);
  const bool k8 = kpg_v2(rep, B * Hkv) == 8;
  switch (rep) {
    // REP <= 4 shares one body per geometry (REP only sizes the register arrays)
    case 1: if (k8) { JLA_AD2(1, 8, 2) } else { JLA_AD2(1, 4, 2) } break;
    case 2: if (k8) { JLA_AD2(2, 8, 2) } else { JLA_AD2(2, 4, 2) } break;
    case 4: if (k8) { JLA_AD2(4, 8, 2) } else { JLA_AD2(4, 4, 2) } break;
    case 8: JLA_AD2(8, 2, 4) break;
    case 16: JLA_AD2(16, 1, 4) break;
    default: return -1;
  }
#undef JLA_AD2
  JLA_CHECK_LAUNCH();
  return 0;
}

JLA_BOUNDS_ACCESSOR(attn_decode)

}  // namespace jla
