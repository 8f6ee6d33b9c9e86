// Decode attention on the matrix cores (v6): one query token per batch row, GQA groups of REP q heads per kv head.
//
// Reference ops: jax_llama/model.py:277-291 (scores, softmax, P.V of FlaxLLaMAAttention) for S = 1 against the
// KV cache (:169-199), with the GQA expand (:269-270) folded into the indexing and the causal / padding mask
// (:236-251) computed from kv_start and the cache slot.
//
// The VALU kernels (v3 / v5: dot products per lane) are compute-bound at rep 8 (Llama-3-70B: 8 q heads share
// each kv head): one (row, kv head) pair is 8 x T dot products of 128. Here the REP heads of a pair are the 16
// columns of one v_mfma_f32_16x16x32_bf16 tile (REP <= 16 used, the rest zero), so a 32-key step costs
//   S^T = K Q^T : 2 key blocks x 4 dk steps = 8 MFMAs   (A = K rows straight from global memory into VGPRs: lane
//                  (key l & 15, group c = l >> 4) holds dims 32j + 8c .. +7 of its key for dk step j, so the 4
//                  lanes of a key read 64 contiguous bytes per load; the Q^T fragments use the same dim permutation)
//   O^T += V^T P^T : 8 dim tiles of 16 = 8 MFMAs          (A = V^T by ds_read_b64_tr_b16 from a row-major V image
//                  in LDS, B = the bf16 P of the lane's own 8 scores: the S^T accumulator layout IS the P^T
//                  operand layout once the k slots are ordered keys {4c .. 4c+3, 16+4c .. 16+4c+3})
// and the online softmax is lane-local (one head per lane column) plus two cross-group max exchanges per step.
//
// Work split: one workgroup per (row, kv head) pair with WPP waves; wave w streams 32-key steps w, w + WPP, ... of
// the pair's valid key range [kv_start, slot] with no barrier in the loop (each wave has its own two 8 KiB V slots
// and its own K register ring: V by LDS-DMA, K by plain loads, both issued one step ahead as inline asm with
// hand-counted waits so the next step's 16 loads stay in flight while this one computes). The WPP waves merge
// (m, l, O) once through LDS at the end. Rows with no valid key output 0.
#include "common.h"
#include "launchers.h"
#include "ring.h"

namespace jla {

constexpr int AD6_DH = 128;
constexpr int AD6_STEP = 32;                        // keys per step
constexpr int AD6_SLOT_BYTES = AD6_STEP * AD6_DH * 2;  // 8 KiB of V per step
constexpr int AD6_WAVE_LDS = 2 * AD6_SLOT_BYTES;        // two V slots per wave

typedef short s16x4_6 __attribute__((ext_vector_type(4)));

// byte offset of 16-byte chunk ch (0..15) of row `row` in a [rows][128 bf16] image: conflict-free for both the
// DMA's lane-linear writes and ds_read_b64_tr_b16's 4-row x 16-column reads (the flash prefill's image)
JLA_DEV int ad6_off(int row, int ch) { return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3))); }

// The O^T accumulators are pinned to AGPRs through inline-asm MFMAs (with the intrinsic, hipcc kept them in VGPRs
// across the loop and copied all 32 in from AGPRs every step). hipcc's hazard recognizer does not look inside the
// asm, so the wait states are explicit: before the PV group (the VALU-written P operand and, after a rescale, the
// v_accvgpr_write of the accumulators) and between the last MFMA and a read of its result (ad6_take).
JLA_DEV void ad6_mfma_acc(f32x4& acc, const u32x4& a, const u32x4& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
JLA_DEV f32x4 ad6_take(f32x4& a) {  // an AGPR accumulator at this point in program order (MFMA -> read: s_nop pad)
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+a"(a));
  return a;
}
JLA_DEV void ad6_put(f32x4& a, const f32x4 v) {
  a = v;
  asm volatile("" : "+a"(a));
}

JLA_DEV u32x2 ad6_tr(const char* lds, int off) {
  return __builtin_bit_cast(u32x2, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                       (__attribute__((address_space(3))) s16x4_6*)(lds + off)));
}

template <int REP, int WPP>
__global__ void __launch_bounds__(WPP * 64)
    attn_decode_v6_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                          const int32_t* __restrict__ slot_ptr, const int32_t* __restrict__ kv_start,
                          const uint8_t* __restrict__ key_mask, int mask_len, bf16_t* __restrict__ out, int H, int Hkv,
                          int T, int t_cap, float scale_log2, bf16_t* __restrict__ out_pack) {
  static_assert(REP >= 1 && REP <= 16, "REP q heads per MFMA column tile");
  extern __shared__ __attribute__((aligned(16))) char lds6[];
  const int pair = blockIdx.x;
  const int b = pair / Hkv, kvh = pair - b * Hkv;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane >> 4, j = lane & 15;  // lane group (key / dim quarter), MFMA column (q head)
  char* const vbuf = lds6 + w * AD6_WAVE_LDS;

  const int slot = slot_ptr[0];
  if (slot >= T && threadIdx.x == 0) JLA_FLAG(JLA_BOUNDS_ATTN_T);
  const int lo = kv_start[b];
  const int hi = min(slot + 1, t_cap);  // keys [lo, hi)
  const uint8_t* mrow = key_mask ? key_mask + (size_t)b * mask_len : nullptr;
  const int h0 = kvh * REP;
  const size_t head_off = ((size_t)b * Hkv + kvh) * (size_t)T * AD6_DH;
  const bf16_t* const kb = kc + head_off;
  const bf16_t* const vb = vc + head_off;

  // Q^T fragments: lane (c, j) holds head h0 + j, dims 32jj + 8c .. +7 for dk step jj (zero columns past REP)
  u32x4 qf[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    qf[jj] = u32x4{0u, 0u, 0u, 0u};
    if (j < REP) qf[jj] = *reinterpret_cast<const u32x4*>(q + ((size_t)b * H + h0 + j) * AD6_DH + 32 * jj + 8 * c);
  }
  // a wait hipcc sees: otherwise it places a vmcnt(0) for these loads inside the loop, behind the hand-counted ring
  ::wait_vmcnt<0>();
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) pin(qf[jj]);

  const int s_begin = lo >= 0 ? lo / AD6_STEP : 0;
  const int n_steps = lo < hi ? (hi - 1) / AD6_STEP - s_begin + 1 : 0;
  const int my_steps = n_steps > w ? (n_steps - w + WPP - 1) / WPP : 0;

  // per-lane load addresses of one step (relative to the step's first key row)
  //   K: key (l & 15) of block kb (kb = 0, 1), bytes 64jj + 16c (jj = 0..3)
  //   V DMA: 1 KiB block bi (rows 4bi .. 4bi+3), lane L -> row 4bi + L / 16, slot L % 16 <- source chunk slot ^ swz(row)
  auto issue = [&](int step, u32x4 (&kr)[8], char* vslot) {
    const int key0 = (s_begin + step) * AD6_STEP;
#pragma unroll
    for (int bi = 0; bi < 8; ++bi) {
      const int row = 4 * bi + (lane >> 4);
      const int ch = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
      const int key = min(key0 + row, T - 1);
      glds16_asm(vb + (size_t)key * AD6_DH + 8 * ch, vslot + 1024 * bi);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int key = min(key0 + 16 * kk + j, T - 1);
      const bf16_t* p = kb + (size_t)key * AD6_DH + 8 * c;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) asm_load<true>(kr[4 * kk + jj], p + 32 * jj);
    }
  };

  float m_run = -INFINITY, l_run = 0.f;
  f32x4 o[8];  // O^T accumulators, pinned to AGPRs (ad6_mfma_acc): touched by the VALU only in the rescale branch
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // valid = false: a ring slot loaded past the wave's last step (clamped addresses, fully masked, adds nothing)
  auto compute = [&](int step, bool valid, u32x4 (&kr)[8], const char* vslot) {
#pragma unroll
    for (int i = 0; i < 8; ++i) pin(kr[i]);
    const int key0 = (s_begin + step) * AD6_STEP;
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      s0 = mfma16x16x32(kr[jj], qf[jj], s0);
      s1 = mfma16x16x32(kr[4 + jj], qf[jj], s1);
    }
    // lane (c, j): s0[r] = score of key key0 + 4c + r, s1[r] = key key0 + 16 + 4c + r, head h0 + j
    float sc[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sc[r] = s0[r] * scale_log2;
      sc[4 + r] = s1[r] * scale_log2;
    }
    if (!(valid && key0 >= lo && key0 + AD6_STEP <= hi && !mrow)) {  // wave-uniform: only the edge steps mask
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int key = key0 + (e < 4 ? 4 * c + e : 16 + 4 * c + e - 4);
        bool ok = valid && key >= lo && key < hi;
        if (mrow) ok = ok && key < mask_len && mrow[key] != 0;
        sc[e] = ok ? sc[e] : -INFINITY;
      }
    }
    float tmax = sc[0];
#pragma unroll
    for (int e = 1; e < 8; ++e) tmax = fmaxf(tmax, sc[e]);
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    // lazy rescale (as the flash prefill): move the running max only when it grows by more than 8 (log2 units)
    if (__ballot(tmax > m_run + 8.f)) {
      const float m_new = fmaxf(m_run, tmax);
      const float alpha = __builtin_amdgcn_exp2f(m_run - (m_new == -INFINITY ? 0.f : m_new));
      l_run *= alpha;
      m_run = m_new;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        f32x4 t = ad6_take(o[dt]);
        t *= alpha;
        ad6_put(o[dt], t);
      }
    }
    const float m_use = m_run == -INFINITY ? 0.f : m_run;
    float p[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      p[e] = __builtin_amdgcn_exp2f(sc[e] - m_use);
      l_run += p[e];
    }
    u32x4 pf = pack8(p);
    asm volatile("s_nop 4" : "+v"(pf));  // VALU write of the P operand (and any accumulator write above) -> MFMA read
    // V^T fragments: lane 4q + pp of group c reads row 4c + q (and 16 + 4c + q), columns 16dt + 4pp .. +3
    const int q4 = (lane & 15) >> 2, pp = lane & 3;
    const int r0 = 4 * c + q4;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      const int ch = 2 * dt + (pp >> 1);
      const u32x2 a = ad6_tr(vslot, ad6_off(r0, ch) + 8 * (pp & 1));
      const u32x2 bb = ad6_tr(vslot, ad6_off(r0 + 16, ch) + 8 * (pp & 1));
      ad6_mfma_acc(o[dt], u32x4{a[0], a[1], bb[0], bb[1]}, pf);
    }
  };

  // Two-slot ring, branch-free around the loads (a branch there makes hipcc merge in-flight ring registers with
  // copies that read them before they land): every half-iteration issues the next step -- clamped to the wave's
  // last step past the end, computed fully masked -- and waits for the current one with a counted vmcnt.
  u32x4 ka[8], kb2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) ka[i] = kb2[i] = u32x4{0u, 0u, 0u, 0u};
  char* const slotA = vbuf;
  char* const slotB = vbuf + AD6_SLOT_BYTES;
  const int last = my_steps - 1;
  auto step_of = [&](int i) { return w + min(i, last) * WPP; };
  if (my_steps > 0) {
    issue(step_of(0), ka, slotA);
    for (int i = 0; i < my_steps; i += 2) {
      issue(step_of(i + 1), kb2, slotB);
      wait_vmcnt<16>();  // step i (slot A) landed; step i + 1 stays in flight
      compute(step_of(i), true, ka, slotA);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot A's V reads are done: refill it
      issue(step_of(i + 2), ka, slotA);
      wait_vmcnt<16>();
      compute(step_of(i + 1), i + 1 < my_steps, kb2, slotB);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    wait_vmcnt<0>();  // the last refill of slot A: drained before the LDS is reused or the wave ends
  }

  // per wave: the row sum over the 4 lane groups (the running max is already shared by them)
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = ad6_take(o[dt]);
  l_run += __shfl_xor(l_run, 16, 64);
  l_run += __shfl_xor(l_run, 32, 64);
  // lane (c, j) holds O[head j][dims 16dt + 4c + r]
  if constexpr (WPP == 1) {
    if (j < REP) {
      const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
      bf16_t* orow = out + ((size_t)b * H + h0 + j) * AD6_DH;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        const u32x2 v = {pack2bf(o[dt][0] * inv, o[dt][1] * inv), pack2bf(o[dt][2] * inv, o[dt][3] * inv)};
        const int d = 16 * dt + 4 * c;
        *reinterpret_cast<u32x2*>(orow + d) = v;
        if (out_pack)
          *reinterpret_cast<u32x2*>(out_pack + pack_off(b, (h0 + j) * AD6_DH + d, H * AD6_DH)) = v;
      }
    }
  } else {
    // merge the WPP waves through LDS (the V slots are free once every wave is past its loop)
    __syncthreads();
    float* sm_o = reinterpret_cast<float*>(lds6);               // [WPP][REP][128]
    float* sm_ml = sm_o + WPP * REP * AD6_DH;                    // [WPP][REP][2]
    if (j < REP) {
#pragma unroll
      for (int dt = 0; dt < 8; ++dt)
        *reinterpret_cast<f32x4*>(sm_o + (w * REP + j) * AD6_DH + 16 * dt + 4 * c) = o[dt];
      if (c == 0) {
        sm_ml[(w * REP + j) * 2] = m_run;
        sm_ml[(w * REP + j) * 2 + 1] = l_run;
      }
    }
    __syncthreads();
    // REP x 16 chunks of 8 dims
    for (int t = threadIdx.x; t < REP * 16; t += WPP * 64) {
      const int h = t >> 4, d0 = 8 * (t & 15);
      float M = -INFINITY;
#pragma unroll
      for (int ww = 0; ww < WPP; ++ww) M = fmaxf(M, sm_ml[(ww * REP + h) * 2]);
      float num[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, den = 0.f;
      if (M != -INFINITY) {
#pragma unroll
        for (int ww = 0; ww < WPP; ++ww) {
          const float mw = sm_ml[(ww * REP + h) * 2];
          const float f = mw == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mw - M);
          den += f * sm_ml[(ww * REP + h) * 2 + 1];
          const float* src = sm_o + (ww * REP + h) * AD6_DH + d0;
#pragma unroll
          for (int e = 0; e < 8; ++e) num[e] += f * src[e];
        }
      }
      const float inv = den > 0.f ? 1.f / den : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) num[e] *= inv;
      const u32x4 v = pack8(num);
      *reinterpret_cast<u32x4*>(out + ((size_t)b * H + h0 + h) * AD6_DH + d0) = v;
      if (out_pack) *reinterpret_cast<u32x4*>(out_pack + pack_off(b, (h0 + h) * AD6_DH + d0, H * AD6_DH)) = v;
    }
  }
}

// waves per (row, kv head) pair: enough workgroups to cover the CUs, fewer waves (less merge) for many pairs;
// attn_set_v6_wpp pins it (A/B)
static int g_v6_wpp = 0;
void attn_set_v6_wpp(int wpp) { g_v6_wpp = (wpp == 1 || wpp == 2 || wpp == 4 || wpp == 8) ? wpp : 0; }
int attn_v6_wpp(int pairs) {
  if (g_v6_wpp) return g_v6_wpp;
  return pairs >= 4096 ? 1 : 2;  // 2 waves were best or tied from 1 to 256 pairs (r5_attn_decode_v6_ab.jsonl)
}

int attn_decode_v6(const bf16_t* q, const bf16_t* kc, const bf16_t* vc, const int32_t* slot, const int32_t* kv_start,
                   const uint8_t* key_mask, int mask_len, bf16_t* out, int B, int H, int Hkv, int T, int t_cap,
                   hipStream_t s, bf16_t* out_pack) {
  const int rep = H / Hkv, pairs = B * Hkv;
  const float scale_log2 = 1.4426950408889634f / sqrtf((float)AD6_DH);
  const int wpp = attn_v6_wpp(pairs);
#define JLA_AD6(R, W)                                                                                              \
  if (rep == R && wpp == W) {                                                                                      \
    attn_decode_v6_kernel<R, W><<<pairs, W * 64, W * AD6_WAVE_LDS, s>>>(q, kc, vc, slot, kv_start, key_mask,       \
                                                                         mask_len, out, H, Hkv, T, t_cap,          \
                                                                         scale_log2, out_pack);                    \
    JLA_CHECK_LAUNCH();                                                                                            \
    return 0;                                                                                                      \
  }
  JLA_AD6(4, 1) JLA_AD6(4, 2) JLA_AD6(4, 4) JLA_AD6(4, 8)
  JLA_AD6(8, 1) JLA_AD6(8, 2) JLA_AD6(8, 4) JLA_AD6(8, 8)
  JLA_AD6(1, 1) JLA_AD6(1, 2) JLA_AD6(1, 4) JLA_AD6(1, 8)
  JLA_AD6(2, 1) JLA_AD6(2, 2) JLA_AD6(2, 4) JLA_AD6(2, 8)
  JLA_AD6(16, 1) JLA_AD6(16, 2) JLA_AD6(16, 4) JLA_AD6(16, 8)
#undef JLA_AD6
  return -1;
}

}  // namespace jla
