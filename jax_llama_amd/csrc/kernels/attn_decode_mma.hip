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
#include "attn_mma.h"
#include "common.h"
#include "launchers.h"
#include "ring.h"

namespace jla {

// DIAG (tools only, attn_set_v6_diag; wrong results): 1 = no compute, 2 = no K loads, 4 = no V DMAs
template <int REP, int WPP, int DIAG = 0>
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

  // Q^T fragments (attn_mma.h); a wait hipcc sees: otherwise it places a vmcnt(0) for these loads inside the loop,
  // behind the hand-counted ring
  u32x4 qf[4];
  ad6_load_q<REP, false>(qf, q + ((size_t)b * H + h0) * AD6_DH, lane);
  ::wait_vmcnt<0>();
  ad6_q_ready<REP>(qf, lane);

  const int s_begin = lo >= 0 ? lo / AD6_STEP : 0;
  const int n_steps = lo < hi ? (hi - 1) / AD6_STEP - s_begin + 1 : 0;
  const int my_steps = n_steps > w ? (n_steps - w + WPP - 1) / WPP : 0;
  auto issue = [&](int step, u32x4 (&kr)[8], char* vslot) {
    ad6_issue<false, DIAG>((s_begin + step) * AD6_STEP, kr, vslot, kb, vb, T, lane);
  };
  constexpr int NV = (DIAG & 2 ? 0 : 8) + (DIAG & 4 ? 0 : 8);  // vector-memory ops per step
  Ad6Acc st;
  ad6_init(st);
  // valid = false: a ring slot loaded past the wave's last step (clamped addresses, fully masked, adds nothing)
  auto compute = [&](int step, bool valid, u32x4 (&kr)[8], const char* vslot) {
    if constexpr (DIAG & 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) pin(kr[i]);
    } else {
      ad6_compute<REP>(st, kr, qf, vslot, (s_begin + step) * AD6_STEP, valid, lo, hi, mrow, mask_len, scale_log2, lane);
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
      wait_vmcnt<NV>();  // step i (slot A) landed; step i + 1 stays in flight
      compute(step_of(i), true, ka, slotA);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot A's V reads are done: refill it
      issue(step_of(i + 2), ka, slotA);
      wait_vmcnt<NV>();
      compute(step_of(i + 1), i + 1 < my_steps, kb2, slotB);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    wait_vmcnt<0>();  // the last refill of slot A: drained before the LDS is reused or the wave ends
  }

  ad6_finish(st);
  const float m_run = st.m, l_run = st.l;
  f32x4 (&o)[8] = st.o;
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
static int g_v6_diag = 0;
void attn_set_v6_diag(int d) { g_v6_diag = d & 7; }
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
  if (g_v6_diag && rep == 8 && wpp == 2) {  // tools only: the ablation instances of the 70B shape (wrong results)
#define JLA_AD6D(D)                                                                                                \
  if (g_v6_diag == D) {                                                                                            \
    attn_decode_v6_kernel<8, 2, D><<<pairs, 128, 2 * AD6_WAVE_LDS, s>>>(q, kc, vc, slot, kv_start, key_mask,       \
                                                                         mask_len, out, H, Hkv, T, t_cap,          \
                                                                         scale_log2, out_pack);                    \
    JLA_CHECK_LAUNCH();                                                                                            \
    return 0;                                                                                                      \
  }
    JLA_AD6D(1) JLA_AD6D(2) JLA_AD6D(3) JLA_AD6D(4) JLA_AD6D(5)
#undef JLA_AD6D
  }
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
