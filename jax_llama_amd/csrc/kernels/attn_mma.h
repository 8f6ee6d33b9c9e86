// Building blocks of the matrix-core decode attention (attn_decode_mma.hip v6, and the attention workgroups fused
// into the small-batch qkv launch, gemv.hip qkv_attn_kernel): one wave processes 32-key steps of one (row, kv head)
// pair with the REP q heads as the 16 columns of a v_mfma_f32_16x16x32_bf16 tile.
//   S^T = K Q^T : 2 key blocks x 4 dk steps = 8 MFMAs (A = K rows straight from global memory into VGPRs: lane
//                 (key l & 15, group c = l >> 4) holds dims 32j + 8c .. +7 of its key for dk step j, so the 4 lanes of
//                 a key read 64 contiguous bytes per load; the Q^T fragments use the same dim permutation)
//   O^T += V^T P^T : 8 dim tiles of 16 = 8 MFMAs (A = V^T by ds_read_b64_tr_b16 from a row-major V image in LDS, B =
//                 the bf16 P of the lane's own 8 scores: the S^T accumulator layout IS the P^T operand layout once the
//                 k slots are ordered keys {4c .. 4c+3, 16+4c .. 16+4c+3})
// Online softmax in the log2 domain, lane-local (one head per lane column) plus two cross-group max exchanges per
// step, with the flash prefill's lazy rescale (the running max moves only when it grows by more than 8).
// Reference ops: jax_llama/model.py:277-291 (scores, softmax, P.V) over the cache (:169-199), GQA by indexing.
#pragma once
#include "common.h"
#include "ring.h"

namespace jla {

constexpr int AD6_DH = 128;
constexpr int AD6_STEP = 32;                           // keys per step
constexpr int AD6_SLOT_BYTES = AD6_STEP * AD6_DH * 2;  // 8 KiB of V per step
constexpr int AD6_WAVE_LDS = 2 * AD6_SLOT_BYTES;       // two V slots per wave

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

// per-wave online-softmax state of one pair: running max (log2 units), running sum, O^T accumulators (AGPRs)
struct Ad6Acc {
  float m, l;
  f32x4 o[8];
};
JLA_DEV void ad6_init(Ad6Acc& a) {
  a.m = -INFINITY;
  a.l = 0.f;
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) a.o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// Q^T fragments of the pair's heads (qrow = q of its first head, [REP][128]); zero columns past REP (those lanes
// load head REP - 1 and zero it after the wait: no divergent asm). SC1: q was written in this launch by other
// workgroups (write-through stores): agent-coherent asm loads the CALLER waits for (then ad6_q_ready); otherwise
// plain compiler-tracked loads.
template <int REP, bool SC1>
JLA_DEV void ad6_load_q(u32x4 (&qf)[4], const bf16_t* qrow, int lane) {
  const int c = lane >> 4, j = min(lane & 15, REP - 1);
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const bf16_t* p = qrow + (size_t)j * AD6_DH + 32 * jj + 8 * c;
    if constexpr (SC1) {
      qf[jj] = u32x4{0u, 0u, 0u, 0u};
      asm_load_sc1(qf[jj], p);
    } else {
      qf[jj] = *reinterpret_cast<const u32x4*>(p);
    }
  }
}
template <int REP>
JLA_DEV void ad6_q_ready(u32x4 (&qf)[4], int lane) {  // after the wait that retired ad6_load_q's loads
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    pin(qf[jj]);
    if ((lane & 15) >= REP) qf[jj] = u32x4{0u, 0u, 0u, 0u};
  }
}

// issue one 32-key step starting at key0 (rows clamped to T - 1): V rows into vslot by LDS-DMA (1 KiB block bi = rows
// 4bi .. 4bi+3, lane L -> row 4bi + L / 16, slot L % 16 <- source chunk slot ^ swz(row)), K rows into kr by asm loads
// (key l & 15 of block kk, bytes 64jj + 16c). 16 vector-memory ops; the caller counts the waits. SC1: agent-coherent.
// DIAG (tools only, wrong results): 2 = no K loads, 4 = no V DMAs
template <bool SC1, int DIAG = 0>
JLA_DEV void ad6_issue(int key0, u32x4 (&kr)[8], char* vslot, const bf16_t* kb, const bf16_t* vb, int T, int lane) {
  const int c = lane >> 4, j = lane & 15;
#pragma unroll
  for (int bi = 0; bi < 8; ++bi) {
    if constexpr (DIAG & 4) break;
    const int row = 4 * bi + (lane >> 4);
    const int ch = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
    const int key = min(key0 + row, T - 1);
    if constexpr (SC1)
      glds16_asm_sc1(vb + (size_t)key * AD6_DH + 8 * ch, vslot + 1024 * bi);
    else
      glds16_asm(vb + (size_t)key * AD6_DH + 8 * ch, vslot + 1024 * bi);
  }
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    if constexpr (DIAG & 2) break;
    const int key = min(key0 + 16 * kk + j, T - 1);
    const bf16_t* p = kb + (size_t)key * AD6_DH + 8 * c;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      if constexpr (SC1)
        asm_load_sc1(kr[4 * kk + jj], p + 32 * jj);
      else
        asm_load<true>(kr[4 * kk + jj], p + 32 * jj);
    }
  }
}

// scores, online softmax and P.V of the step at key0 (its loads have landed: the caller waited). Keys outside
// [lo, hi) or masked are -inf; valid = false masks the whole step (a ring slot loaded past the wave's last step).
template <int REP>
JLA_DEV void ad6_compute(Ad6Acc& st, u32x4 (&kr)[8], const u32x4 (&qf)[4], const char* vslot, int key0, bool valid,
                         int lo, int hi, const uint8_t* mrow, int mask_len, float scale_log2, int lane) {
  const int c = lane >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) pin(kr[i]);
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    s0 = mfma16x16x32(kr[jj], qf[jj], s0);
    s1 = mfma16x16x32(kr[4 + jj], qf[jj], s1);
  }
  // lane (c, j): s0[r] = score of key key0 + 4c + r, s1[r] = key key0 + 16 + 4c + r, head j
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
  if (__ballot(tmax > st.m + 8.f)) {  // lazy rescale
    const float m_new = fmaxf(st.m, tmax);
    const float alpha = __builtin_amdgcn_exp2f(st.m - (m_new == -INFINITY ? 0.f : m_new));
    st.l *= alpha;
    st.m = m_new;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      f32x4 t = ad6_take(st.o[dt]);
      t *= alpha;
      ad6_put(st.o[dt], t);
    }
  }
  const float m_use = st.m == -INFINITY ? 0.f : st.m;
  float p[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    p[e] = __builtin_amdgcn_exp2f(sc[e] - m_use);
    st.l += p[e];
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
    ad6_mfma_acc(st.o[dt], u32x4{a[0], a[1], bb[0], bb[1]}, pf);
  }
}

// per wave after its last step: the accumulators out of the AGPRs, the row sum over the 4 lane groups (the running
// max is already shared by them). Lane (c, j) then holds O[head j][dims 16dt + 4c + r] in o[dt][r].
JLA_DEV void ad6_finish(Ad6Acc& st) {
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) st.o[dt] = ad6_take(st.o[dt]);
  st.l += __shfl_xor(st.l, 16, 64);
  st.l += __shfl_xor(st.l, 32, 64);
}

}  // namespace jla
