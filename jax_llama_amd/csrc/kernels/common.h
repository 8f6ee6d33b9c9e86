// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels of jax_llama_amd.
//
// Conventions
//  * bf16 is carried as raw uint16_t (``bf16_t``) and converted with explicit round-to-nearest-even,
//    matching torch's float->bfloat16 cast bit for bit (the CPU reference path relies on this).
//  * Linear weights use the MFMA fragment-packed layout (see ops/reference.py: pack_frag16x32):
//        P[nt][ks][lane][e] = W[16*nt + (lane & 15)][32*ks + 8*(lane >> 4) + e]
//    so one 16(n) x 32(k) block is the B operand of one v_mfma_f32_16x16x32_bf16 and one 1 KiB
//    contiguous run that a wave fetches with a single global_load_dwordx4 per lane.
//  * Waves are 64 lanes. Block sizes are multiples of 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// Linear epilogue modes (mirrors ops/__init__.py)
#define MODE_STORE 0
#define MODE_RESIDUAL 1
#define MODE_SWIGLU 2
#define MODE_QKV 3
#define MODE_ARGMAX 8
#define MODE_TPRESID 9  // row-parallel partial -> granule all-reduce over the TP group -> residual (gemv.hip)

// ---- bounds-checked debug build (python build.py --debug-bounds -> jax_llama_amd/_C_dbg*.so, loaded when
// JLA_DEBUG_BOUNDS=1). The kernels clamp or skip out-of-range indices that come from device state (token ids,
// the KV-cache slot counter, RoPE positions, the sequence length): in a release build silently, in the debug
// build each such event also sets a bit in this translation unit's error word (a vector atomic OR), which the
// host reads with ops.bounds_error() / raises on in ops.check_bounds(). Bit = JLA_BOUNDS_* code.
#define JLA_BOUNDS_TOKEN 0      // token id outside [0, vocab)
#define JLA_BOUNDS_KV_SLOT 1    // KV-cache write at slot >= T (cache full)
#define JLA_BOUNDS_SEQ 2        // decode step past the sequence buffer
#define JLA_BOUNDS_ATTN_T 3     // attention asked for keys past the cache (slot >= T)
#define JLA_BOUNDS_ROPE_POS 4   // position outside the RoPE table
#ifdef JLA_DEBUG_BOUNDS
static __device__ unsigned int g_jla_bounds_err;
#define JLA_FLAG(code) atomicOr(&g_jla_bounds_err, 1u << (code))
#define JLA_BOUNDS_ACCESSOR(tu)                                                     \
  unsigned jla_bounds_##tu(int reset) {                                             \
    unsigned v = 0;                                                                 \
    (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_jla_bounds_err), sizeof(v));         \
    if (reset) {                                                                    \
      const unsigned z = 0;                                                         \
      (void)hipMemcpyToSymbol(HIP_SYMBOL(g_jla_bounds_err), &z, sizeof(z));         \
    }                                                                               \
    return v;                                                                       \
  }
#else
#define JLA_FLAG(code) ((void)0)
#define JLA_BOUNDS_ACCESSOR(tu) \
  unsigned jla_bounds_##tu(int) { return 0; }
#endif  // greedy lm_head: first-max (value, index) partials instead of logits

#define JLA_DEV __device__ __forceinline__

JLA_DEV float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// fp32 -> bf16 round-to-nearest-even: gfx950's v_cvt_pk_bf16_f32 (one instruction for two values,
// no branches); bit-identical to torch's float->bfloat16 cast for finite values.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

JLA_DEV bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

JLA_DEV uint32_t pack2bf(float lo, float hi) {
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// unpack the 8 bf16 of a 16-byte vector into floats
JLA_DEV void unpack8(const u32x4 v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}

JLA_DEV u32x4 pack8(const float* f) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = pack2bf(f[2 * i], f[2 * i + 1]);
  return r;
}

// acc + sum_e a[e] * b[e] over the 8 bf16 of two 16-byte vectors (4 x v_dot2_f32_bf16, fp32 accumulate).
// Whole-vector bit casts + literal shuffles: bit-casting single ext-vector elements miscompiles here.
JLA_DEV float dot8_bf16(const u32x4 a, const u32x4 b, float acc) {
  const bf16x8_t x = __builtin_bit_cast(bf16x8_t, a), y = __builtin_bit_cast(bf16x8_t, b);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(x, x, 0, 1), __builtin_shufflevector(y, y, 0, 1), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(x, x, 2, 3), __builtin_shufflevector(y, y, 2, 3), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(x, x, 4, 5), __builtin_shufflevector(y, y, 4, 5), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(x, x, 6, 7), __builtin_shufflevector(y, y, 6, 7), acc, false);
  return acc;
}

// "Packed" activation layout: the MFMA A fragments of x [M, K] stored contiguously, [ceil(M/16)][K/32][64][8]
// (one 1 KiB run per 16-row x 32-k fragment, like the packed weights). Element (m, k) lives at pack_off(m, k, K).
// Written beside the row-major copy by the decode epilogues that produce the next projection's input, read by the
// GEMV's packed-x variants (12-15): one contiguous 1 KiB load per fragment instead of 16 half-used 128-B lines.
JLA_DEV size_t pack_off(int m, int k, int K) {
  return ((size_t)((m >> 4) * (K >> 5) + (k >> 5)) * 64 + (m & 15) + 16 * ((k & 31) >> 3)) * 8 + (k & 7);
}

JLA_DEV f32x4 mfma16x16x32(const u32x4 a, const u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

// LDS-DMA: 16 bytes per lane from a per-lane global address into LDS at (wave-uniform base + 16*lane).
JLA_DEV void glds16(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}
// The same DMA as inline asm: hipcc's waitcnt pass does not see it write LDS, so it adds no vmcnt(0) before LDS
// reads it cannot prove disjoint from the DMA target (with the builtin, a read of ring slot i waits for the DMA into
// slot i + 1 issued just before it). The caller owns the wait: s_waitcnt vmcnt before the barrier that publishes
// the slot. (Loads the compiler counts stay safe: a DMA it does not count only makes its own waits stronger.)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved: nothing else in these kernels keeps a value in it
JLA_DEV void glds16_asm(const void* gsrc, void* lds_wave_base) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)(__attribute__((address_space(3))) char*)lds_wave_base);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(m0) : "memory", "m0");
}
#pragma clang diagnostic pop
// s_waitcnt vmcnt(N) only (expcnt/lgkmcnt left at their maxima)
template <int N>
JLA_DEV void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt(0xF70 | (N & 15) | ((N >> 4) << 14));
}

// Non-temporal 16-byte load for once-read streams (decode weights).
JLA_DEV u32x4 load_nt(const u32x4* p) { return __builtin_nontemporal_load(p); }

JLA_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

JLA_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024; `red` must hold >= 16 floats. All threads get the result.
JLA_DEV float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

JLA_DEV float silu(float x) { return x / (1.f + __expf(-x)); }

// DPP lane moves within a 16-lane row (no LDS traffic, unlike __shfl_xor's ds_bpermute).
template <int CTRL>
JLA_DEV float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// Sum over the 16 lanes of each row; every lane receives the row total.
JLA_DEV float row16_sum(float v) {
  v += dppf<0xB1>(v);   // quad_perm [1,0,3,2]  (xor 1)
  v += dppf<0x4E>(v);   // quad_perm [2,3,0,1]  (xor 2)
  v += dppf<0x141>(v);  // row_half_mirror      (other quad of the 8-lane half)
  v += dppf<0x140>(v);  // row_mirror           (other half of the row)
  return v;
}

// Host-side error check used by every launcher.
#define JLA_CHECK_LAUNCH()                                                        \
  do {                                                                            \
    hipError_t e__ = hipGetLastError();                                           \
    if (e__ != hipSuccess) return (int)e__;                                       \
  } while (0)
