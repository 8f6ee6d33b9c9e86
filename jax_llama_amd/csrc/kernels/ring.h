// Register load ring helpers of the decode GEMV (gemv.hip).
#pragma once
#include "common.h"

namespace jla {

// Loads of the main loop are issued as inline asm so the ring's waits are counted by hand:
// hipcc's own waitcnt insertion drains the whole ring (vmcnt(0)) at the loop back-edge, which turns
// the pipeline back into batches (checked in the .s). Each slot is waited with one counted
// s_waitcnt vmcnt(L*(U-1)) and its registers are pinned behind that wait ("+v"), so no consumer
// can read them early (cdna_hip_programming.md section 5.7, form (ii)).
// The destination is a "+v" (tied) operand: the ring slot is one variable whose register the
// allocator keeps across the loop back-edge (no phi copies of in-flight registers; verified by
// tools/check_asm_ring.py on the generated assembly).
// With ASM = false (used where register pressure makes the allocator shuffle ring registers,
// i.e. MT > 1) the same ring uses ordinary compiler-counted loads: always correct, sometimes
// drained at the back-edge. build.py runs tools/check_asm_ring.py on every build.
template <bool ASM>
JLA_DEV void asm_load_nt(u32x4& r, const void* p) {
  if constexpr (ASM)
    asm volatile("global_load_dwordx4 %0, %1, off nt" : "+v"(r) : "v"(p) : "memory");
  else
    r = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}
template <bool ASM>
JLA_DEV void asm_load(u32x4& r, const void* p) {
  if constexpr (ASM)
    asm volatile("global_load_dwordx4 %0, %1, off" : "+v"(r) : "v"(p) : "memory");
  else
    r = *reinterpret_cast<const u32x4*>(p);
}
template <bool ASM>
JLA_DEV void asm_load16(u32x4& r, const void* p) {
  if constexpr (ASM)
    asm volatile("global_load_dwordx4 %0, %1, off offset:16" : "+v"(r) : "v"(p) : "memory");
  else
    r = reinterpret_cast<const u32x4*>(p)[1];
}
// agent-coherent (sc1) load: bypasses the caches that can hold a stale copy of a line another
// workgroup of the same launch wrote write-through (in-launch hand-offs, Guideline 16 R1)
JLA_DEV void asm_load_sc1(u32x4& r, const void* p) {
  asm volatile("global_load_dwordx4 %0, %1, off sc1" : "+v"(r) : "v"(p) : "memory");
}
// LDS-DMA with the agent-coherent (sc1) policy: rows another workgroup of the same launch wrote write-through
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
JLA_DEV void glds16_asm_sc1(const void* gsrc, void* lds_wave_base) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)(__attribute__((address_space(3))) char*)lds_wave_base);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off sc1" ::"v"(gsrc), "s"(m0)
               : "memory", "m0");
}
#pragma clang diagnostic pop

// write-through (sc1) store: the producer side of the same hand-off. hipcc's hazard recognizer does not see into the
// asm, and a store of more than 8 bytes reads its upper data dwords after issue: the s_nop is the wait state a VALU
// write of those registers right behind the store needs (without it lanes' upper dwords came out corrupted).
JLA_DEV void st_sc1_x4(void* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
template <int N>
JLA_DEV void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
JLA_DEV void pin(u32x4& r) { asm volatile("" : "+v"(r)); }

template <typename XT>
struct XRaw;

template <>
struct XRaw<float> {  // 8 fp32 activations per lane (two 16-byte loads)
  static constexpr int LOADS = 2;
  u32x4 a, b;
  template <bool ASM>
  JLA_DEV void load(const float* p) {
    asm_load<ASM>(a, p);
    asm_load16<ASM>(b, p);
  }
  JLA_DEV void pin_regs() {
    pin(a);
    pin(b);
  }
  JLA_DEV u32x4 frag(float& ss) const {
    float f[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[i] = __uint_as_float(a[i]);
      f[4 + i] = __uint_as_float(b[i]);
    }
    u32x4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ss += f[2 * i] * f[2 * i] + f[2 * i + 1] * f[2 * i + 1];
      r[i] = pack2bf(f[2 * i], f[2 * i + 1]);
    }
    return r;
  }
};

template <>
struct XRaw<bf16_t> {  // 8 bf16 activations per lane (one 16-byte load)
  static constexpr int LOADS = 1;
  u32x4 v;
  template <bool ASM>
  JLA_DEV void load(const bf16_t* p) {
    asm_load<ASM>(v, p);
  }
  JLA_DEV void pin_regs() { pin(v); }
  // sum of squares straight from the packed pairs (v_dot2_f32_bf16): no unpacked temporaries, which at
  // MT > 1 made hipcc copy in-flight ring registers (tools/check_asm_ring.py hazards) and forced the
  // compiler-counted ring that drains at every back-edge. dot8_bf16 bit-casts the WHOLE vector: casting
  // single elements (v[i]) into the dot2 operand miscompiles to element 0 for every i.
  JLA_DEV u32x4 frag(float& ss) const {
    ss = dot8_bf16(v, v, ss);
    return v;
  }
};

}  // namespace jla
