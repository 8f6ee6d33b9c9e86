// Fused RoPE + KV-cache write (reference: apply_rotary_emb model.py:58-92 with Meta's interleaved
// (complex-pair) layout; cache update _concatenate_to_cache model.py:169-199).
//
// Input is the fused projection row qkv[m] = [q (H*Dh) | k (Hkv*Dh) | v (Hkv*Dh)] in bf16. One
// 16-byte vector (4 rotation pairs) per thread: q is rotated into q_out, k is rotated and v copied
// straight into the [B, Hkv, T, Dh] cache at slot slot0 + s, where slot0 is read from device
// memory so the same launch is replayed by the decode hipGraph at every step. RoPE math is fp32
// from an fp32 (cos, sin) table (never bf16, unlike a naive port of precompute_freqs_cis).
#include "common.h"
#include "launchers.h"

namespace jla {

__global__ void __launch_bounds__(256)
    rope_kv_kernel(const bf16_t* __restrict__ qkv, const float2* __restrict__ table, int table_len,
                   const int32_t* __restrict__ positions, bf16_t* __restrict__ kc, bf16_t* __restrict__ vc,
                   const int32_t* __restrict__ slot_ptr, int S, int H, int Hkv, int Dh, int T,
                   bf16_t* __restrict__ q_out) {
  const int m = blockIdx.x;
  const int b = m / S, s = m - b * S;
  const int vec_per_head = Dh >> 3;
  const int nvec = (H + 2 * Hkv) * vec_per_head;
  int pos = positions[m];
  if (pos < 0 || pos >= table_len) JLA_FLAG(JLA_BOUNDS_ROPE_POS);
  pos = pos < 0 ? 0 : (pos >= table_len ? table_len - 1 : pos);
  const int slot = slot_ptr[0] + s;
  const u32x4* row = reinterpret_cast<const u32x4*>(qkv + (size_t)m * (H + 2 * Hkv) * Dh);
  for (int v = threadIdx.x; v < nvec; v += blockDim.x) {
    const int head = v / vec_per_head, d0 = (v - head * vec_per_head) * 8;
    u32x4 val = row[v];
    if (head < H + Hkv) {
      float f[8];
      unpack8(val, f);
      const float2* cs = table + (size_t)pos * (Dh >> 1) + (d0 >> 1);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const float2 t = cs[p];
        const float xr = f[2 * p], xi = f[2 * p + 1];
        f[2 * p] = xr * t.x - xi * t.y;
        f[2 * p + 1] = xr * t.y + xi * t.x;
      }
      val = pack8(f);
    }
    if (head < H) {
      reinterpret_cast<u32x4*>(q_out + ((size_t)m * H + head) * Dh + d0)[0] = val;
    } else if (slot < T) {
      const int kh = head < H + Hkv ? head - H : head - H - Hkv;
      bf16_t* cache = head < H + Hkv ? kc : vc;
      reinterpret_cast<u32x4*>(cache + (((size_t)b * Hkv + kh) * T + slot) * Dh + d0)[0] = val;
    } else {
      JLA_FLAG(JLA_BOUNDS_KV_SLOT);
    }
  }
}

int rope_kv_write(const bf16_t* qkv, const float* table, int table_len, const int32_t* positions, bf16_t* kc,
                  bf16_t* vc, const int32_t* slot, int M, int S, int H, int Hkv, int Dh, int T, bf16_t* q_out,
                  hipStream_t s) {
  if (M <= 0) return 0;
  if (Dh % 8 || S <= 0 || M % S) return -1;
  rope_kv_kernel<<<M, 256, 0, s>>>(qkv, reinterpret_cast<const float2*>(table), table_len, positions, kc, vc, slot,
                                   S, H, Hkv, Dh, T, q_out);
  JLA_CHECK_LAUNCH();
  return 0;
}

JLA_BOUNDS_ACCESSOR(rope_kv)

}  // namespace jla
