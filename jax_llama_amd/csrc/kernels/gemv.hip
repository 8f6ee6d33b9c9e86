// Skinny (decode) linear layer: y[M, N] = epilogue( [inv_rms(x) *] x[M, K] @ W[N, K]^T ), M <= 64.
//
// Reference ops: every nn.Dense of model.py (wq/wk/wv :210, wo :294, w1/w3/w2 :338, lm_head :736)
// plus the RMSNorm that precedes qkv / w1|w3 / lm_head (model.py:384, :395, :662), the residual
// adds (:392, :398), and -- for the fused qkv projection -- RoPE + the KV-cache write
// (apply_rotary_emb :58-92, _concatenate_to_cache :169-199).
//
// Decode is HBM-bound on the weight stream (batch 1..64 rows), so the kernel is organised around
// streaming the packed weights exactly once at full bandwidth:
//   * one workgroup = NT consecutive 16-column n-tiles x the WHOLE K, split across NW waves
//     (intra-workgroup split-K: wave w takes k-steps w, w+NW, ... so the waves of a workgroup
//     fetch consecutive KiB of the n-tile's contiguous packed block);
//   * each k-step is one 1 KiB non-temporal global_load_dwordx4 per n-tile (already the B operand
//     of v_mfma_f32_16x16x32_bf16) plus the 16(m) x 32(k) activation fragment (L2-resident x);
//   * the main loop is a rolling register pipeline: U slots, each slot refilled with the k-step
//     U ahead right after its MFMA, so every wave keeps U KiB (x NT) in flight at all times with
//     no branches and no vmcnt(0) (past-the-end refills read a zero fragment: MFMA adds 0);
//   * MT = ceil(M/16) m-tiles reuse each weight fragment (M <= 16 costs the same as M = 1);
//   * RMSNorm's sum of squares comes from the same activation loads (each x element is loaded
//     exactly once per workgroup): no extra pass, no extra launch;
//   * partial accumulators are reduced through LDS; the fused epilogue applies the norm scale and
//     stores bf16/fp32, accumulates into the fp32 residual stream, applies SiLU(gate)*up over the
//     interleaved [w1;w3] weight, or (QKV mode) rotates q/k pairs with RoPE and writes q plus the
//     k/v cache rows at the device-side cache slot.
// No atomics: results are deterministic and the residual add happens exactly once.
#include "attn_mma.h"
#include "car.h"
#include "common.h"
#include "launchers.h"
#include "ring.h"

namespace jla {

__device__ u32x4 g_zero_frag[64];  // 1 KiB of zeros (static storage is zero-initialised)

// 2-byte agent-coherent (sc1, write-through) store: outputs another workgroup of the SAME launch reads (the qkv
// epilogue of the fused qkv + attention launch)
JLA_DEV void st_sc1_b16(bf16_t* p, bf16_t v) {
  asm volatile("global_store_short %0, %1, off sc1" ::"v"(p), "v"((unsigned)v) : "memory");
}

// The epilogue of one skinny workgroup: the cross-wave reduction of its accumulators (and RMS row sums) through LDS,
// then the MODE's fused output. Shared by skinny_body and the o-projection workgroups of the fused decode launch.
template <int MT, int NT, int MODE, int NW, bool SPLIT, bool SC1>
JLA_DEV void skinny_epilogue(const f32x4 (&acc)[MT][NT], const float (&ss)[MT], int tp_calls, void* __restrict__ out,
                             int M, int N, int K, float eps, int use_rms, int accumulate, int out_f32,
                             const QKVArgs& qa, int bx, int by, int gy) {
  extern __shared__ float smem[];
  float* red = smem;                              // [NW][MT][NT][64][4]
  float* red_ss = red + NW * MT * NT * 256;       // [NW][MT][16]
  float* inv_rms = red_ss + NW * MT * 16;         // [MT*16]
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int NTT = N >> 4;
  const int nt0 = bx * NT;
  // the residual values this thread's epilogue elements add to, loaded now: the load's round trip hides behind the
  // LDS reduction (and, with the TP exchange, behind its granule round trips) instead of following them
  constexpr int EPT = (MT * NT * 256 + NW * 64 - 1) / (NW * 64);  // epilogue elements per thread
  float hpre[EPT];     // MODE_RESIDUAL: h at (m, col)
  float2 hpre2[EPT];   // MODE_TPRESID: h at (m, col .. col + 1), even columns
  int ppre[EPT];       // MODE_QKV: the element's row position (its RoPE factor is one dependent load fewer later)
  if constexpr (MODE == MODE_QKV) {
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const int e = threadIdx.x + j * NW * 64;
      const int m = (e / (256 * NT)) * 16 + ((e >> 4) & 15);
      ppre[j] = qa.positions[min(m, M - 1)];
    }
  }
  if constexpr (MODE == MODE_RESIDUAL || MODE == MODE_TPRESID) {
    const float* h = static_cast<const float*>(out);
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const int e = threadIdx.x + j * NW * 64;
      const int c = e & 15, ml = (e >> 4) & 15, t = (e >> 8) % NT, mt = e / (256 * NT);
      const int m = mt * 16 + ml;
      const bool ok = e < MT * NT * 256 && m < M && nt0 + t < NTT;
      const size_t idx = (size_t)m * N + (nt0 + t) * 16 + c;
      if constexpr (MODE == MODE_RESIDUAL) {
        hpre[j] = ok && accumulate ? h[idx] : 0.f;
      } else {
        hpre2[j] = ok && !(c & 1) ? *reinterpret_cast<const float2*>(h + idx) : make_float2(0.f, 0.f);
      }
    }
  }

  // ---- cross-wave reduction through LDS
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t)
      *reinterpret_cast<f32x4*>(red + (((w * MT + mt) * NT + t) * 64 + lane) * 4) = acc[mt][t];
  if (use_rms) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      float s = ss[mt];
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      if (lane < 16) red_ss[(w * MT + mt) * 16 + lane] = s;
    }
  }
  if constexpr (MODE == MODE_TPRESID) {
    if (threadIdx.x == 0) reinterpret_cast<int*>(inv_rms + MT * 16)[0] = tp_calls + 1;
  }
  __syncthreads();
  // SPLIT: the workgroup's wave-summed partial (and RMS row sums) go to its own slab with write-through (sc1) stores;
  // every storing wave drains them, one agent-scope ticket add per workgroup picks the group's last arriver, which
  // sums the splits in split order (sc1 loads: cdna_hip_programming.md Guideline 16, sc1-store + agent ticket +
  // sc1-load form) into wave 0's slot of `red` and runs the normal epilogue from there. Deterministic; the
  // ticket resets itself for the next call.
  constexpr int NWR = SPLIT ? 1 : NW;  // wave slots of `red` / `red_ss` the epilogue sums
  if constexpr (SPLIT) {
    constexpr int E = MT * NT * 256, SLAB = E + MT * 16;
    const int ns = gy, grp = bx;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(qa.sk_ws, 0, qa.sk_ws_floats * 4, 0x00020000);
    const int mine = (grp * ns + by) * SLAB * 4;
    for (int e = threadIdx.x; e < E; e += NW * 64) {
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) v += red[ww * E + e];
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, mine + e * 4, 0, 16);
    }
    if (use_rms && threadIdx.x < MT * 16) {
      float v = 0.f;
      for (int ww = 0; ww < NW; ++ww) v += red_ss[ww * MT * 16 + threadIdx.x];
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, mine + (E + threadIdx.x) * 4, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* last_flag = reinterpret_cast<int*>(inv_rms + MT * 16) + 1;
    if (threadIdx.x == 0) {
      const int prev = __hip_atomic_fetch_add(qa.sk_tk + grp, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == ns - 1;
      if (last) __hip_atomic_store(qa.sk_tk + grp, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *last_flag = last;
    }
    __syncthreads();
    if (!*last_flag) return;
    const int first = grp * ns * SLAB * 4;
    for (int e = threadIdx.x; e < E; e += NW * 64) {
      float v = 0.f;
      for (int sp = 0; sp < ns; ++sp)
        v += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, first + (sp * SLAB + e) * 4, 0, 16));
      red[e] = v;
    }
    if (use_rms && threadIdx.x < MT * 16) {
      float v = 0.f;
      for (int sp = 0; sp < ns; ++sp)
        v += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, first + (sp * SLAB + E + threadIdx.x) * 4, 0, 16));
      red_ss[threadIdx.x] = v;
    }
    __syncthreads();
  }
  if (threadIdx.x < MT * 16) {
    float r = 1.f;
    if (use_rms) {
      float s = 0.f;
      for (int ww = 0; ww < NWR; ++ww) s += red_ss[ww * MT * 16 + threadIdx.x];
      r = rsqrtf(s / (float)K + eps);
    }
    inv_rms[threadIdx.x] = r;
  }
  __syncthreads();

  auto reduced = [&](int mt, int t, int ln, int i) {
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < NWR; ++ww) v += red[(((ww * MT + mt) * NT + t) * 64 + ln) * 4 + i];
    return v;
  };

  // ---- fused epilogue; c (column within the tile) is the fastest index -> 64 B row segments
  if constexpr (MODE == MODE_SWIGLU) {
    constexpr int NP = NT / 2;
    const int F = N >> 1;
    bf16_t* o = static_cast<bf16_t*>(out);
    for (int e = threadIdx.x; e < MT * NP * 256; e += NW * 64) {
      const int c = e & 15, ml = (e >> 4) & 15, p = (e >> 8) % NP, mt = e / (256 * NP);
      const int m = mt * 16 + ml;
      const int ln = (ml >> 2) * 16 + c, i = ml & 3;
      const int gtile = nt0 + 2 * p;
      if (m < M && gtile < NTT) {
        const float sc = inv_rms[m];
        const float g = reduced(mt, 2 * p, ln, i) * sc, u = reduced(mt, 2 * p + 1, ln, i) * sc;
        const bf16_t r = f2bf(silu(g) * u);
        o[(size_t)m * F + (gtile >> 1) * 16 + c] = r;
        if (qa.pack) qa.pack[pack_off(m, (gtile >> 1) * 16 + c, F)] = r;
      }
    }
  } else if constexpr (MODE == MODE_TPRESID) {
    // ---- row-parallel partial all-reduced in the epilogue (no separate collective launch): every rank's workgroup
    // bx computes the same (rows, columns) of its own K shard. Each even-column lane packs its value and its
    // neighbour's (RNE to bf16, as the unfused partial) into one 8-byte granule {2 x bf16, tag} and stores it into
    // slot [parity][rank] of every peer (this workgroup's fixed TPRES_REGION), then polls the same granule of every
    // rank's slot in its own buffer until it carries this call's tag, sums in rank order in fp32 and applies the
    // residual epilogue (h += sum, mirror, packed mirror). Workgroup w pairs only with workgroup w of the peers and
    // its counter orders its calls, so the parity argument of allreduce.hip holds per workgroup; bit-identical to
    // partial + car_reduce_kernel (same roundings, same order).
    const CarDevice& d = *static_cast<const CarDevice*>(qa.tp);
    const int calls = reinterpret_cast<const int*>(inv_rms + MT * 16)[0];
    const unsigned tag = gran_tag_fused(calls);
    const long long wg_base = (long long)bx * TPRES_REGION;
    const long long par_base = (long long)(calls & 1) * d.world * d.max_bytes;
    const __amdgpu_buffer_rsrc_t mine = rsrc(d.buf[d.rank]);
    float* h = static_cast<float*>(out);
    for (int e = threadIdx.x; e < MT * NT * 256; e += NW * 64) {
      const int c = e & 15, ml = (e >> 4) & 15, t = (e >> 8) % NT, mt = e / (256 * NT);
      const int m = mt * 16 + ml;
      const int ln = (ml >> 2) * 16 + c, i = ml & 3;
      const float v = reduced(mt, t, ln, i);
      const float vn = __shfl_down(v, 1, 64);  // column c + 1 (lanes e, e + 1 are adjacent)
      if ((c & 1) || m >= M || nt0 + t >= NTT) continue;
      const long long g = wg_base + ((long long)m * (NT * 16) + t * 16 + c) * 4;  // granule (m, c / 2): 8 bytes
      const u32x2 gv = {pack2bf(v, vn), tag};
      for (int p = 0; p < d.world; ++p) st_sys8(rsrc(d.buf[p]), par_base + (long long)d.rank * d.max_bytes + g, gv);
    }
    const bool give_up = __hip_atomic_load(d.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const int e = threadIdx.x + j * NW * 64;
      const int c = e & 15, ml = (e >> 4) & 15, t = (e >> 8) % NT, mt = e / (256 * NT);
      const int m = mt * 16 + ml;
      if (e >= MT * NT * 256 || (c & 1) || m >= M || nt0 + t >= NTT) continue;
      const long long g = wg_base + ((long long)m * (NT * 16) + t * 16 + c) * 4;
      float s0 = 0.f, s1 = 0.f;
      if constexpr (EPT <= 2) {  // every rank's granule in one round trip (the small-batch, latency-bound calls)
        u32x2 r[CAR_MAX_WORLD];
        car_gather8(d, mine, par_base + g, d.max_bytes, tag, give_up, r);
#pragma unroll
        for (int p = 0; p < CAR_MAX_WORLD; ++p) {
          if (p < d.world) {
            s0 += __uint_as_float(r[p][0] << 16);
            s1 += __uint_as_float(r[p][0] & 0xffff0000u);
          }
        }
      } else {  // (more elements per thread: the gather's registers would spill; one round trip per rank)
        for (int p = 0; p < d.world; ++p) {
          const u32x2 r = car_granule(d, mine, par_base + (long long)p * d.max_bytes + g, tag, give_up);
          s0 += __uint_as_float(r[0] << 16);
          s1 += __uint_as_float(r[0] & 0xffff0000u);
        }
      }
      const int col = (nt0 + t) * 16 + c;
      const size_t idx = (size_t)m * N + col;
      const float n0 = hpre2[j].x + s0, n1 = hpre2[j].y + s1;
      *reinterpret_cast<float2*>(h + idx) = make_float2(n0, n1);
      const uint32_t pk = pack2bf(n0, n1);
      if (qa.res_bf16) *reinterpret_cast<uint32_t*>(qa.res_bf16 + idx) = pk;
      if (qa.pack) *reinterpret_cast<uint32_t*>(qa.pack + pack_off(m, col, N)) = pk;
    }
    if (threadIdx.x == 0)
      __hip_atomic_store(d.wg_ctr + bx, calls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const int e = threadIdx.x + j * NW * 64;
      if (e >= MT * NT * 256) break;
      const int c = e & 15, ml = (e >> 4) & 15, t = (e >> 8) % NT, mt = e / (256 * NT);
      const int m = mt * 16 + ml;
      const int ln = (ml >> 2) * 16 + c, i = ml & 3;
      const int tile = nt0 + t;
      if constexpr (MODE == MODE_ARGMAX) {
        // first max of this (row, 16-column tile): (value, index) partial [M][N / 16]; every lane of the
        // 16-lane group takes part in the shuffles (invalid rows/tiles compete with -inf)
        const bool ok = m < M && tile < NTT;
        float bv = ok ? reduced(mt, t, ln, i) * inv_rms[min(m, MT * 16 - 1)] : -INFINITY;
        int bi = ok ? tile * 16 + c : 0x7fffffff;
#pragma unroll
        for (int sh = 1; sh < 16; sh <<= 1) {
          const float ov = __shfl_xor(bv, sh, 64);
          const int oi = __shfl_xor(bi, sh, 64);
          if (ov > bv || (ov == bv && oi < bi)) {
            bv = ov;
            bi = oi;
          }
        }
        if (ok && c == 0) static_cast<float2*>(out)[(size_t)m * NTT + tile] = make_float2(bv, __int_as_float(bi));
        continue;
      }
      if (m >= M || tile >= NTT) continue;
      const float v = reduced(mt, t, ln, i) * inv_rms[m];
      const int col = tile * 16 + c;
      if constexpr (MODE == MODE_QKV) {
        // column -> (head, d); RoPE pairs (d, d^1) are both in this 16-column tile
        const int head = col / qa.Dh, d = col - head * qa.Dh;
        const int b = m / qa.S, s = m - b * qa.S;
        float r = v;
        if (head < qa.H + qa.Hkv) {
          const float pv = reduced(mt, t, ln ^ 1, i) * inv_rms[m];
          int pos = ppre[j];
          if (pos < 0 || pos >= qa.table_len) JLA_FLAG(JLA_BOUNDS_ROPE_POS);
          pos = pos < 0 ? 0 : (pos >= qa.table_len ? qa.table_len - 1 : pos);
          const float2 cs = qa.table[(size_t)pos * (qa.Dh >> 1) + (d >> 1)];
          r = (d & 1) ? (pv * cs.y + v * cs.x) : (v * cs.x - pv * cs.y);
        }
        if (head < qa.H) {
          if constexpr (SC1)
            st_sc1_b16(qa.q + ((size_t)m * qa.H + head) * qa.Dh + d, f2bf(r));
          else
            qa.q[((size_t)m * qa.H + head) * qa.Dh + d] = f2bf(r);
        } else {
          const int slot = qa.slot[0] + s;
          if (slot < qa.T) {
            const bool is_k = head < qa.H + qa.Hkv;
            const int kh = is_k ? head - qa.H : head - qa.H - qa.Hkv;
            bf16_t* cache = is_k ? qa.kc : qa.vc;
            if constexpr (SC1)
              st_sc1_b16(cache + (((size_t)b * qa.Hkv + kh) * qa.T + slot) * qa.Dh + d, f2bf(r));
            else
              cache[(((size_t)b * qa.Hkv + kh) * qa.T + slot) * qa.Dh + d] = f2bf(r);
          } else {
            JLA_FLAG(JLA_BOUNDS_KV_SLOT);
          }
        }
      } else {
        const size_t idx = (size_t)m * N + col;
        if constexpr (MODE == MODE_RESIDUAL) {
          float* o = static_cast<float*>(out);
          const float nv = accumulate ? hpre[j] + v : v;
          o[idx] = nv;
          if (qa.res_bf16) qa.res_bf16[idx] = f2bf(nv);
          if (qa.pack) qa.pack[pack_off(m, col, N)] = f2bf(nv);
        } else {
          if (out_f32)
            static_cast<float*>(out)[idx] = v;
          else
            static_cast<bf16_t*>(out)[idx] = f2bf(v);
        }
      }
    }
  }
}

// The GEMV body of one workgroup (bx: column group, by / gy: K split index / count), shared by linear_skinny_kernel
// and the fused qkv + attention launch. SC1: the QKV epilogue's q / cache stores are write-through (sc1), for the
// attention workgroups of the same launch.
template <typename XT, int MT, int NT, int MODE, int NW, int U, bool XP = false, bool SPLIT = false, bool SC1 = false>
JLA_DEV void skinny_body(const XT* __restrict__ x, const u32x4* __restrict__ W, void* __restrict__ out, int M, int N,
                         int K, float eps, int use_rms, int accumulate, int out_f32, const QKVArgs& qa, int bx, int by,
                         int gy) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar loop control
  const int KS = K >> 5;
  const int NTT = N >> 4;
  const int nt0 = bx * NT;
  // SPLIT: K is cut over gy workgroups per column group; this one streams k-steps [kb, kb + kn)
  int kb = 0, kn = KS;
  if constexpr (SPLIT) {
    kb = (int)((long long)KS * by / gy);
    kn = (int)((long long)KS * (by + 1) / gy) - kb;
  }

  const u32x4* wt[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) wt[t] = W + ((size_t)min(nt0 + t, NTT - 1) * KS + kb) * 64 + lane;
  const XT* xp[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int row = min(mt * 16 + (lane & 15), M - 1);  // padding rows re-read the last row (not stored)
    // XP: activations pre-packed as MFMA A fragments [MT][KS][64 lanes][8] (1 KiB contiguous per k-step,
    // like the weights) instead of row-major (16 rows x 64 B = 16 half-used cache lines per fragment)
    xp[mt] = XP ? x + (((size_t)mt * KS + kb) * 64 + lane) * 8 : x + (size_t)row * K + (size_t)kb * 32 + 8 * (lane >> 4);
  }
  const u32x4* zfrag = g_zero_frag + lane;
  const XT* zx = reinterpret_cast<const XT*>(g_zero_frag);
  // MODE_TPRESID: this workgroup's call counter (parity + granule tag), read now so the uncached round trip hides
  // behind the weight stream
  int tp_calls = 0;
  if constexpr (MODE == MODE_TPRESID) {
    if (threadIdx.x == 0)
      tp_calls = __hip_atomic_load(static_cast<const CarDevice*>(qa.tp)->wg_ctr + bx, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
  }

  const int n = (kn - w + NW - 1) / NW;  // k-steps of this wave: ks = kb + w + i*NW, i < n

  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[mt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) ss[mt] = 0.f;

  u32x4 bq[U][NT] = {};
  XRaw<XT> aq[U][MT] = {};
  constexpr int L = NT + MT * XRaw<XT>::LOADS;  // loads per ring slot
  // hand-counted ring (see asm_load_nt) where the assembly check passes: every bf16-activation
  // variant (the decode path: the residual stream's bf16 mirror) up to 8 waves, single or doubled ring,
  // and fp32 at MT = 1
  constexpr int U_BASE = ((NT == 1 ? 8 : 4) / MT) < 2 ? 2 : ((NT == 1 ? 8 : 4) / MT);
  constexpr bool ASM = (MT == 1 || sizeof(XT) == 2) && NW <= 8 && U <= 2 * U_BASE;
  auto issue = [&](int i, u32x4* b, XRaw<XT>* a) {
    const bool valid = i < n;
    const size_t ks = (size_t)(w + i * NW);
#pragma unroll
    for (int t = 0; t < NT; ++t)
      asm_load_nt<ASM>(b[t], valid ? (const void*)(wt[t] + ks * 64) : (const void*)zfrag);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) a[mt].template load<ASM>(valid ? xp[mt] + ks * (XP ? 512 : 32) : zx);
  };
  // No separate prologue: the first trip computes on the zero-initialised slots (MFMA adds 0) while
  // issuing k-steps 0..U-1, so every ring register has exactly one definition site (the tied
  // refill) and the compiler never needs to copy an in-flight register across the loop entry.
  for (int i0 = -U; i0 < n; i0 += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (ASM) {
        wait_vmcnt<L * (U - 1)>();  // slot u (the oldest L loads) has landed
#pragma unroll
        for (int t = 0; t < NT; ++t) pin(bq[u][t]);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) aq[u][mt].pin_regs();
      }
      u32x4 af[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) af[mt] = aq[u][mt].frag(ss[mt]);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[mt][t] = mfma16x16x32(af[mt], bq[u][t], acc[mt][t]);
      issue(i0 + U + u, bq[u], aq[u]);  // refill: k-step U ahead (zero fragment past the end)
    }
  }
  if constexpr (ASM) {
    // retire the past-the-end refills, and keep every ring register live until then: a register
    // the compiler thinks is dead could otherwise be reused while its load is still in flight
    wait_vmcnt<0>();
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int t = 0; t < NT; ++t) pin(bq[u][t]);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) aq[u][mt].pin_regs();
    }
  }

  skinny_epilogue<MT, NT, MODE, NW, SPLIT, SC1>(acc, ss, tp_calls, out, M, N, K, eps, use_rms, accumulate, out_f32, qa,
                                               bx, by, gy);
}

template <typename XT, int MT, int NT, int MODE, int NW, int U, bool XP = false, bool SPLIT = false>
__global__ void __launch_bounds__(NW * 64)
    linear_skinny_kernel(const XT* __restrict__ x, const u32x4* __restrict__ W, void* __restrict__ out,
                         int M, int N, int K, float eps, int use_rms, int accumulate, int out_f32, QKVArgs qa) {
  skinny_body<XT, MT, NT, MODE, NW, U, XP, SPLIT>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, blockIdx.x,
                                                  blockIdx.y, gridDim.y);
}

template <typename XT, int MT, int NT, int MODE, int NW, int DEEP = 0, bool XP = false, bool SPLIT = false>
static int launch_skinny(const void* x, const void* W, void* out, int M, int N, int K, float eps, int use_rms,
                         int accumulate, int out_f32, const QKVArgs& qa, hipStream_t s, int ksplit = 1) {
  // k-steps in flight per wave: 8 KiB of weights per wave at MT = 1; fp32 activations double the
  // activation registers, so MT > 1 keeps fewer steps in flight to stay spill-free. DEEP = 1 doubles
  // the ring (bf16 activations at M = 17..64: more bytes in flight per wave).
  constexpr int U0 = (NT == 1) ? 8 : 4;
  constexpr int UD = MT;
  constexpr int U1 = (U0 / UD) < 2 ? 2 : (U0 / UD);
  constexpr int U = DEEP ? 2 * U1 : U1;
  const int NTT = N >> 4;
  const int grid = (NTT + NT - 1) / NT;
  const size_t lds = sizeof(float) * (NW * MT * NT * 256 + NW * MT * 16 + MT * 16 + 4);
  auto kern = &linear_skinny_kernel<XT, MT, NT, MODE, NW, U, XP, SPLIT>;
  if (lds > 65536) {  // opt in to > 64 KiB of dynamic LDS once (not a stream op: capture-safe)
    static bool attr_set = false;
    if (!attr_set) {
      hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr_set = true;
    }
  }
  if (SPLIT && (ksplit < 2 || grid > GEMV_SPLIT_MAX_GROUPS || !qa.sk_ws || !qa.sk_tk ||
                (size_t)qa.sk_ws_floats < (size_t)grid * ksplit * (MT * NT * 256 + MT * 16) ||
                (K >> 5) < ksplit))
    return -3;  // split plan and workspace must fit (host checks the buffers' sizes against these)
  kern<<<dim3(grid, SPLIT ? ksplit : 1), NW * 64, lds, s>>>(static_cast<const XT*>(x), static_cast<const u32x4*>(W),
                                                            out, M, N, K, eps, use_rms, accumulate, out_f32, qa);
  JLA_CHECK_LAUNCH();
  return 0;
}

// waves per workgroup: 4 at M <= 16 (measured best on MI355X for every Llama-3-8B projection at M = 1 and 16), 8
// above. (The 8 / 16-wave forms of the one-m-tile GEMV, variants 2 / 3, were never picked at a bench or latency
// shape -- 8B, 70B MP 1, the TP8 rank proxy -- and were removed in round 4: profiles/r4_variant_pruning.md.)
template <typename XT, int MT, int NT, int MODE>
static int dispatch_nw(const void* x, const void* W, void* out, int M, int N, int K, float eps, int use_rms,
                       int accumulate, int out_f32, const QKVArgs& qa, hipStream_t s) {
  if constexpr (MT == 1)
    return launch_skinny<XT, MT, NT, MODE, 4>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, s);
  return launch_skinny<XT, MT, NT, MODE, 8>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, s);
}

template <typename XT, int MT, int MODE>
static int dispatch_nt(const void* x, const void* W, void* out, int M, int N, int K, float eps, int use_rms,
                       int accumulate, int out_f32, const QKVArgs& qa, int variant, hipStream_t s) {
  // SwiGLU needs the gate/up tile pair in one workgroup; very wide outputs (lm_head, w1|w3) use
  // 2 tiles per workgroup to halve the activation re-reads.
  // variant 5 / 6: 4 waves with 4 / 2 tiles per workgroup (x re-reads / 4, / 2) for tuning; at MT > 1
  // the activation fragments outnumber the weight fragments of a 1-tile workgroup, so these matter more.
  {
    if (variant == 5 && (N & 63) == 0)
      return launch_skinny<XT, MT, 4, MODE, 4>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, s);
    if (variant == 6)
      return launch_skinny<XT, MT, 2, MODE, 4>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, s);
    // variant 10 (bf16 activations, M > 16): 2 tiles per workgroup (as 6) with a doubled ring -- more weight +
    // activation bytes in flight per wave for the latency-bound projections
    if constexpr (MT > 1 && sizeof(XT) == 2) {
      if (variant == 10)
        return launch_skinny<XT, MT, 2, MODE, 4, 1>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, s);
    }
    // split-K variants (bf16 activations): K cut over 2 workgroups per column group (16; 18 on packed x), the last
    // arriver sums the splits and runs the epilogue -- for projections with few column groups (tensor-parallel qkv
    // shards, N = 1280 at Llama-3-70B MP 8: 80 one-tile workgroups leave most CUs idle).
    // 1 tile per workgroup (SwiGLU: the gate/up pair), 4 waves at M <= 16, 8 above.
    if constexpr (sizeof(XT) == 2 && MODE != MODE_ARGMAX) {
      // 26: 4 tiles x 8 waves per workgroup on packed x with K over 4 workgroups -- the 4-tile x re-read ratio of 22/23
      // for the narrow, deep projections at M = 17..64 (w2 at N = 4096: 64 column groups alone leave most CUs idle).
      // The 4-wave forms with 2 / 4 splits never won a shape (profiles/r3_gemv_split4tile_candidates.jsonl).
      if (variant == 26) {
        if (N & 63) return -1;
        return launch_skinny<XT, MT, 4, MODE, 8, 0, true, true>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32,
                                                                qa, s, 4);
      }
      if (gemv_split_variant(variant)) {
        constexpr int SNT = MODE == MODE_SWIGLU ? 2 : 1, SNW = MT == 1 ? 4 : 8;
        const int ks = 2;  // (K over 4 lost to 2 on the 70B MP 8 qkv shard at M = 1 / 32: profiles/README.md round 5)
        if (variant == 18)
          return launch_skinny<XT, MT, SNT, MODE, SNW, 0, true, true>(x, W, out, M, N, K, eps, use_rms, accumulate,
                                                                      out_f32, qa, s, ks);
        return launch_skinny<XT, MT, SNT, MODE, SNW, 0, false, true>(x, W, out, M, N, K, eps, use_rms, accumulate,
                                                                     out_f32, qa, s, ks);
      }
    }
    // 2 tiles x 8 waves (20 row-major, 21 packed x): twice the bytes in flight per workgroup of the 2-tile variants
    // for wide projections with few column groups (w1|w3 at Llama-3-70B MP 8: 224 workgroups of the SwiGLU pairs)
    if (variant == 20)
      return launch_skinny<XT, MT, 2, MODE, 8>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, s);
    if constexpr (sizeof(XT) == 2) {
      if (variant == 21)
        return launch_skinny<XT, MT, 2, MODE, 8, 0, true>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, s);
      // 4 tiles x 4 waves reading packed x (22): half the activation bytes per weight byte of the 2-tile variants,
      // for wide projections at M = 17..64 (w1|w3: 1792 column tiles at Llama-3-8B)
      if (variant == 22) {  // (x is the packed copy: never fall through to a row-major variant)
        if (N & 63) return -1;
        return launch_skinny<XT, MT, 4, MODE, 4, 0, true>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, s);
      }
    }
    // packed-x variants (x is the packed copy, common.h pack_off, padded to MT * 16 rows): 12 = 1 tile x 8 waves,
    // 15 = 2 tiles x 4 waves with a doubled ring (also the SwiGLU form)
    if constexpr (sizeof(XT) == 2) {
      if (variant == 15)
        return launch_skinny<XT, MT, 2, MODE, 4, 1, true>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, s);
      if constexpr (MODE != MODE_SWIGLU) {
        if (variant == 12)
          return launch_skinny<XT, MT, 1, MODE, 8, 0, true>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, s);
      }
    }
  }
  if constexpr (MODE == MODE_SWIGLU) {
    return dispatch_nw<XT, MT, 2, MODE>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, s);
  } else {
    if (MODE != MODE_QKV && (N >> 4) >= 2048)
      return dispatch_nw<XT, MT, 2, MODE>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, s);
    return dispatch_nw<XT, MT, 1, MODE>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, s);
  }
}

template <typename XT, int MODE>
static int dispatch_mt(const void* x, const void* W, void* out, int M, int N, int K, float eps, int use_rms,
                       int accumulate, int out_f32, const QKVArgs& qa, int variant, hipStream_t s) {
  if (M <= 16) return dispatch_nt<XT, 1, MODE>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, variant, s);
  if (M <= 32) return dispatch_nt<XT, 2, MODE>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, variant, s);
  return dispatch_nt<XT, 4, MODE>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, variant, s);
}

// the fused TP epilogue reads the bf16 decode activations only (no fp32-input instantiation)
template <typename XT>
static int dispatch_tp(const void* x, const void* W, void* out, int M, int N, int K, float eps, int use_rms,
                       int accumulate, const QKVArgs& qa, int variant, hipStream_t s) {
  if constexpr (sizeof(XT) == 2) {
    return dispatch_mt<XT, MODE_TPRESID>(x, W, out, M, N, K, eps, use_rms, accumulate, 1, qa, variant, s);
  } else {
    return -1;
  }
}

// ---------------------------------------------------------------------------------------------
// Fused small-batch decode launch: the qkv projection (this GEMV, MODE_QKV: fused norm, RoPE, KV-cache write) on
// workgroups [0, grid_q) and the decode attention (attn_mma.h, the v6 step) on the next pairs x splits workgroups --
// one launch instead of two (reference model.py:210-291 for S = 1). While the qkv workgroups stream their weights, every
// attention wave prefetches its 32-key step of K (registers) and V (LDS) from the cache; one lane per attention
// workgroup then polls the qkv-done counter (every qkv workgroup adds to it once its write-through q / K / V stores
// have drained), the waves load the pair's q and re-load the one cache row this launch wrote (write-through loads),
// score their step, merge through LDS, and the pair's splits merge by last arriver (write-through partials + ticket).
// Optionally (FO > 0) a third kind on the last workgroups runs the o projection into the residual (qa_o_proj), waiting
// on go flags the last attention workgroup sets. Every wait is on lower-numbered workgroups (dispatched first), and the
// host launches this only when every workgroup fits on the CUs at once (grid <= CUs x the occupancy API's count), so
// the waits always end; each is also bounded (the error word records a timeout).
constexpr int QA_SPLIT_KEYS = 128;  // keys per attention workgroup (4 waves x one 32-key step)
constexpr int QA_MAX_SPLITS = 4;    // attention workgroups per (row, kv head) pair: cache length <= 512
constexpr int QA_PART = AD6_DH + 4; // floats per (split, head) partial: O[128], m, l, pad
struct FusedAttn {
  bf16_t* out;              // [B, H * Dh]
  bf16_t* out_pack;         // optional packed copy (the o projection's packed x)
  const int32_t* kv_start;  // [B]
  float* ws;                // [pairs][splits][REP][QA_PART] write-through partials
  int32_t* tickets;         // [pairs] merge tickets (self-resetting)
  int32_t* sync;            // [0] qkv-done counter, [1] attention-seen counter (both self-resetting), [2] error word,
                            // [3] attention-done counter (self-resetting), [QO_GO + QO_GO_STRIDE * ob] the go flag of
                            // o workgroup ob (fused o projection; each cleared by its workgroup)
  int splits, grid_q, t_cap;
  float scale_log2;
  int diag;                 // tools / tests only (qkv_attn_set_diag): 1 = the qkv workgroups never publish
  int grid_a, grid_o;       // attention workgroups (pairs x splits); o-projection workgroups (0: no fused o)
  unsigned long long* stamps;  // tools only (qkv_attn_set_stamps): [grid][8] phase timestamps (wall clock, 100 MHz)
};
// phase timestamp i of this workgroup (tools/qkv_attn_timeline.py); a no-op unless a stamp buffer is set
JLA_DEV void qa_stamp(const FusedAttn& fa, int i) {
  if (fa.stamps && threadIdx.x == 0) fa.stamps[(size_t)blockIdx.x * 8 + i] = wall_clock64();
}
// The fused o projection (FO > 0): the last grid_o workgroups of the launch compute h += attn_out @ Wo^T (FO 16-column
// tiles each, K <= 32 x 4 waves x QO_PF) with the standalone GEMV's residual (or TP-exchange, MODE_TPRESID) epilogue.
struct FusedO {
  const u32x4* W;  // packed Wo [N / 16][K / 32][64 lanes] u32x4
  float* h;        // fp32 residual [M, N]
  int N, K;
};
constexpr int QO_PF = 8;  // k-steps per wave held in registers (o weights fetched while qkv / attention run)
// one go flag per o workgroup, a cache line apart: the workgroups poll their own lines (256 pollers of one counter made
// that line's memory channel a hotspot the whole launch queued behind: the fused o measured 1.1 ms per token slower)
constexpr int QO_GO = 64, QO_GO_STRIDE = 16, QO_MAX_GROUPS = 1024;

// 16-byte store of the attention output: write-through (sc1) when the o projection of the same launch reads it
template <bool SC1>
JLA_DEV void qa_store16(bf16_t* p, u32x4 v) {
  if constexpr (SC1)
    st_sc1_x4(p, v);
  else
    *reinterpret_cast<u32x4*>(p) = v;
}

// The attention workgroups of the fused launch (workgroup a of pairs x splits). SCO: output stores write-through.
template <int REP, bool SCO>
JLA_DEV void qa_attention(const QKVArgs& qa, const FusedAttn& fa, int a) {
  extern __shared__ __attribute__((aligned(16))) char ldsq[];
  const int pair = a / fa.splits, sp = a - pair * fa.splits;
  const int b = pair / qa.Hkv, kvh = pair - b * qa.Hkv;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int T = qa.T;
  const int slot = qa.slot[0];
  const int lo = fa.kv_start[b], hi = min(slot + 1, fa.t_cap);
  const int k0 = sp * QA_SPLIT_KEYS + AD6_STEP * w;
  const bool wave_live = k0 < hi && k0 + AD6_STEP > lo;
  const size_t head_off = ((size_t)b * qa.Hkv + kvh) * (size_t)T * AD6_DH;
  const bf16_t* const kb = qa.kc + head_off;
  const bf16_t* const vb = qa.vc + head_off;
  char* const vslot = ldsq + w * AD6_SLOT_BYTES;

  // 1. prefetch this wave's step (rows clamped into the cache; the row at `slot` is re-loaded after the wait)
  u32x4 kr[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) kr[i] = u32x4{0u, 0u, 0u, 0u};
  ad6_issue<false>(k0, kr, vslot, kb, vb, T, lane);

  // 2. wait until every qkv workgroup has published (one polling lane, bounded). A timeout is sticky: the error word
  //    stays set (the host raises at its next poll: ops.check_inlaunch), the counters are never reset again (a late
  //    publish would leave them off by its count), and every later launch's attention workgroups skip the wait and
  //    write zeros -- no token is ever computed from a stale q / K / V without the error word saying so.
  int* flag = reinterpret_cast<int*>(ldsq + 4 * AD6_SLOT_BYTES + 1008);
  if (threadIdx.x == 0) {
    int err = __hip_atomic_load(fa.sync + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const long long t0 = (long long)wall_clock64();
    while (!err && __hip_atomic_load(fa.sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < fa.grid_q) {
      if ((long long)wall_clock64() - t0 > 20000000LL) {  // 0.2 s at the 100 MHz constant clock
        __hip_atomic_store(fa.sync + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        err = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    // the last attention workgroup past the wait resets both counters for the next launch -- unless some workgroup
    // of this launch (or an earlier one) timed out: the acq_rel add orders a timed-out workgroup's error store before
    // its arrival, and the last arriver's error load after every arrival
    const int seen = __hip_atomic_fetch_add(fa.sync + 1, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (seen == fa.grid_a - 1 &&
        __hip_atomic_load(fa.sync + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
      __hip_atomic_store(fa.sync, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(fa.sync + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *flag = err;
  }
  __syncthreads();
  qa_stamp(fa, 1);
  // the prefetch landed during the qkv phase: retire it here, before any branch (hipcc must never copy a ring
  // register that is still in flight)
  ::wait_vmcnt<0>();
#pragma unroll
  for (int i = 0; i < 8; ++i) pin(kr[i]);
  if (*flag) {  // failed state (timeout now or earlier): the pair's output is zeros (the host raises at its next poll)
    if (sp == 0 && threadIdx.x < REP * 16) {
      const int col = (kvh * REP + (threadIdx.x >> 4)) * AD6_DH + 8 * (threadIdx.x & 15);
      qa_store16<SCO>(fa.out + (size_t)b * qa.H * AD6_DH + col, u32x4{0u, 0u, 0u, 0u});
      if (fa.out_pack) qa_store16<SCO>(fa.out_pack + pack_off(b, col, qa.H * AD6_DH), u32x4{0u, 0u, 0u, 0u});
    }
    return;
  }
  const int split_lo = sp * QA_SPLIT_KEYS;
  const bool split_live = split_lo < hi && split_lo + QA_SPLIT_KEYS > lo;
  if (!split_live) {
    if (sp == 0 && lo >= hi && threadIdx.x < REP * 16) {  // a row with no valid key: zeros (as the other kernels)
      const int col = (kvh * REP + (threadIdx.x >> 4)) * AD6_DH + 8 * (threadIdx.x & 15);
      qa_store16<SCO>(fa.out + (size_t)b * qa.H * AD6_DH + col, u32x4{0u, 0u, 0u, 0u});
      if (fa.out_pack) qa_store16<SCO>(fa.out_pack + pack_off(b, col, qa.H * AD6_DH), u32x4{0u, 0u, 0u, 0u});
    }
    return;
  }

  // 3. the pair's q (written by this launch: write-through loads) and the cache row at `slot` (K lanes holding that
  //    key / V DMA lanes of that row re-load it agent-coherently), all issued before one wait: one round trip, not
  //    three (tools/check_asm_ring.py verifies no in-flight register is copied across the conditional re-loads)
  u32x4 qf[4];
  {
    const int key0 = k0;
    const int c = lane >> 4, j = lane & 15;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      if (key0 + 16 * kk + j == slot) {
        const bf16_t* p = kb + (size_t)slot * AD6_DH + 8 * c;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) asm_load_sc1(kr[4 * kk + jj], p + 32 * jj);
      }
    }
    const int vrow = slot - key0;  // 0 .. 31 when the new row is in this wave's step
    if (vrow >= 0 && vrow < AD6_STEP) {
      // only the lanes of the DMA block holding that row: block vrow / 4, lanes 16 (vrow % 4) .. +15
      const int bi = vrow >> 2;
      if ((lane >> 4) == (vrow & 3)) {
        const int ch = (lane & 15) ^ (((vrow & 3) << 2) | ((vrow >> 2) & 3));
        glds16_asm_sc1(vb + (size_t)slot * AD6_DH + 8 * ch, vslot + 1024 * bi);
      }
    }
  }
  ad6_load_q<REP, true>(qf, qa.q + ((size_t)b * qa.H + kvh * REP) * AD6_DH, lane);
  ::wait_vmcnt<0>();
#pragma unroll
  for (int i = 0; i < 8; ++i) pin(kr[i]);
  ad6_q_ready<REP>(qf, lane);

  // 4. this wave's step, then its (m, l, O)
  Ad6Acc st;
  ad6_init(st);
  ad6_compute<REP>(st, kr, qf, vslot, k0, wave_live, lo, hi, nullptr, 0, fa.scale_log2, lane);
  ad6_finish(st);

  // 5. the 4 waves through LDS (the V slots are free once every wave is past its step)
  __syncthreads();
  qa_stamp(fa, 2);
  float* sm_o = reinterpret_cast<float*>(ldsq);  // [4][REP][128]
  float* sm_ml = sm_o + 4 * REP * AD6_DH;        // [4][REP][2]
  {
    const int c = lane >> 4, j = lane & 15;
    if (j < REP) {
#pragma unroll
      for (int dt = 0; dt < 8; ++dt)
        *reinterpret_cast<f32x4*>(sm_o + (w * REP + j) * AD6_DH + 16 * dt + 4 * c) = st.o[dt];
      if (c == 0) {
        sm_ml[(w * REP + j) * 2] = st.m;
        sm_ml[(w * REP + j) * 2 + 1] = st.l;
      }
    }
  }
  __syncthreads();
  // this workgroup's (m, l, unnormalised O) per head: thread (h, 8 dims) for REP x 16 chunks
  const int nlive = min((hi - 1) / QA_SPLIT_KEYS, fa.splits - 1) - max(lo, 0) / QA_SPLIT_KEYS + 1;
  const int first = max(lo, 0) / QA_SPLIT_KEYS;
  const int t = threadIdx.x;
  const bool chunk = t < REP * 16;
  const int h = t >> 4, d0 = 8 * (t & 15);
  float Mw = -INFINITY, L = 0.f, num[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (chunk) {
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) Mw = fmaxf(Mw, sm_ml[(ww * REP + h) * 2]);
    if (Mw != -INFINITY) {
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) {
        const float mw = sm_ml[(ww * REP + h) * 2];
        const float f = mw == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mw - Mw);
        L += f * sm_ml[(ww * REP + h) * 2 + 1];
        const float* src = sm_o + (ww * REP + h) * AD6_DH + d0;
#pragma unroll
        for (int e = 0; e < 8; ++e) num[e] += f * src[e];
      }
    }
  }
  auto write_out = [&](const float* o8, float den) {
    const float inv = den > 0.f ? 1.f / den : 0.f;
    float r[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] = o8[e] * inv;
    const u32x4 v = pack8(r);
    const int col = (kvh * REP + h) * AD6_DH + d0;
    qa_store16<SCO>(fa.out + (size_t)b * qa.H * AD6_DH + col, v);
    if (fa.out_pack) qa_store16<SCO>(fa.out_pack + pack_off(b, col, qa.H * AD6_DH), v);
  };
  if (nlive <= 1) {  // the pair's only live split: no merge
    if (chunk) write_out(num, L);
    return;
  }
  // 6. the pair's splits: write-through partial, ticket, the last arriver merges in split order
  float* part = fa.ws + ((size_t)pair * fa.splits) * REP * QA_PART;
  if (chunk) {
    float* mine = part + ((size_t)sp * REP + h) * QA_PART;
    st_sc1_x4(mine + d0, u32x4{__float_as_uint(num[0]), __float_as_uint(num[1]), __float_as_uint(num[2]),
                               __float_as_uint(num[3])});
    st_sc1_x4(mine + d0 + 4, u32x4{__float_as_uint(num[4]), __float_as_uint(num[5]), __float_as_uint(num[6]),
                                   __float_as_uint(num[7])});
    if (d0 == 0) st_sc1_x4(mine + AD6_DH, u32x4{__float_as_uint(Mw), __float_as_uint(L), 0u, 0u});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(fa.tickets + pair, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == nlive - 1;
    if (last) __hip_atomic_store(fa.tickets + pair, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  if (!*flag || !chunk) return;
  u32x4 po[QA_MAX_SPLITS][2], pml[QA_MAX_SPLITS];
#pragma unroll
  for (int s2 = 0; s2 < QA_MAX_SPLITS; ++s2) {  // (all issued, then one wait; splits past the live ones re-read the last)
    const float* src = part + ((size_t)(first + min(s2, nlive - 1)) * REP + h) * QA_PART;
    po[s2][0] = po[s2][1] = pml[s2] = u32x4{0u, 0u, 0u, 0u};
    asm_load_sc1(po[s2][0], src + d0);
    asm_load_sc1(po[s2][1], src + d0 + 4);
    asm_load_sc1(pml[s2], src + AD6_DH);
  }
  ::wait_vmcnt<0>();
  float Mx = -INFINITY;
#pragma unroll
  for (int s2 = 0; s2 < QA_MAX_SPLITS; ++s2) {
    pin(po[s2][0]);
    pin(po[s2][1]);
    pin(pml[s2]);
    if (s2 < nlive) Mx = fmaxf(Mx, __uint_as_float(pml[s2][0]));
  }
  float o8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, den = 0.f;
  if (Mx != -INFINITY) {
#pragma unroll
    for (int s2 = 0; s2 < QA_MAX_SPLITS; ++s2) {
      if (s2 >= nlive) break;
      const float ms = __uint_as_float(pml[s2][0]);
      const float f = ms == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(ms - Mx);
      den += f * __uint_as_float(pml[s2][1]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o8[e] += f * __uint_as_float(po[s2][0][e]);
        o8[4 + e] += f * __uint_as_float(po[s2][1][e]);
      }
    }
  }
  write_out(o8, den);
}

// The o-projection workgroups of the fused launch (workgroup ob of grid_o; NTO 16-column tiles, MODE_RESIDUAL or
// MODE_TPRESID): each wave issues its QO_PF k-steps of weights (k-steps w, w + 4, ...) at once, so the weight stream
// lands while the qkv and attention workgroups run; one lane polls the attention-done counter (bounded, as the
// attention side's wait); the waves load the attention output agent-coherently (this launch wrote it write-through),
// multiply, and run the standalone GEMV's epilogue (skinny_epilogue: LDS reduction, residual + mirrors, or the TP
// granule exchange with the peers' workgroup ob).
template <int NTO, int OMODE>
JLA_DEV void qa_o_proj(const FusedAttn& fa, const FusedO& fo, const QKVArgs& qo, int M, int ob) {
  extern __shared__ __attribute__((aligned(16))) char ldsq[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int KS = fo.K >> 5, NTT = fo.N >> 4, nt0 = ob * NTO;
  int tp_calls = 0;
  if constexpr (OMODE == MODE_TPRESID) {
    if (threadIdx.x == 0)
      tp_calls = __hip_atomic_load(static_cast<const CarDevice*>(qo.tp)->wg_ctr + ob, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
  }
  const u32x4* zfrag = g_zero_frag + lane;
  u32x4 bw[QO_PF][NTO];
#pragma unroll
  for (int i = 0; i < QO_PF; ++i) {
    const int ks = w + 4 * i;
#pragma unroll
    for (int t = 0; t < NTO; ++t) {
      bw[i][t] = u32x4{0u, 0u, 0u, 0u};
      asm_load_nt<true>(bw[i][t], ks < KS ? (const void*)(fo.W + ((size_t)min(nt0 + t, NTT - 1) * KS + ks) * 64 + lane)
                                          : (const void*)zfrag);
    }
  }
  int* flag = reinterpret_cast<int*>(ldsq + 4 * AD6_SLOT_BYTES + 1008);
  if (threadIdx.x == 0) {
    // this workgroup's go flag (set by the last attention workgroup to finish), bounded; cleared for the next launch.
    // A timeout (or an attention-side one: the error word) is sticky: h is not updated now or in any later launch.
    int* go = fa.sync + QO_GO + QO_GO_STRIDE * ob;
    int err = 0;
    const long long t0 = (long long)wall_clock64();
    while (__hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
      if ((long long)wall_clock64() - t0 > 20000000LL) {  // 0.2 s
        __hip_atomic_store(fa.sync + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        err = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (!err) __hip_atomic_store(go, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = err || __hip_atomic_load(fa.sync + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  }
  __syncthreads();
  qa_stamp(fa, 1);
  ::wait_vmcnt<0>();  // the weights (retired before any branch: no in-flight register is ever copied)
#pragma unroll
  for (int i = 0; i < QO_PF; ++i)
#pragma unroll
    for (int t = 0; t < NTO; ++t) pin(bw[i][t]);
  if (*flag) return;  // failed state: h is not updated (the host raises at its next poll)
  // the attention output, row-major [M, K]: padding rows re-read the last row (not stored)
  const bf16_t* xr = fa.out + (size_t)min(lane & 15, M - 1) * fo.K + 8 * (lane >> 4);
  u32x4 xa[QO_PF];
#pragma unroll
  for (int i = 0; i < QO_PF; ++i) {
    const int ks = w + 4 * i;
    xa[i] = u32x4{0u, 0u, 0u, 0u};
    asm_load_sc1(xa[i], ks < KS ? (const void*)(xr + (size_t)ks * 32) : (const void*)zfrag);
  }
  ::wait_vmcnt<0>();
  f32x4 acc[1][NTO];
#pragma unroll
  for (int t = 0; t < NTO; ++t) acc[0][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < QO_PF; ++i) {
    pin(xa[i]);
#pragma unroll
    for (int t = 0; t < NTO; ++t) acc[0][t] = mfma16x16x32(xa[i], bw[i][t], acc[0][t]);
  }
  const float ss[1] = {0.f};
  qa_stamp(fa, 2);
  skinny_epilogue<1, NTO, OMODE, 4, false, false>(acc, ss, tp_calls, fo.h, M, fo.N, fo.K, 0.f, 0, 1, 1, qo, ob, 0, 1);
}

// SPL: K of the qkv GEMV cut over SPL workgroups per column group (the split GEMV's last-arriver sum; only that
// workgroup writes q / the cache rows, but every qkv workgroup counts itself in the publish below).
// FO > 0: the launch also runs the o projection (qa_o_proj, FO tiles per workgroup, epilogue OMODE) on its last
// fa.grid_o workgroups; the attention workgroups then store their output write-through and count themselves done.
template <int MT, int NT, int NW, int U, bool XP, int REP, int SPL, int FO, int OMODE>
__global__ void __launch_bounds__(256)
    qkv_attn_kernel(const bf16_t* __restrict__ x, const u32x4* __restrict__ W, int M, int N, int K, float eps,
                    int use_rms, QKVArgs qa, FusedAttn fa, FusedO fo, QKVArgs qo) {
  static_assert(NW == 4, "4-wave workgroups (the attention side uses 4 waves x 32 keys)");
  qa_stamp(fa, 0);
  if ((int)blockIdx.x < fa.grid_q) {
    skinny_body<bf16_t, MT, NT, MODE_QKV, NW, U, XP, (SPL > 1), true>(x, W, nullptr, M, N, K, eps, use_rms, 0, 0, qa,
                                                                      (int)blockIdx.x / SPL, (int)blockIdx.x % SPL,
                                                                      SPL);
    qa_stamp(fa, 1);
    // publish (Guideline 16, sc1-store + agent-counter form): every storing wave drains its write-through stores,
    // the workgroup's barrier, then one agent-scope add
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && !fa.diag) __hip_atomic_fetch_add(fa.sync, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    qa_stamp(fa, 2);
    return;
  }
  if constexpr (FO > 0) {
    static_assert(MT == 1, "fused o projection: M <= 16");
    const int ob = (int)blockIdx.x - fa.grid_q - fa.grid_a;
    if (ob >= 0) {
      qa_o_proj<FO, OMODE>(fa, fo, qo, M, ob);
      qa_stamp(fa, 3);
      return;
    }
  }
  qa_attention<REP, (FO > 0)>(qa, fa, (int)blockIdx.x - fa.grid_q);
  qa_stamp(fa, 3);
  if constexpr (FO > 0) {
    // done (same publish form): every path out of qa_attention, stores drained, then one add per workgroup; the last
    // one to finish resets the counter and sets every o workgroup's go flag (one store per thread)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    extern __shared__ __attribute__((aligned(16))) char ldsq[];
    int* last = reinterpret_cast<int*>(ldsq + 4 * AD6_SLOT_BYTES + 1012);
    if (threadIdx.x == 0) {
      const int prev = __hip_atomic_fetch_add(fa.sync + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *last = prev == fa.grid_a - 1;
      if (*last) __hip_atomic_store(fa.sync + 3, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (*last)
      for (int i = threadIdx.x; i < fa.grid_o; i += 256)
        __hip_atomic_store(fa.sync + QO_GO + QO_GO_STRIDE * i, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    qa_stamp(fa, 4);
  }
}

size_t qkv_attn_lds(int mt) {
  const size_t attn = 4 * AD6_SLOT_BYTES + 1024;  // V slots, the merge's (m, l) and a flag (the merge reuses the slots)
  const size_t gemv = sizeof(float) * (4 * mt * 1 * 256 + 4 * mt * 16 + mt * 16 + 4);  // NT = 1, NW = 4
  // (the o workgroups' epilogue: NT <= 2 tiles at MT = 1, 8.4 KiB, below both)
  return attn > gemv ? attn : gemv;
}

// workgroups of the fused launch that are resident at once per CU (occupancy API, one below its answer as a margin:
// cdna_hip_programming.md warns it can be one block too high; at least 1)
// (MT m-tiles: the GEMV ring depth U = 8 / MT, as launch_skinny)
template <int MT, int REP, int SPL, int FO = 0, int OMODE = 0>
static int qkv_attn_per_cu() {
  static int cached = 0;
  if (cached == 0) {
    int a = 0, b = 0;
    const size_t lds = qkv_attn_lds(MT);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, qkv_attn_kernel<MT, 1, 4, 8 / MT, false, REP, SPL, FO, OMODE>,
                                                     256, lds) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, qkv_attn_kernel<MT, 1, 4, 8 / MT, true, REP, SPL, FO, OMODE>,
                                                     256, lds) != hipSuccess)
      a = b = 1;
    const int n = a < b ? a : b;
    cached = n > 1 ? n - 1 : 1;
  }
  return cached;
}
template <int MT, int SPL>
static int qkv_attn_per_cu_rep(int rep) {
  switch (rep) {
    case 1: return qkv_attn_per_cu<MT, 1, SPL>();
    case 2: return qkv_attn_per_cu<MT, 2, SPL>();
    case 4: return qkv_attn_per_cu<MT, 4, SPL>();
    case 8: return qkv_attn_per_cu<MT, 8, SPL>();
    case 16: return qkv_attn_per_cu<MT, 16, SPL>();
    default: return 0;
  }
}
// the fused-o instances: one m-tile, 8 query heads per kv head (the Llama-3-70B tensor-parallel shard)
template <int SPL, int FO>
static int qkv_attn_per_cu_o() {
  const int a = qkv_attn_per_cu<1, 8, SPL, FO, MODE_RESIDUAL>(), b = qkv_attn_per_cu<1, 8, SPL, FO, MODE_TPRESID>();
  return a < b ? a : b;
}

static int g_qa_o_nt = 2;  // o tiles per workgroup of the fused o projection (1 or 2; qkv_attn_set_o_nt, for A/B)
void qkv_attn_set_o_nt(int nt) { g_qa_o_nt = nt == 1 ? 1 : 2; }
int qkv_attn_o_groups(int M, int rep, int N, int K) {
  if (M < 1 || M > 16 || rep != 8 || (N & 15) || (K & 31) || K > 32 * 4 * QO_PF) return 0;
  const int g = ((N >> 4) + g_qa_o_nt - 1) / g_qa_o_nt;
  return g <= QO_MAX_GROUPS ? g : 0;
}
size_t qkv_attn_sync_ints() { return QO_GO + (size_t)QO_GO_STRIDE * QO_MAX_GROUPS; }

// 0 when the fused launch does not apply (then the caller runs the qkv GEMV and the attention kernel). Every workgroup
// of the launch must be resident at once (the attention workgroups wait for the qkv ones, the o workgroups for the
// attention ones).
int qkv_attn_occupancy(int M, int rep, int spl, int o_groups) {
  if (o_groups > 0) {
    if (M > 16 || rep != 8) return 0;
    if (g_qa_o_nt == 1) return spl == 2 ? qkv_attn_per_cu_o<2, 1>() : qkv_attn_per_cu_o<1, 1>();
    return spl == 2 ? qkv_attn_per_cu_o<2, 2>() : qkv_attn_per_cu_o<1, 2>();
  }
  if (spl == 2) return M <= 16 ? qkv_attn_per_cu_rep<1, 2>(rep) : qkv_attn_per_cu_rep<2, 2>(rep);
  return M <= 16 ? qkv_attn_per_cu_rep<1, 1>(rep) : qkv_attn_per_cu_rep<2, 1>(rep);
}
int qkv_attn_splits(int M, int B, int Hkv, int rep, int t_cap, int N, int cus, int spl, int o_groups) {
  if (M != B || M > 32 || (rep & (rep - 1)) || rep > 16 || t_cap > QA_MAX_SPLITS * QA_SPLIT_KEYS) return 0;
  // (K over 3 / 4 workgroups measured slower than 2 at the 70B shard's B = 1: profiles/r6_qkv_attn_o_timeline.jsonl)
  if ((spl != 1 && spl != 2) || (spl > 1 && (N >> 4) > GEMV_SPLIT_MAX_GROUPS) || o_groups < 0) return 0;
  const int splits = (t_cap + QA_SPLIT_KEYS - 1) / QA_SPLIT_KEYS;
  const int grid = (N >> 4) * spl + B * Hkv * splits + o_groups;
  return grid <= cus * qkv_attn_occupancy(M, rep, spl, o_groups) ? splits : 0;
}

static int g_qa_diag = 0;
void qkv_attn_set_diag(int d) { g_qa_diag = d; }
static unsigned long long* g_qa_stamps = nullptr;
void qkv_attn_set_stamps(unsigned long long* p) { g_qa_stamps = p; }

int linear_qkv_attn(const bf16_t* x, const void* W, int M, int N, int K, float rms_eps, const QKVArgs& qa, bool xp,
                    bf16_t* out, bf16_t* out_pack, const int32_t* kv_start, float* ws, int32_t* tickets, int32_t* sync,
                    int t_cap, int splits, int spl, hipStream_t s, const void* o_w, float* o_h, int o_n, int o_k,
                    int o_mode, const QKVArgs* qo) {
  if (M <= 0) return 0;
  if (M > 32 || (N & 15) || (K & 31) || qa.Dh != AD6_DH || qa.S != 1 || qa.H % qa.Hkv) return -1;
  const int rep = qa.H / qa.Hkv;
  const int grid_q = (N >> 4) * spl, pairs = M * qa.Hkv;
  if (spl != 1 && spl != 2) return -1;
  if (spl > 1) {  // the split GEMV's slabs and tickets (as launch_skinny checks them)
    const int mt0 = M <= 16 ? 1 : 2;
    if ((N >> 4) > GEMV_SPLIT_MAX_GROUPS || !qa.sk_ws || !qa.sk_tk || (K >> 5) < spl ||
        (size_t)qa.sk_ws_floats < (size_t)(N >> 4) * spl * (mt0 * 256 + mt0 * 16))
      return -3;
  }
  if (splits < 1 || splits > QA_MAX_SPLITS || splits * QA_SPLIT_KEYS < t_cap) return -1;
  // the fused o projection: h += out @ Wo^T (Wo [o_n, o_k], o_k = H * Dh)
  int grid_o = 0;
  if (o_w) {
    grid_o = qkv_attn_o_groups(M, rep, o_n, o_k);
    if (!grid_o || !o_h || !qo || o_k != qa.H * AD6_DH || (o_mode != MODE_RESIDUAL && o_mode != MODE_TPRESID) ||
        (o_mode == MODE_TPRESID && !qo->tp))
      return -1;
  }
  const FusedAttn fa{out,    out_pack, kv_start, ws, tickets, sync, splits, grid_q, t_cap,
                     1.4426950408889634f / sqrtf((float)AD6_DH), g_qa_diag, pairs * splits, grid_o, g_qa_stamps};
  const FusedO fo{static_cast<const u32x4*>(o_w), o_h, o_n, o_k};
  const QKVArgs qo_v = qo ? *qo : QKVArgs{};
  const int use_rms = rms_eps >= 0.f;
  const float eps = use_rms ? rms_eps : 0.f;
  const int mt = M <= 16 ? 1 : 2;
  const size_t lds = qkv_attn_lds(mt);
  const int grid = grid_q + pairs * splits + grid_o;
  const u32x4* Wq = static_cast<const u32x4*>(W);
#define JLA_QA_K(MTV, R, SP, FOV, OM)                                                                             \
  {                                                                                                               \
    if (xp)                                                                                                       \
      qkv_attn_kernel<MTV, 1, 4, 8 / MTV, true, R, SP, FOV, OM><<<grid, 256, lds, s>>>(x, Wq, M, N, K, eps,         \
                                                                                      use_rms, qa, fa, fo, qo_v);  \
    else                                                                                                          \
      qkv_attn_kernel<MTV, 1, 4, 8 / MTV, false, R, SP, FOV, OM><<<grid, 256, lds, s>>>(x, Wq, M, N, K, eps,        \
                                                                                       use_rms, qa, fa, fo, qo_v); \
    JLA_CHECK_LAUNCH();                                                                                           \
    return 0;                                                                                                     \
  }
  if (grid_o > 0) {
#define JLA_QA_O(SP, FOV)                                                                  \
  if (spl == SP && g_qa_o_nt == FOV) {                                                     \
    if (o_mode == MODE_TPRESID) JLA_QA_K(1, 8, SP, FOV, MODE_TPRESID)                      \
    JLA_QA_K(1, 8, SP, FOV, MODE_RESIDUAL)                                                 \
  }
    JLA_QA_O(1, 1) JLA_QA_O(1, 2) JLA_QA_O(2, 1) JLA_QA_O(2, 2)
#undef JLA_QA_O
    return -1;
  }
#define JLA_QA_S(MTV, R, SP) \
  if (mt == MTV && rep == R && spl == SP) JLA_QA_K(MTV, R, SP, 0, 0)
#define JLA_QA(MTV, R) JLA_QA_S(MTV, R, 1) JLA_QA_S(MTV, R, 2)
  JLA_QA(1, 1) JLA_QA(1, 2) JLA_QA(1, 4) JLA_QA(1, 8) JLA_QA(1, 16)
  JLA_QA(2, 1) JLA_QA(2, 2) JLA_QA(2, 4) JLA_QA(2, 8) JLA_QA(2, 16)
#undef JLA_QA
#undef JLA_QA_S
#undef JLA_QA_K
  return -1;
}

size_t gemv_split_workspace_floats(int M, int N) {
  const int groups = N >> 4;  // upper bound: 1 tile per column group
  if (groups > GEMV_SPLIT_MAX_GROUPS || M < 1 || M > SKINNY_MAX_M) return 0;
  const int mt = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  return (size_t)groups * 4 * (mt * 256 + mt * 16);  // (variant 26: 4 tiles per group, K over 4)
}
int gemv_split_tickets(int N) { return (N >> 4) > GEMV_SPLIT_MAX_GROUPS ? 0 : (N >> 4); }

int linear_skinny(const void* x, int x_is_f32, const void* W, void* out, int M, int N, int K, int mode,
                  float rms_eps, int accumulate, int out_f32, const QKVArgs* qkv, int variant, hipStream_t s) {
  if (M <= 0) return 0;
  if (M > SKINNY_MAX_M || (N & 15) || (K & 31)) return -1;
  if (mode == MODE_SWIGLU && (N & 31)) return -1;
  if (mode == MODE_QKV && (!qkv || qkv->Dh % 16 || M % qkv->S)) return -1;
  if (mode == MODE_TPRESID && (!qkv || !qkv->tp)) return -1;
  if (gemv_split_variant(variant) && (x_is_f32 || mode == MODE_ARGMAX)) return -1;
  const int use_rms = rms_eps >= 0.f;
  const float eps = use_rms ? rms_eps : 0.f;
  QKVArgs qa{};
  if (qkv) qa = *qkv;
#define JLA_ARGS x, W, out, M, N, K, eps, use_rms, accumulate
#define JLA_MODE(XT)                                                                                 \
  switch (mode) {                                                                                    \
    case MODE_STORE: return dispatch_mt<XT, MODE_STORE>(JLA_ARGS, out_f32, qa, variant, s);          \
    case MODE_RESIDUAL: return dispatch_mt<XT, MODE_RESIDUAL>(JLA_ARGS, 1, qa, variant, s);          \
    case MODE_SWIGLU: return dispatch_mt<XT, MODE_SWIGLU>(JLA_ARGS, 0, qa, variant, s);              \
    case MODE_QKV: return dispatch_mt<XT, MODE_QKV>(JLA_ARGS, 0, qa, variant, s);                    \
    case MODE_ARGMAX: return dispatch_mt<XT, MODE_ARGMAX>(JLA_ARGS, 0, qa, variant, s);              \
    case MODE_TPRESID: return dispatch_tp<XT>(JLA_ARGS, qa, variant, s);                             \
    default: return -1;                                                                              \
  }
  if (x_is_f32) {
    JLA_MODE(float)
  } else {
    JLA_MODE(bf16_t)
  }
#undef JLA_MODE
#undef JLA_ARGS
}

JLA_BOUNDS_ACCESSOR(gemv)

}  // namespace jla
