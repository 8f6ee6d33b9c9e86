// Batched-decode linear layer (M <= 64 rows), split-K "skinny GEMM":
//   y[M, N] = epilogue( [inv_rms(x) *] x[M, K] @ W[N, K]^T )
//
// Why a second decode kernel (gemv.hip keeps the K-split-across-waves GEMV): with M = 16..64 rows
// the activation fragments cost as many bytes as the weights when every wave reads its own K slice
// of x. Here the waves of a workgroup split N instead and SHARE one LDS copy of x:
//   * workgroup = (column group of 4 waves x NT tiles x 16 columns, K chunk); its x chunk
//     [M, Kc] is staged once into LDS as bf16 MFMA A-fragments (lane-linear 1 KiB blocks ->
//     conflict-free ds_read_b128), RMSNorm's sum of squares accumulated on the way;
//   * each wave streams its NT packed weight tiles over the chunk through a register ring of U
//     k-steps (weights read exactly once, non-temporal); x traffic per weight byte drops to
//     M*2 / (NT*4*32*2) (<= 1/8 at M = 16, NT = 2);
//   * K is split over ksplit workgroups so even small-N projections launch 2-4 workgroups per CU;
//     partial tiles go to a workspace with write-through (sc1) stores, a per-group ticket picks the
//     last arriver, which sums the splits in fixed order (deterministic) and runs the fused
//     epilogue from registers (store / residual add / SwiGLU / RoPE + KV-cache write)
//     -- cdna_hip_programming.md Guideline 16, sc1-store + agent-atomic ticket + sc1-load form.
// Reference ops: model.py:210 (wq/wk/wv), :294 (wo), :338 (w1/w3/w2), :736 (lm_head), RMSNorm
// :28-48, RoPE :58-92, cache write :169-199, residual adds :392/:398.
#include "common.h"
#include "launchers.h"

namespace jla {

constexpr int SK_NW = 4;  // waves per workgroup

JLA_DEV void st_wt(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
JLA_DEV float ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct SplitArgs {
  int ksplit, kc;        // K split count, k-steps (of 32) per split
  float* slabs;          // [groups * ksplit][NW][MT][NT][64][4] + ss [groups * ksplit][MT * 16]
  int32_t* tickets;      // [groups], self-resetting
};

template <typename XT, int MT, int NT, int MODE, int U>
__global__ void __launch_bounds__(SK_NW * 64)
    skinny_kernel(const XT* __restrict__ x, const u32x4* __restrict__ W, void* __restrict__ out, int M, int N, int K,
                  float eps, int use_rms, int accumulate, int out_f32, QKVArgs qa, SplitArgs sa) {
  extern __shared__ __attribute__((aligned(16))) u32x4 xs[];  // [MT][kc][64] A fragments
  __shared__ float ss_l[MT * 16];
  __shared__ float inv_l[MT * 16];
  __shared__ int last_flag;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int KS = K >> 5, NTT = N >> 4;
  const int group = blockIdx.x / sa.ksplit, split = blockIdx.x - group * sa.ksplit;
  const int ks0 = split * sa.kc;
  const int nk = max(0, min(KS, ks0 + sa.kc) - ks0);

  // ---- stage x[:, ks0*32 : (ks0+nk)*32] -> LDS fragments (bf16), sum of squares per row
  if (threadIdx.x < MT * 16) ss_l[threadIdx.x] = 0.f;
  __syncthreads();
  {
    float ssp[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) ssp[mt] = 0.f;
    const int npieces = nk * 64;  // per m-tile
    for (int p = threadIdx.x; p < npieces; p += SK_NW * 64) {
      const int j = p >> 6;  // lane of piece p == lane (p & 63) == threadIdx.x & 63
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int row = min(mt * 16 + (lane & 15), M - 1);
        const size_t off = (size_t)row * K + (size_t)(ks0 + j) * 32 + 8 * (lane >> 4);
        u32x4 v;
        if constexpr (sizeof(XT) == 4) {
          const float4* src = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(x) + off);
          const float4 a = src[0], b = src[1];
          ssp[mt] += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w + b.x * b.x + b.y * b.y + b.z * b.z + b.w * b.w;
          v[0] = pack2bf(a.x, a.y);
          v[1] = pack2bf(a.z, a.w);
          v[2] = pack2bf(b.x, b.y);
          v[3] = pack2bf(b.z, b.w);
        } else {
          v = *reinterpret_cast<const u32x4*>(reinterpret_cast<const bf16_t*>(x) + off);
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int e = 0; e < 8; ++e) ssp[mt] += f[e] * f[e];
        }
        xs[(mt * nk + j) * 64 + lane] = v;
      }
    }
    if (use_rms) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        float s = ssp[mt];
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        if (lane < 16) atomicAdd(&ss_l[mt * 16 + lane], s);
      }
    }
  }
  __syncthreads();

  // ---- stream this wave's NT weight tiles over the chunk
  const int tile0 = (group * SK_NW + w) * NT;
  const u32x4* wt[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) wt[t] = W + ((size_t)min(tile0 + t, NTT - 1) * KS + ks0) * 64 + lane;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[mt][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 bq[U][NT] = {};
  for (int j0 = -U; j0 < nk; j0 += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = j0 + u;
      if (j >= 0 && j < nk) {
        u32x4 af[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) af[mt] = xs[(mt * nk + j) * 64 + lane];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[mt][t] = mfma16x16x32(af[mt], bq[u][t], acc[mt][t]);
      }
      const int jn = j + U;
      const bool valid = jn < nk;
#pragma unroll
      for (int t = 0; t < NT; ++t)
        bq[u][t] = __builtin_nontemporal_load(valid ? wt[t] + (size_t)jn * 64 : wt[t]);
    }
  }

  // ---- split-K: publish partials, last arriver reduces (fixed split order)
  if (sa.ksplit > 1) {
    const size_t slab_sz = (size_t)SK_NW * MT * NT * 256;
    float* slab = sa.slabs + (size_t)blockIdx.x * slab_sz + (size_t)w * MT * NT * 256;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) st_wt(slab + ((mt * NT + t) * 64 + lane) * 4 + i, acc[mt][t][i]);
    float* ss_slab = sa.slabs + (size_t)gridDim.x * slab_sz + (size_t)blockIdx.x * MT * 16;
    if (threadIdx.x < MT * 16) st_wt(ss_slab + threadIdx.x, ss_l[threadIdx.x]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const int prev = __hip_atomic_fetch_add(sa.tickets + group, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == sa.ksplit - 1;
      if (last) __hip_atomic_store(sa.tickets + group, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_flag = last;
    }
    __syncthreads();
    if (!last_flag) return;
    const int b0 = group * sa.ksplit;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[mt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < sa.ksplit; ++s) {
      const float* sl = sa.slabs + (size_t)(b0 + s) * slab_sz + (size_t)w * MT * NT * 256;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[mt][t][i] += ld_wt(sl + ((mt * NT + t) * 64 + lane) * 4 + i);
    }
    if (threadIdx.x < MT * 16) {
      float s = 0.f;
      for (int sp = 0; sp < sa.ksplit; ++sp) s += ld_wt(sa.slabs + (size_t)gridDim.x * slab_sz + (size_t)(b0 + sp) * MT * 16 + threadIdx.x);
      ss_l[threadIdx.x] = s;
    }
  }
  if (threadIdx.x < MT * 16) inv_l[threadIdx.x] = use_rms ? rsqrtf(ss_l[threadIdx.x] / (float)K + eps) : 1.f;
  __syncthreads();

  // ---- fused epilogue from the accumulator layout: lane holds rows 4*(lane>>4)+i, column lane&15
  const int c = lane & 15;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = mt * 16 + 4 * (lane >> 4) + i;
      const float sc = inv_l[min(m, MT * 16 - 1)];
      if constexpr (MODE == MODE_SWIGLU) {
#pragma unroll
        for (int t = 0; t < NT; t += 2) {
          const int gtile = tile0 + t;  // even: gate tile; gtile + 1: up tile
          if (m < M && gtile < NTT) {
            const float g = acc[mt][t][i] * sc, u = acc[mt][t + 1][i] * sc;
            static_cast<bf16_t*>(out)[(size_t)m * (N >> 1) + (gtile >> 1) * 16 + c] = f2bf(silu(g) * u);
          }
        }
      } else {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int tile = tile0 + t;
          const float v = acc[mt][t][i] * sc;
          if constexpr (MODE == MODE_QKV) {
            const float pv = __shfl_xor(v, 1, 64);  // RoPE partner column (d ^ 1) lives in lane ^ 1
            if (m < M && tile < NTT) {
              const int col = tile * 16 + c;
              const int head = col / qa.Dh, d = col - head * qa.Dh;
              const int b = m / qa.S, s = m - b * qa.S;
              float r = v;
              if (head < qa.H + qa.Hkv) {
                int pos = qa.positions[m];
                pos = pos < 0 ? 0 : (pos >= qa.table_len ? qa.table_len - 1 : pos);
                const float2 cs = qa.table[(size_t)pos * (qa.Dh >> 1) + (d >> 1)];
                r = (d & 1) ? (pv * cs.y + v * cs.x) : (v * cs.x - pv * cs.y);
              }
              if (head < qa.H) {
                qa.q[((size_t)m * qa.H + head) * qa.Dh + d] = f2bf(r);
              } else {
                const int slot = qa.slot[0] + s;
                if (slot < qa.T) {
                  const bool is_k = head < qa.H + qa.Hkv;
                  const int kh = is_k ? head - qa.H : head - qa.H - qa.Hkv;
                  bf16_t* cache = is_k ? qa.kc : qa.vc;
                  cache[(((size_t)b * qa.Hkv + kh) * qa.T + slot) * qa.Dh + d] = f2bf(r);
                }
              }
            }
          } else if (m < M && tile < NTT) {
            const size_t idx = (size_t)m * N + tile * 16 + c;
            if constexpr (MODE == MODE_RESIDUAL) {
              float* o = static_cast<float*>(out);
              o[idx] = accumulate ? o[idx] + v : v;
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
}

// ----------------------------------------------------------------------------------------------
// host side: shape -> (NT, ksplit) and workspace sizing
struct SkPlan {
  int nt, groups, ksplit, kc;
};

static SkPlan sk_plan(int M, int N, int K, int mode) {
  const int KS = K >> 5, NTT = N >> 4;
  const int mt = (M + 15) / 16;
  SkPlan p;
  p.nt = (mode == MODE_SWIGLU || NTT >= 8 * SK_NW) ? 2 : 1;
  p.groups = (NTT + SK_NW * p.nt - 1) / (SK_NW * p.nt);
  // LDS: MT * kc fragments of 1 KiB <= 64 KiB; target ~512 workgroups; >= 4 k-steps per split
  const int kc_max = max(1, 64 / mt);
  int ks = (512 + p.groups - 1) / p.groups;
  ks = max(ks, (KS + kc_max - 1) / kc_max);
  ks = min(ks, max(1, KS / 4));
  ks = max(ks, (KS + kc_max - 1) / kc_max);
  p.kc = (KS + ks - 1) / ks;
  p.ksplit = (KS + p.kc - 1) / p.kc;
  return p;
}

size_t skinny_workspace_floats(int M, int N, int K, int mode) {
  const SkPlan p = sk_plan(M, N, K, mode);
  if (p.ksplit <= 1) return 0;
  const int mt = (M + 15) / 16;
  const size_t wgs = (size_t)p.groups * p.ksplit;
  return wgs * ((size_t)SK_NW * mt * p.nt * 256 + mt * 16);
}

int skinny_tickets(int M, int N, int K, int mode) { return sk_plan(M, N, K, mode).groups; }

template <typename XT, int MT, int NT, int MODE>
static int launch_sk(const void* x, const void* W, void* out, int M, int N, int K, float eps, int use_rms,
                     int accumulate, int out_f32, const QKVArgs& qa, const SkPlan& p, float* ws, int32_t* tickets,
                     hipStream_t s) {
  constexpr int U = NT == 1 ? 8 : 4;
  SplitArgs sa{p.ksplit, p.kc, ws, tickets};
  const size_t lds = (size_t)MT * p.kc * 1024;
  auto kern = &skinny_kernel<XT, MT, NT, MODE, U>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    attr_set = true;
  }
  kern<<<p.groups * p.ksplit, SK_NW * 64, lds, s>>>(static_cast<const XT*>(x), static_cast<const u32x4*>(W), out, M,
                                                     N, K, eps, use_rms, accumulate, out_f32, qa, sa);
  JLA_CHECK_LAUNCH();
  return 0;
}

template <typename XT, int MT, int MODE>
static int sk_nt(const void* x, const void* W, void* out, int M, int N, int K, float eps, int use_rms, int accumulate,
                 int out_f32, const QKVArgs& qa, const SkPlan& p, float* ws, int32_t* tickets, hipStream_t s) {
  if constexpr (MODE != MODE_SWIGLU) {
    if (p.nt == 1)
      return launch_sk<XT, MT, 1, MODE>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, p, ws, tickets, s);
  }
  return launch_sk<XT, MT, 2, MODE>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, p, ws, tickets, s);
}

template <typename XT, int MODE>
static int sk_mt(const void* x, const void* W, void* out, int M, int N, int K, float eps, int use_rms, int accumulate,
                 int out_f32, const QKVArgs& qa, const SkPlan& p, float* ws, int32_t* tickets, hipStream_t s) {
  if (M <= 16) return sk_nt<XT, 1, MODE>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, p, ws, tickets, s);
  if (M <= 32) return sk_nt<XT, 2, MODE>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, p, ws, tickets, s);
  return sk_nt<XT, 4, MODE>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, qa, p, ws, tickets, s);
}

int linear_splitk(const void* x, int x_is_f32, const void* W, void* out, int M, int N, int K, int mode, float rms_eps,
                  int accumulate, int out_f32, const QKVArgs* qkv, float* ws, size_t ws_floats, int32_t* tickets,
                  int n_tickets, hipStream_t s) {
  if (M <= 0) return 0;
  if (M > SKINNY_MAX_M || (N & 15) || (K & 31)) return -1;
  if (mode == MODE_SWIGLU && (N & 31)) return -1;
  if (mode == MODE_QKV && (!qkv || qkv->Dh % 16 || M % qkv->S)) return -1;
  const SkPlan p = sk_plan(M, N, K, mode);
  if (p.ksplit > 1 && (ws_floats < skinny_workspace_floats(M, N, K, mode) || n_tickets < p.groups)) return -3;
  const int use_rms = rms_eps >= 0.f;
  const float eps = use_rms ? rms_eps : 0.f;
  QKVArgs qa{};
  if (qkv) qa = *qkv;
#define JLA_ARGS x, W, out, M, N, K, eps, use_rms, accumulate
#define JLA_MODE(XT)                                                                                      \
  switch (mode) {                                                                                         \
    case MODE_STORE: return sk_mt<XT, MODE_STORE>(JLA_ARGS, out_f32, qa, p, ws, tickets, s);              \
    case MODE_RESIDUAL: return sk_mt<XT, MODE_RESIDUAL>(JLA_ARGS, 1, qa, p, ws, tickets, s);              \
    case MODE_SWIGLU: return sk_mt<XT, MODE_SWIGLU>(JLA_ARGS, 0, qa, p, ws, tickets, s);                  \
    case MODE_QKV: return sk_mt<XT, MODE_QKV>(JLA_ARGS, 0, qa, p, ws, tickets, s);                        \
    default: return -1;                                                                                   \
  }
  if (x_is_f32) {
    JLA_MODE(float)
  } else {
    JLA_MODE(bf16_t)
  }
#undef JLA_MODE
#undef JLA_ARGS
}

}  // namespace jla
