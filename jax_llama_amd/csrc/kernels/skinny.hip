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

constexpr int SK_NW = 8;  // waves per workgroup

// Hand-counted register ring for the weight stream (same scheme as gemv.hip: tied asm loads, one
// definition site, counted vmcnt; tools/check_asm_ring.py verifies the assembly at build time).
JLA_DEV void sk_load_nt(u32x4& r, const void* p) {
  asm volatile("global_load_dwordx4 %0, %1, off nt" : "+v"(r) : "v"(p) : "memory");
}
template <int N>
JLA_DEV void sk_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
JLA_DEV void sk_pin(u32x4& r) { asm volatile("" : "+v"(r)); }

__device__ u32x4 g_sk_zero[64];  // zero fragment for past-the-end refills (MFMA adds 0)

struct SplitArgs {
  int ksplit, kc;        // K split count, k-steps (of 32) per split
  float* slabs;          // [wgs][NW][MT][NT][64][4] partial tiles, then [wgs][MT * 16] sums of squares
  int slab_bytes;        // total bytes of the workspace (buffer descriptor range)
  int32_t* tickets;      // [groups], zero-initialised once, reset by each group's last arriver
};

template <typename XT, int MT, int NT, int MODE, int U>
__global__ void __launch_bounds__(SK_NW * 64)
    skinny_kernel(const XT* __restrict__ x, const u32x4* __restrict__ W, void* __restrict__ out, int M, int N, int K,
                  float eps, int use_rms, int accumulate, int out_f32, QKVArgs qa, SplitArgs sa) {
  extern __shared__ __attribute__((aligned(16))) u32x4 xs[];  // [MT][kc][64] bf16 A fragments
  __shared__ float ss_w[SK_NW][MT * 16];
  __shared__ float ss_l[MT * 16];
  __shared__ float inv_l[MT * 16];
  __shared__ int last_flag;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int KS = K >> 5, NTT = N >> 4;
  const int group = blockIdx.x / sa.ksplit, split = blockIdx.x - group * sa.ksplit;
  const int ks0 = split * sa.kc;
  const int nk = max(1, min(KS, ks0 + sa.kc) - ks0);
  const int tile0 = (group * SK_NW + w) * NT;

  const u32x4* wt[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) wt[t] = W + ((size_t)min(tile0 + t, NTT - 1) * KS + ks0) * 64 + lane;
  const u32x4* zf = g_sk_zero + lane;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[mt][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- stage x[:, ks0*32 : (ks0+nk)*32] -> LDS as bf16 A fragments; RMS sums of squares.
  // Done BEFORE the weight ring is issued: the compiler's waits for these (ordinary) loads count only
  // the loads it can see, so staging behind the hand-counted ring drained the ring once per staging
  // round (s_waitcnt vmcnt(0) in the staging loop: ~4 serial HBM round trips per workgroup). Here the
  // activation loads (L2-resident) are all issued up front, the waits cover only them, and the weight
  // stream starts right after.
  {
    float ssp[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) ssp[mt] = 0.f;
    const int nq = MT * nk * 64;  // (mt, j, lane) fragment pieces of 16 B
    auto piece = [&](int q, int& mt, int& j) {
      mt = q / (nk * 64);
      j = (q - mt * nk * 64) >> 6;
    };
    if constexpr (sizeof(XT) == 2) {
      constexpr int XL = 8;  // nk * MT <= 64 (LDS plan) -> at most 8 pieces per thread
      u32x4 xv[XL];
#pragma unroll
      for (int i = 0; i < XL; ++i) {
        const int q = threadIdx.x + SK_NW * 64 * i;
        int mt, j;
        piece(min(q, nq - 1), mt, j);
        const int row = min(mt * 16 + (lane & 15), M - 1);
        xv[i] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const bf16_t*>(x) + (size_t)row * K +
                                                (size_t)(ks0 + j) * 32 + 8 * (lane >> 4));
      }
#pragma unroll
      for (int i = 0; i < XL; ++i) {
        const int q = threadIdx.x + SK_NW * 64 * i;
        if (q < nq) {
          int mt, j;
          piece(q, mt, j);
          const float sq = dot8_bf16(xv[i], xv[i], 0.f);  // whole-vector cast (see common.h)
#pragma unroll
          for (int m2 = 0; m2 < MT; ++m2)
            if (m2 == mt) ssp[m2] += sq;
          xs[(mt * nk + j) * 64 + lane] = xv[i];
        }
      }
    } else {
      for (int q = threadIdx.x; q < nq; q += SK_NW * 64) {
        int mt, j;
        piece(q, mt, j);
        const int row = min(mt * 16 + (lane & 15), M - 1);
        const size_t off = (size_t)row * K + (size_t)(ks0 + j) * 32 + 8 * (lane >> 4);
        const float4* src = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(x) + off);
        const float4 a = src[0], b = src[1];
        const float sq =
            a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w + b.x * b.x + b.y * b.y + b.z * b.z + b.w * b.w;
#pragma unroll
        for (int m2 = 0; m2 < MT; ++m2)
          if (m2 == mt) ssp[m2] += sq;
        u32x4 v;
        v[0] = pack2bf(a.x, a.y);
        v[1] = pack2bf(a.z, a.w);
        v[2] = pack2bf(b.x, b.y);
        v[3] = pack2bf(b.z, b.w);
        xs[(mt * nk + j) * 64 + lane] = v;
      }
    }
    // per-wave partials, summed in wave order below (deterministic: no LDS float atomics)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      float sv = ssp[mt];
      sv += __shfl_xor(sv, 16, 64);
      sv += __shfl_xor(sv, 32, 64);
      if (lane < 16) ss_w[w][mt * 16 + lane] = sv;
    }
    __syncthreads();
    if (threadIdx.x < MT * 16) {
      float sv = 0.f;
#pragma unroll
      for (int ww = 0; ww < SK_NW; ++ww) sv += ss_w[ww][threadIdx.x];
      ss_l[threadIdx.x] = sv;
    }
  }

  u32x4 bq[U][NT] = {};
  // Trip j0 = -U only issues k-steps 0..U-1 (the ring's single definition site); every later trip
  // consumes slot u and refills it.
  for (int j0 = -U; j0 < nk; j0 += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (j0 >= 0) {
        sk_wait<NT * (U - 1)>();
#pragma unroll
        for (int t = 0; t < NT; ++t) sk_pin(bq[u][t]);
        const int j = min(j0 + u, nk - 1);  // past the end: zero weights, any valid x
        u32x4 af[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) af[mt] = xs[(mt * nk + j) * 64 + lane];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[mt][t] = mfma16x16x32(af[mt], bq[u][t], acc[mt][t]);
      }
      const int jn = j0 + u + U;
#pragma unroll
      for (int t = 0; t < NT; ++t) sk_load_nt(bq[u][t], jn < nk ? (const void*)(wt[t] + (size_t)jn * 64) : (const void*)zf);
    }
  }
  sk_wait<0>();  // retire the zero-fragment refills; ring registers stay live until here
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int t = 0; t < NT; ++t) sk_pin(bq[u][t]);

  // ---- split-K: publish partial tile (write-through sc1 stores), last arriver reduces in order
  if (sa.ksplit > 1) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(sa.slabs, 0, sa.slab_bytes, 0x00020000);
    const int tile_bytes = SK_NW * MT * NT * 1024;
    const int ss_base = gridDim.x * tile_bytes;
    const int wave_off = w * MT * NT * 1024 + lane * 16;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int t = 0; t < NT; ++t)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[mt][t]), rs,
                                               blockIdx.x * tile_bytes + wave_off + (mt * NT + t) * 1024, 0, 16);
    if (threadIdx.x < MT * 16)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ss_l[threadIdx.x]), rs,
                                            ss_base + (blockIdx.x * MT * 16 + threadIdx.x) * 4, 0, 16);
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
    int s = 0;
    for (; s + 4 <= sa.ksplit; s += 4) {  // 4 splits' loads in flight per step
      u32x4 v[4][MT][NT];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int t = 0; t < NT; ++t)
            v[q][mt][t] = __builtin_amdgcn_raw_buffer_load_b128(
                rs, (b0 + s + q) * tile_bytes + wave_off + (mt * NT + t) * 1024, 0, 16);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[mt][t] += __builtin_bit_cast(f32x4, v[q][mt][t]);
    }
    for (; s < sa.ksplit; ++s)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[mt][t] += __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (b0 + s) * tile_bytes + wave_off + (mt * NT + t) * 1024,
                                                           0, 16));
    if (threadIdx.x < MT * 16) {
      float sum = 0.f;
      for (int sp = 0; sp < sa.ksplit; ++sp)
        sum += __uint_as_float(
            __builtin_amdgcn_raw_buffer_load_b32(rs, ss_base + ((b0 + sp) * MT * 16 + threadIdx.x) * 4, 0, 16));
      ss_l[threadIdx.x] = sum;
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
              const int b = m / qa.S, sq = m - b * qa.S;
              float r = v;
              if (head < qa.H + qa.Hkv) {
                int pos = qa.positions[m];
                if (pos < 0 || pos >= qa.table_len) JLA_FLAG(JLA_BOUNDS_ROPE_POS);
                pos = pos < 0 ? 0 : (pos >= qa.table_len ? qa.table_len - 1 : pos);
                const float2 cs = qa.table[(size_t)pos * (qa.Dh >> 1) + (d >> 1)];
                r = (d & 1) ? (pv * cs.y + v * cs.x) : (v * cs.x - pv * cs.y);
              }
              if (head < qa.H) {
                qa.q[((size_t)m * qa.H + head) * qa.Dh + d] = f2bf(r);
              } else {
                const int slot = qa.slot[0] + sq;
                if (slot < qa.T) {
                  const bool is_k = head < qa.H + qa.Hkv;
                  const int kh = is_k ? head - qa.H : head - qa.H - qa.Hkv;
                  bf16_t* cache = is_k ? qa.kc : qa.vc;
                  cache[(((size_t)b * qa.Hkv + kh) * qa.T + slot) * qa.Dh + d] = f2bf(r);
                } else {
                  JLA_FLAG(JLA_BOUNDS_KV_SLOT);
                }
              }
            }
          } else if (m < M && tile < NTT) {
            const size_t idx = (size_t)m * N + tile * 16 + c;
            if constexpr (MODE == MODE_RESIDUAL) {
              float* o = static_cast<float*>(out);
              const float nv = accumulate ? o[idx] + v : v;
              o[idx] = nv;
              if (qa.res_bf16) qa.res_bf16[idx] = f2bf(nv);
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

static int sk_mt(int M) { return M <= 16 ? 1 : (M <= 32 ? 2 : 4); }  // == the kernel's MT template

static int g_sk_nt = 0, g_sk_ks = 0;  // plan override for tuning (0 = heuristic)
void skinny_set_plan(int nt, int ksplit) {
  g_sk_nt = nt;
  g_sk_ks = ksplit;
}

static SkPlan sk_plan(int M, int N, int K, int mode) {
  const int KS = K >> 5, NTT = N >> 4;
  const int mt = sk_mt(M);
  SkPlan p;
  p.nt = (mode == MODE_SWIGLU || NTT >= 32 * SK_NW) ? 2 : 1;
  if (g_sk_nt > 0 && mode != MODE_SWIGLU) p.nt = g_sk_nt > 1 ? 2 : 1;
  p.groups = (NTT + SK_NW * p.nt - 1) / (SK_NW * p.nt);
  // LDS holds MT * kc A fragments of 1 KiB (<= 64 KiB); aim for ~512 workgroups, >= 8 k-steps
  // per split, at most 8 splits unless LDS forces more.
  const int kc_max = 64 / mt;
  int ks = (512 + p.groups - 1) / p.groups;
  ks = min(ks, 8);
  ks = min(ks, max(1, KS / 8));
  if (g_sk_ks > 0) ks = min(g_sk_ks, KS);
  ks = max(ks, (KS + kc_max - 1) / kc_max);
  ks = max(ks, 1);
  p.kc = (KS + ks - 1) / ks;
  p.ksplit = (KS + p.kc - 1) / p.kc;
  return p;
}

size_t skinny_workspace_floats(int M, int N, int K, int mode) {
  const SkPlan p = sk_plan(M, N, K, mode);
  if (p.ksplit <= 1) return 0;
  const int mt = sk_mt(M);
  const size_t wgs = (size_t)p.groups * p.ksplit;
  return wgs * ((size_t)SK_NW * mt * p.nt * 256 + mt * 16);
}

int skinny_tickets(int M, int N, int K, int mode) { return sk_plan(M, N, K, mode).groups; }

template <typename XT, int MT, int NT, int MODE>
static int launch_sk(const void* x, const void* W, void* out, int M, int N, int K, float eps, int use_rms,
                     int accumulate, int out_f32, const QKVArgs& qa, const SkPlan& p, float* ws, int32_t* tickets,
                     hipStream_t s) {
  constexpr int U = NT == 1 ? 8 : 4;
  SplitArgs sa{p.ksplit, p.kc, ws, (int)(skinny_workspace_floats(M, N, K, MODE) * 4), tickets};
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
static int sk_m(const void* x, const void* W, void* out, int M, int N, int K, float eps, int use_rms, int accumulate,
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
    case MODE_STORE: return sk_m<XT, MODE_STORE>(JLA_ARGS, out_f32, qa, p, ws, tickets, s);              \
    case MODE_RESIDUAL: return sk_m<XT, MODE_RESIDUAL>(JLA_ARGS, 1, qa, p, ws, tickets, s);              \
    case MODE_SWIGLU: return sk_m<XT, MODE_SWIGLU>(JLA_ARGS, 0, qa, p, ws, tickets, s);                  \
    case MODE_QKV: return sk_m<XT, MODE_QKV>(JLA_ARGS, 0, qa, p, ws, tickets, s);                        \
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

JLA_BOUNDS_ACCESSOR(skinny)

}  // namespace jla
