// Skinny (decode) linear layer: y[M, N] = epilogue( [inv_rms(x) *] x[M, K] @ W[N, K]^T ), M <= 64.
//
// Reference ops: every nn.Dense of model.py (wq/wk/wv :210, wo :294, w1/w3/w2 :338, lm_head :736)
// plus the RMSNorm that precedes qkv / w1|w3 / lm_head (model.py:384, :395, :662) and the residual
// adds (:392, :398).
//
// Decode is HBM-bound on the weight stream (batch 1..64 rows), so the kernel is organised around
// streaming the packed weights exactly once at full bandwidth:
//   * one workgroup = NT consecutive 16-column n-tiles x the WHOLE K, split across NW = 8 waves
//     (intra-workgroup split-K: wave w takes k-steps w, w+8, w+16, ... so the 8 waves of a
//     workgroup fetch 8 consecutive KiB of the n-tile's contiguous packed block at a time);
//   * each k-step is one 1 KiB non-temporal global_load_dwordx4 per n-tile (the B operand of
//     v_mfma_f32_16x16x32_bf16 as-is) plus the 16(m) x 32(k) activation fragment, read straight
//     from the L2-resident x (fp32 residual stream converted to bf16 in registers);
//   * MT = ceil(M/16) m-tiles reuse each weight fragment (M <= 16 costs the same as M = 1);
//   * the sum of squares for RMSNorm is accumulated from the same activation loads (every x element
//     is loaded exactly once per workgroup), so the norm costs no extra pass and no extra launch;
//   * the 8 partial accumulators are reduced through LDS and a fused epilogue applies the norm scale
//     and stores bf16/fp32, accumulates into the fp32 residual stream, or applies SiLU(gate)*up for
//     the interleaved [w1;w3] weight (gate/up alternate in 16-row tiles so one workgroup owns both).
// No atomics: results are deterministic and the residual add happens exactly once.
#include "common.h"
#include "launchers.h"

namespace jla {

constexpr int GEMV_NW = 8;  // waves per workgroup

template <typename XT>
struct XFrag;

template <>
struct XFrag<float> {
  // lane's 8 consecutive fp32 activations -> bf16 fragment; accumulate squares for RMSNorm
  static JLA_DEV u32x4 load(const float* x, size_t off, float& ss) {
    const float4* p = reinterpret_cast<const float4*>(x + off);
    float4 a = p[0], b = p[1];
    ss += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w + b.x * b.x + b.y * b.y + b.z * b.z + b.w * b.w;
    u32x4 r;
    r[0] = pack2bf(a.x, a.y);
    r[1] = pack2bf(a.z, a.w);
    r[2] = pack2bf(b.x, b.y);
    r[3] = pack2bf(b.z, b.w);
    return r;
  }
};

template <>
struct XFrag<bf16_t> {
  static JLA_DEV u32x4 load(const bf16_t* x, size_t off, float& ss) {
    u32x4 r = *reinterpret_cast<const u32x4*>(x + off);
    float f[8];
    unpack8(r, f);
#pragma unroll
    for (int i = 0; i < 8; ++i) ss += f[i] * f[i];
    return r;
  }
};

template <typename XT, int MT, int NT, int MODE>
__global__ void __launch_bounds__(GEMV_NW * 64)
    linear_skinny_kernel(const XT* __restrict__ x, const u32x4* __restrict__ W, void* __restrict__ out,
                         int M, int N, int K, float eps, int use_rms, int accumulate, int out_f32) {
  // k-steps in flight per wave (8 KiB of weights at M <= 16); fp32 activations cost 2x the
  // registers of bf16 ones, so fewer steps are kept in flight for MT > 1 to stay spill-free.
  constexpr int U0 = (NT == 1) ? 8 : 4;
  constexpr int UD = (sizeof(XT) == 4 && MT > 1) ? MT : 1;
  constexpr int U = (U0 / UD) < 2 ? 2 : (U0 / UD);
  extern __shared__ float smem[];
  float* red = smem;                                    // [NW][MT][NT][64][4]
  float* red_ss = red + GEMV_NW * MT * NT * 256;        // [NW][MT][16]
  float* inv_rms = red_ss + GEMV_NW * MT * 16;          // [MT*16]

  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int KS = K >> 5;
  const int NTT = N >> 4;
  const int nt0 = blockIdx.x * NT;

  // clamp tiles of a ragged last workgroup (computed but not stored)
  int ntile[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) ntile[t] = min(nt0 + t, NTT - 1);

  size_t xoff[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    int row = min(mt * 16 + (lane & 15), M - 1);  // padding rows re-read the last row (not stored)
    xoff[mt] = (size_t)row * K + 8 * (lane >> 4);
  }

  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[mt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) ss[mt] = 0.f;

  const u32x4* wt[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) wt[t] = W + (size_t)ntile[t] * KS * 64 + lane;

  int ks = w;
  // main loop: U k-steps per iteration, all loads issued before the MFMAs
  for (; ks + (U - 1) * GEMV_NW < KS; ks += U * GEMV_NW) {
    u32x4 b[U][NT];
    u32x4 a[U][MT];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < NT; ++t) b[u][t] = load_nt(wt[t] + (size_t)(ks + u * GEMV_NW) * 64);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) a[u][mt] = XFrag<XT>::load(x, xoff[mt] + (size_t)(ks + u * GEMV_NW) * 32, ss[mt]);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[mt][t] = mfma16x16x32(a[u][mt], b[u][t], acc[mt][t]);
  }
  // remainder k-steps
  for (; ks < KS; ks += GEMV_NW) {
    u32x4 b[NT], a[MT];
#pragma unroll
    for (int t = 0; t < NT; ++t) b[t] = load_nt(wt[t] + (size_t)ks * 64);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) a[mt] = XFrag<XT>::load(x, xoff[mt] + (size_t)ks * 32, ss[mt]);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[mt][t] = mfma16x16x32(a[mt], b[t], acc[mt][t]);
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
  __syncthreads();
  if (threadIdx.x < MT * 16) {
    float r = 1.f;
    if (use_rms) {
      float s = 0.f;
      for (int ww = 0; ww < GEMV_NW; ++ww) s += red_ss[ww * MT * 16 + threadIdx.x];
      r = rsqrtf(s / (float)K + eps);
    }
    inv_rms[threadIdx.x] = r;
  }
  __syncthreads();

  // ---- fused epilogue; c (column within the tile) is the fastest index -> 64 B row segments
  if (MODE == MODE_SWIGLU) {
    constexpr int NP = NT / 2;
    const int F = N >> 1;
    bf16_t* o = static_cast<bf16_t*>(out);
    for (int e = threadIdx.x; e < MT * NP * 256; e += GEMV_NW * 64) {
      const int c = e & 15, ml = (e >> 4) & 15, p = (e >> 8) % NP, mt = e / (256 * NP);
      const int m = mt * 16 + ml;
      const int ln = (ml >> 2) * 16 + c, i = ml & 3;
      float g = 0.f, u = 0.f;
      for (int ww = 0; ww < GEMV_NW; ++ww) {
        g += red[(((ww * MT + mt) * NT + 2 * p) * 64 + ln) * 4 + i];
        u += red[(((ww * MT + mt) * NT + 2 * p + 1) * 64 + ln) * 4 + i];
      }
      const int gtile = nt0 + 2 * p;
      if (m < M && gtile + 1 < NTT + 1 && gtile < NTT) {
        const float sc = inv_rms[m];
        g *= sc;
        u *= sc;
        o[(size_t)m * F + (gtile >> 1) * 16 + c] = f2bf(silu(g) * u);
      }
    }
  } else {
    for (int e = threadIdx.x; e < MT * NT * 256; e += GEMV_NW * 64) {
      const int c = e & 15, ml = (e >> 4) & 15, t = (e >> 8) % NT, mt = e / (256 * NT);
      const int m = mt * 16 + ml;
      const int ln = (ml >> 2) * 16 + c, i = ml & 3;
      float v = 0.f;
      for (int ww = 0; ww < GEMV_NW; ++ww) v += red[(((ww * MT + mt) * NT + t) * 64 + ln) * 4 + i];
      const int tile = nt0 + t;
      if (m < M && tile < NTT) {
        v *= inv_rms[m];
        const size_t idx = (size_t)m * N + tile * 16 + c;
        if (MODE == MODE_RESIDUAL) {
          float* o = static_cast<float*>(out);
          o[idx] = accumulate ? o[idx] + v : v;
        } else if (out_f32) {
          static_cast<float*>(out)[idx] = v;
        } else {
          static_cast<bf16_t*>(out)[idx] = f2bf(v);
        }
      }
    }
  }
}

template <typename XT, int MT, int NT, int MODE>
static int launch_skinny(const void* x, const void* W, void* out, int M, int N, int K, float eps, int use_rms,
                         int accumulate, int out_f32, hipStream_t s) {
  const int NTT = N >> 4;
  const int grid = (NTT + NT - 1) / NT;
  const size_t lds = sizeof(float) * (GEMV_NW * MT * NT * 256 + GEMV_NW * MT * 16 + MT * 16);
  if (lds > 65536) {  // opt in to > 64 KiB of dynamic LDS once (not a stream op: capture-safe)
    static bool attr_set = false;
    if (!attr_set) {
      hipFuncSetAttribute(reinterpret_cast<const void*>(&linear_skinny_kernel<XT, MT, NT, MODE>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr_set = true;
    }
  }
  linear_skinny_kernel<XT, MT, NT, MODE><<<grid, GEMV_NW * 64, lds, s>>>(
      static_cast<const XT*>(x), static_cast<const u32x4*>(W), out, M, N, K, eps, use_rms, accumulate, out_f32);
  JLA_CHECK_LAUNCH();
  return 0;
}

template <typename XT, int MT, int MODE>
static int dispatch_nt(const void* x, const void* W, void* out, int M, int N, int K, float eps, int use_rms,
                       int accumulate, int out_f32, hipStream_t s) {
  const int NTT = N >> 4;
  // one n-tile per workgroup unless that leaves > 2 workgroups per CU anyway; SwiGLU needs the
  // gate/up tile pair in one workgroup.
  if (MODE == MODE_SWIGLU || NTT >= 1024)
    return launch_skinny<XT, MT, 2, MODE>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, s);
  return launch_skinny<XT, MT, (MODE == MODE_SWIGLU ? 2 : 1), MODE>(x, W, out, M, N, K, eps, use_rms, accumulate,
                                                                     out_f32, s);
}

template <typename XT, int MODE>
static int dispatch_mt(const void* x, const void* W, void* out, int M, int N, int K, float eps, int use_rms,
                       int accumulate, int out_f32, hipStream_t s) {
  if (M <= 16) return dispatch_nt<XT, 1, MODE>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, s);
  if (M <= 32) return dispatch_nt<XT, 2, MODE>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, s);
  return dispatch_nt<XT, 4, MODE>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, s);
}

int linear_skinny(const void* x, int x_is_f32, const void* W, void* out, int M, int N, int K, int mode,
                  float rms_eps, int accumulate, int out_f32, hipStream_t s) {
  if (M <= 0) return 0;
  if (M > SKINNY_MAX_M || (N & 15) || (K & 31)) return -1;
  if (mode == MODE_SWIGLU && (N & 31)) return -1;
  const int use_rms = rms_eps >= 0.f;
  const float eps = use_rms ? rms_eps : 0.f;
#define JLA_MODE(XT)                                                                                          \
  switch (mode) {                                                                                             \
    case MODE_STORE: return dispatch_mt<XT, MODE_STORE>(x, W, out, M, N, K, eps, use_rms, accumulate, out_f32, s); \
    case MODE_RESIDUAL: return dispatch_mt<XT, MODE_RESIDUAL>(x, W, out, M, N, K, eps, use_rms, accumulate, 1, s);   \
    case MODE_SWIGLU: return dispatch_mt<XT, MODE_SWIGLU>(x, W, out, M, N, K, eps, use_rms, accumulate, 0, s);       \
    default: return -1;                                                                                       \
  }
  if (x_is_f32) {
    JLA_MODE(float)
  } else {
    JLA_MODE(bf16_t)
  }
#undef JLA_MODE
}

}  // namespace jla
