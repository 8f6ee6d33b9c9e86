// Embedding gather and RMSNorm kernels (reference: model.py:28-48 RMSNorm, :611-617 wte).
//
// The residual stream is fp32 [M, D]. RMSNorm weights are folded into the next projection at load
// time, so the decode path never runs these norm kernels: the skinny GEMM computes inv_rms in its
// own K loop. These kernels serve the prefill path (rms_scale -> bf16 GEMM operand), the final
// norm of hidden-state outputs, and the embedding lookup.
#include "common.h"
#include "launchers.h"

namespace jla {

// one block per row; 16-byte vectorised bf16 loads, fp32 stores
__global__ void __launch_bounds__(256) embedding_kernel(const int32_t* __restrict__ ids,
                                                        const bf16_t* __restrict__ table,
                                                        float* __restrict__ out, bf16_t* __restrict__ mirror,
                                                        int D, int V) {
  const int row = blockIdx.x;
  int id = ids[row];
  if ((id < 0 || id >= V) && threadIdx.x == 0) JLA_FLAG(JLA_BOUNDS_TOKEN);
  id = id < 0 ? 0 : (id >= V ? V - 1 : id);
  const u32x4* src = reinterpret_cast<const u32x4*>(table + (size_t)id * D);
  float4* dst = reinterpret_cast<float4*>(out + (size_t)row * D);
  u32x4* mdst = mirror ? reinterpret_cast<u32x4*>(mirror + (size_t)row * D) : nullptr;
  for (int i = threadIdx.x; i < D / 8; i += blockDim.x) {
    const u32x4 v = src[i];
    float f[8];
    unpack8(v, f);
    dst[2 * i] = make_float4(f[0], f[1], f[2], f[3]);
    dst[2 * i + 1] = make_float4(f[4], f[5], f[6], f[7]);
    if (mdst) mdst[i] = v;  // bf16 mirror of the residual stream (exact: rows are bf16)
  }
}

int embedding(const int32_t* ids, const bf16_t* table, float* out, bf16_t* mirror, int M, int D, int V,
              hipStream_t s) {
  if (D % 8) return -1;
  if (M == 0) return 0;
  embedding_kernel<<<M, 256, 0, s>>>(ids, table, out, mirror, D, V);
  JLA_CHECK_LAUNCH();
  return 0;
}

// out_bf16[m, :] = bf16(x[m, :] * rsqrt(mean(x^2) + eps)); optional weight (fp32) -> fp32 out.
template <bool WEIGHTED>
__global__ void __launch_bounds__(256) rms_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                  void* __restrict__ out, int D, float eps) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const float4* xr = reinterpret_cast<const float4*>(x + (size_t)row * D);
  float ss = 0.f;
  for (int i = threadIdx.x; i < D / 4; i += blockDim.x) {
    float4 v = xr[i];
    ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / (float)D + eps);
  if (WEIGHTED) {
    float4* o = reinterpret_cast<float4*>(static_cast<float*>(out) + (size_t)row * D);
    const float4* wr = reinterpret_cast<const float4*>(w);
    for (int i = threadIdx.x; i < D / 4; i += blockDim.x) {
      float4 v = xr[i], g = wr[i];
      o[i] = make_float4(v.x * inv * g.x, v.y * inv * g.y, v.z * inv * g.z, v.w * inv * g.w);
    }
  } else {
    uint2* o = reinterpret_cast<uint2*>(static_cast<bf16_t*>(out) + (size_t)row * D);
    for (int i = threadIdx.x; i < D / 4; i += blockDim.x) {
      float4 v = xr[i];
      o[i] = make_uint2(pack2bf(v.x * inv, v.y * inv), pack2bf(v.z * inv, v.w * inv));
    }
  }
}

int rms_scale(const float* x, bf16_t* out, int M, int D, float eps, hipStream_t s) {
  if (D % 4) return -1;
  if (M == 0) return 0;
  rms_kernel<false><<<M, 256, 0, s>>>(x, nullptr, out, D, eps);
  JLA_CHECK_LAUNCH();
  return 0;
}

// bf16 input (the residual mirror): statistics from the bf16 values, like the decode kernels
__global__ void __launch_bounds__(256) rms_bf16_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ out,
                                                       int D, float eps) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const u32x4* xr = reinterpret_cast<const u32x4*>(x + (size_t)row * D);
  u32x4* o = reinterpret_cast<u32x4*>(out + (size_t)row * D);
  float ss = 0.f;
  for (int i = threadIdx.x; i < D / 8; i += blockDim.x) {
    float f[8];
    unpack8(xr[i], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += f[j] * f[j];
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / (float)D + eps);
  for (int i = threadIdx.x; i < D / 8; i += blockDim.x) {
    float f[8];
    unpack8(xr[i], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] *= inv;
    o[i] = pack8(f);
  }
}

// inv[row] = 1 / sqrt(mean(x[row]^2) + eps) of bf16 rows (reference model.py:42-43), one wave per row, 4 rows per
// block: the fused-RMSNorm statistic of a tiled GEMM computed ahead of it (gemm.hip gemm4, RMS mode 2), so the
// GEMM's MFMA stream carries no sum-of-squares VALU work (that cost gemm4 ~10 %).
__global__ void __launch_bounds__(256) rms_rowinv_kernel(const bf16_t* __restrict__ x, float* __restrict__ inv, int M,
                                                         int D, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const u32x4* xr = reinterpret_cast<const u32x4*>(x + (size_t)row * D);
  float s0 = 0.f, s1 = 0.f;
  // 4 of the row's 16-byte pieces per lane in flight at once (D = 4096: all 8 in two round trips, not eight)
#pragma unroll 4
  for (int i = lane; i < D / 8; i += 64) {
    const u32x4 v = xr[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float lo = __uint_as_float(v[e] << 16), hi = __uint_as_float(v[e] & 0xffff0000u);
      s0 = fmaf(lo, lo, s0);
      s1 = fmaf(hi, hi, s1);
    }
  }
  const float t = wave_sum(s0 + s1);
  if (lane == 0) inv[row] = 1.f / sqrtf(t / (float)D + eps);
}

int rms_rowinv(const bf16_t* x, float* inv, int M, int D, float eps, hipStream_t s) {
  if (D % 8) return -1;
  if (M == 0) return 0;
  rms_rowinv_kernel<<<(M + 3) / 4, 256, 0, s>>>(x, inv, M, D, eps);
  JLA_CHECK_LAUNCH();
  return 0;
}

int rms_scale_bf16(const bf16_t* x, bf16_t* out, int M, int D, float eps, hipStream_t s) {
  if (D % 8) return -1;
  if (M == 0) return 0;
  rms_bf16_kernel<<<M, 256, 0, s>>>(x, out, D, eps);
  JLA_CHECK_LAUNCH();
  return 0;
}

int rmsnorm(const float* x, const float* w, float* out, int M, int D, float eps, hipStream_t s) {
  if (D % 4) return -1;
  if (M == 0) return 0;
  rms_kernel<true><<<M, 256, 0, s>>>(x, w, out, D, eps);
  JLA_CHECK_LAUNCH();
  return 0;
}

// h (fp32) += p (bf16 or fp32); hb = bf16(h) -- the residual epilogue of a row-parallel projection whose
// partial sums came back from RCCL (tensor-parallel prefill-sized messages): one pass instead of add_ + copy_.
template <bool BF16>
__global__ void __launch_bounds__(256) residual_add_kernel(float* __restrict__ h, const void* __restrict__ p,
                                                           bf16_t* __restrict__ hb, long long n8) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    float a[8];
    if constexpr (BF16) {
      unpack8(reinterpret_cast<const u32x4*>(p)[i], a);
    } else {
      const float4 v0 = reinterpret_cast<const float4*>(p)[2 * i], v1 = reinterpret_cast<const float4*>(p)[2 * i + 1];
      a[0] = v0.x; a[1] = v0.y; a[2] = v0.z; a[3] = v0.w; a[4] = v1.x; a[5] = v1.y; a[6] = v1.z; a[7] = v1.w;
    }
    float4* hv = reinterpret_cast<float4*>(h) + 2 * i;
    float4 x0 = hv[0], x1 = hv[1];
    x0.x += a[0]; x0.y += a[1]; x0.z += a[2]; x0.w += a[3];
    x1.x += a[4]; x1.y += a[5]; x1.z += a[6]; x1.w += a[7];
    hv[0] = x0;
    hv[1] = x1;
    const float r[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
    reinterpret_cast<u32x4*>(hb)[i] = pack8(r);
  }
}

int residual_add(float* h, const void* p, int p_bf16, bf16_t* hb, long long n, hipStream_t s) {
  if (n % 8) return -1;
  if (n == 0) return 0;
  const long long n8 = n / 8;
  const long long want = (n8 + 255) / 256;
  const int grid = (int)(want < 4096 ? want : 4096);
  if (p_bf16) residual_add_kernel<true><<<grid, 256, 0, s>>>(h, p, hb, n8);
  else residual_add_kernel<false><<<grid, 256, 0, s>>>(h, p, hb, n8);
  JLA_CHECK_LAUNCH();
  return 0;
}

// Cache warm-up of a stream: every byte of [p, p + n16 * 16) is loaded with the default cache policy (allocates in the
// 256 MiB Infinity Cache) and discarded. Diagnostic (tools/bench_prefetch.py, tools/graph_concurrency.py): a decode
// GEMV whose weights were just warmed this way runs no faster (profiles/r3_prefetch_gemv.jsonl), so the model does
// not use it. 16 loads in flight per lane; the xor keeps the loads alive (the sink is written only when it
// matches `key`, a condition the compiler cannot see through and the host never arranges).
__global__ void __launch_bounds__(256) prefetch_kernel(const u32x4* __restrict__ p, long long n16,
                                                       unsigned* __restrict__ sink, unsigned key) {
  constexpr int U = 16;
  unsigned acc = 0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = p[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u][0] ^ v[u][3];
  }
  for (; i < n16; i += stride) acc ^= p[i][1];
  if (acc == key) sink[0] = acc;  // (practically) never true, but the loads must happen to know
}

int prefetch(const void* p, long long nbytes, int grid, unsigned* sink, hipStream_t s) {
  if (nbytes <= 0) return 0;
  prefetch_kernel<<<grid, 256, 0, s>>>(static_cast<const u32x4*>(p), nbytes / 16, sink, 0x9e3779b9u);
  JLA_CHECK_LAUNCH();
  return 0;
}

// Streaming-read probe in the decode kernels' own access pattern (runtime/benchmark.py calibration,
// stream_read_seq_tbps): each wave reads ONE contiguous range front to back, 1 KiB per wave instruction, U
// instructions in flight -- as the decode attention streams a (row, kv head) pair and the GEMV a weight column group
// (the grid-strided prefetch_kernel above scatters every wave's loads over the whole buffer and reads ~20 % slower).
__global__ void __launch_bounds__(256) stream_probe_kernel(const u32x4* __restrict__ p, long long n16_per_wave,
                                                           unsigned* __restrict__ sink, unsigned key) {
  constexpr int U = 8;
  const int lane = threadIdx.x & 63;
  const long long wave = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const u32x4* q = p + wave * n16_per_wave;
  unsigned acc = 0;
  for (long long i = lane; i + (U - 1) * 64 < n16_per_wave; i += U * 64) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = q[i + u * 64];
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u][0] ^ v[u][3];
  }
  if (acc == key) sink[0] = acc;
}

int stream_probe(const void* p, long long nbytes, int grid, unsigned* sink, hipStream_t s) {
  const long long waves = (long long)grid * 4;
  const long long per = nbytes / 16 / waves / 512 * 512;  // whole 8 KiB groups per wave
  if (per <= 0) return -1;
  stream_probe_kernel<<<grid, 256, 0, s>>>(static_cast<const u32x4*>(p), per, sink, 0x9e3779b9u);
  JLA_CHECK_LAUNCH();
  return 0;
}

// Shader-clock probe (runtime/benchmark.py calibration): every workgroup keeps its SIMDs' matrix pipes busy with
// dependent MFMA chains for `iters` rounds, the first lane of workgroup 0 reads the shader cycle counter (s_memtime)
// and the constant 100 MHz counter (s_memrealtime) before and after: cycles / real time = the clock the chip runs at
// under a full matrix load (sysfs pp_dpm_sclk shows a DPM request level, not the running clock).
__global__ void __launch_bounds__(256) clock_probe_kernel(int iters, unsigned long long* __restrict__ out) {
  const bool rec = blockIdx.x == 0 && threadIdx.x == 0;
  unsigned long long c0 = 0, r0 = 0;
  if (rec) {
    c0 = __builtin_readcyclecounter();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  f32x4 acc[4] = {};
  const u32x4 a = {threadIdx.x, 1u, 2u, 3u}, b = {blockIdx.x, 5u, 6u, 7u};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = mfma16x16x32(a, b, acc[j]);
  }
  if (rec) {
    const unsigned long long c1 = __builtin_readcyclecounter(), r1 = __builtin_amdgcn_s_memrealtime();
    out[0] = c1 - c0;
    out[1] = r1 - r0;
  }
  if (acc[0][0] == 1.2345f && acc[3][1] == 6.789f) out[2] = 1;  // keep the chain alive
}

int clock_probe(int iters, int grid, unsigned long long* out, hipStream_t s) {
  clock_probe_kernel<<<grid, 256, 0, s>>>(iters, out);
  JLA_CHECK_LAUNCH();
  return 0;
}

JLA_BOUNDS_ACCESSOR(norm_embed)

}  // namespace jla
