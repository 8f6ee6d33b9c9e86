// Decode chain (M <= 16 rows): the second half of a decoder layer plus the first projection of the
// next one -- wo (+ residual), w1|w3 (RMSNorm + SiLU * up), w2 (+ residual), next layer's wqkv (RMSNorm
// + RoPE + KV-cache write) -- as ONE launch instead of four.
//
// Reference ops: model.py:294 (wo), :392 / :398 (residual adds), :395 + :338 (norm, w1/w3/w2, SiLU),
// :384 + :210 + :58-92 + :169-199 (norm, wq/wk/wv, RoPE, cache write of the next block).
//
// Why: at batch 1-16 every decode GEMV streams its weights at ~6.9 TB/s but pays ~4 us of fill and
// drain per launch (profiles/README.md, "Small-batch decode": t = 3.9 us + bytes / 6.9 TB/s), five times
// per layer. Here the stages are consecutive blockIdx ranges of one grid; a workgroup of stage s first
// issues its weight ring (weights do not depend on the previous stage), THEN waits for every
// workgroup of stage s-1 to have published, then loads its activations and streams on. The fill of
// stage s overlaps the tail of stage s-1 (the "prefetch credit" of cdna_hip_programming.md section 5.6).
//
// Hand-offs (cdna_hip_programming.md Guideline 16, R1 form; placement-independent):
//   * every handed-off byte (h fp32, its bf16 mirror hb, the SwiGLU output) is stored write-through
//     (sc1 buffer stores), each storing wave drains (s_waitcnt vmcnt(0)), the workgroup barriers, and
//     one lane adds 1 to its XCD shard's arrival counter (relaxed, agent scope; 8 shards by blockIdx % 8 so
//     ~32 arrivals land on each word instead of 256+ on one);
//   * a consumer polls the 8 shards of its producer stage (8 lanes, relaxed agent loads, bounded by a
//     wall-clock timeout that sets the error word instead of hanging) and reads every handed-off byte
//     with sc1 loads (the activation ring and the residual read), so no acquire fence is needed.
// Counters are cumulative: after decode step e (device word `epoch`, bumped once per forward by
// chain_epoch_bump) shard t of stage s holds e * expect[t]. No per-call memset node.
// Deadlock freedom: a consumer only waits on LOWER blockIdx values, and each XCD dispatches its
// workgroups in blockIdx order, so every producer a resident consumer waits for is already resident.
//
// Per-stage tiling is the decode GEMV's (gemv.hip) at M <= 16: 4 waves split K, 1 (wo, w2) or 2 (w1|w3,
// wqkv) 16-column tiles per workgroup, 8 / 4 hand-counted ring slots; the cross-wave reduction and the
// epilogues are the same arithmetic (bit-identical outputs, tests/test_kernels_gpu.py::test_decode_chain).
#include "common.h"
#include "launchers.h"
#include "ring.h"

namespace jla {

__device__ u32x4 g_chain_zero[64];  // 1 KiB of zeros: past-the-end ring refills (MFMA adds 0)

constexpr int CH_NW = 4;
constexpr int CH_THREADS = CH_NW * 64;
constexpr int CH_SC1 = 16;  // buffer-op aux: sc1 (agent-coherent, write-through)

JLA_DEV __amdgpu_buffer_rsrc_t ch_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}

// wait until every workgroup of the producer stage has published for this epoch: ONE lane polls the 8 shards in
// turn (each shard word on its own 128-B line), sleeping between polls -- hundreds of waiting workgroups must not
// flood the counter lines the producers are adding to
constexpr int CH_LINE = 32;  // ints per counter line
JLA_DEV void chain_wait(const ChainArgs& a, const ChainStage& st, unsigned epoch) {
  if (threadIdx.x == 0) {
    const long long t0 = (long long)wall_clock64();
    bool timed_out = false;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const unsigned target = epoch * (unsigned)st.expect[t];
      const unsigned* c = a.counters + (st.dep * 8 + t) * CH_LINE;
      while (!timed_out && (int)(__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
        if ((long long)wall_clock64() - t0 > a.timeout_ticks) {
          __hip_atomic_store(a.error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          timed_out = true;
        }
        __builtin_amdgcn_s_sleep(4);
      }
    }
  }
  __syncthreads();
}

template <int NT, int MODE, int U>
JLA_DEV void chain_stage(const ChainArgs& a, const ChainStage& st, const int s, const int wg, const unsigned epoch,
                         float* smem) {
  float* red = smem;                       // [NW][NT][64][4]
  float* red_ss = red + CH_NW * NT * 256;  // [NW][16]
  float* inv_rms = red_ss + CH_NW * 16;    // [16]
  const int M = a.M, N = st.N, K = st.K;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int KS = K >> 5, NTT = N >> 4, nt0 = wg * NT;

  const u32x4* wt[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) wt[t] = static_cast<const u32x4*>(st.W) + (size_t)min(nt0 + t, NTT - 1) * KS * 64 + lane;
  const bf16_t* xp = st.x + (size_t)min(lane & 15, M - 1) * K + 8 * (lane >> 4);  // padding rows re-read row M-1
  const u32x4* zfrag = g_chain_zero + lane;
  const int n = (KS - w + CH_NW - 1) / CH_NW;  // k-steps of this wave: ks = w + i * NW

  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss = 0.f;
  u32x4 bq[U][NT] = {};
  u32x4 aq[U] = {};
  constexpr int L = NT + 1;  // loads per ring slot
  auto issue_w = [&](int i, u32x4* b) {
    const bool valid = i < n;
    const size_t ks = (size_t)(w + i * CH_NW);
#pragma unroll
    for (int t = 0; t < NT; ++t) asm_load_nt<true>(b[t], valid ? (const void*)(wt[t] + ks * 64) : (const void*)zfrag);
  };
  auto issue_x = [&](int i, u32x4& xr) {
    const bool valid = i < n;
    const size_t ks = (size_t)(w + i * CH_NW);
    asm_load_sc1(xr, valid ? (const void*)(xp + ks * 32) : (const void*)zfrag);
  };

  unsigned long long* stamp = a.stamps ? a.stamps + (size_t)blockIdx.x * 4 : nullptr;  // diagnostic timeline
  if (stamp && threadIdx.x == 0) stamp[0] = wall_clock64();
  // prologue: the weight ring first (independent of the producer), then the hand-off wait, then x
#pragma unroll
  for (int u = 0; u < U; ++u) issue_w(u, bq[u]);
  if (st.dep >= 0) chain_wait(a, st, epoch);
  if (stamp && threadIdx.x == 0) stamp[1] = wall_clock64();
#pragma unroll
  for (int u = 0; u < U; ++u) issue_x(u, aq[u]);
  wait_vmcnt<0>();  // the x loads of the first slots are the dependent round trip: wait for all of them
#pragma unroll
  for (int u = 0; u < U; ++u) {
#pragma unroll
    for (int t = 0; t < NT; ++t) pin(bq[u][t]);
    pin(aq[u]);
  }
  for (int i0 = 0; i0 < n; i0 += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      wait_vmcnt<L * (U - 1)>();  // slot u (the oldest L loads) has landed
#pragma unroll
      for (int t = 0; t < NT; ++t) pin(bq[u][t]);
      pin(aq[u]);
      ss = dot8_bf16(aq[u], aq[u], ss);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mfma16x16x32(aq[u], bq[u][t], acc[t]);
      issue_w(i0 + U + u, bq[u]);
      issue_x(i0 + U + u, aq[u]);
    }
  }
  wait_vmcnt<0>();  // retire the past-the-end refills; keep every ring register live until then
#pragma unroll
  for (int u = 0; u < U; ++u) {
#pragma unroll
    for (int t = 0; t < NT; ++t) pin(bq[u][t]);
    pin(aq[u]);
  }

  if (stamp && threadIdx.x == 0) stamp[2] = wall_clock64();
  // ---- cross-wave reduction through LDS
#pragma unroll
  for (int t = 0; t < NT; ++t) *reinterpret_cast<f32x4*>(red + ((w * NT + t) * 64 + lane) * 4) = acc[t];
  const bool use_rms = st.eps >= 0.f;
  if (use_rms) {
    float v = ss;
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (lane < 16) red_ss[w * 16 + lane] = v;
  }
  __syncthreads();
  if (threadIdx.x < 16) {
    float r = 1.f;
    if (use_rms) {
      float v = 0.f;
      for (int ww = 0; ww < CH_NW; ++ww) v += red_ss[ww * 16 + threadIdx.x];
      r = rsqrtf(v / (float)K + st.eps);
    }
    inv_rms[threadIdx.x] = r;
  }
  __syncthreads();
  auto reduced = [&](int t, int ln, int i) {
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < CH_NW; ++ww) v += red[((ww * NT + t) * 64 + ln) * 4 + i];
    return v;
  };

  // ---- epilogue; c (column within the tile) is the fastest index
  if constexpr (MODE == MODE_SWIGLU) {
    const int F = N >> 1;
    const __amdgpu_buffer_rsrc_t ro = ch_rsrc(st.out);
    for (int e = threadIdx.x; e < (NT / 2) * 256; e += CH_THREADS) {
      const int c = e & 15, m = (e >> 4) & 15, p = e >> 8;
      const int ln = (m >> 2) * 16 + c, i = m & 3;
      const int gtile = nt0 + 2 * p;
      if (m < M && gtile < NTT) {
        const float sc = inv_rms[m];
        const float g = reduced(2 * p, ln, i) * sc, u = reduced(2 * p + 1, ln, i) * sc;
        __builtin_amdgcn_raw_buffer_store_b16(f2bf(silu(g) * u), ro, (int)(((size_t)m * F + (gtile >> 1) * 16 + c) * 2),
                                             0, CH_SC1);
      }
    }
  } else if constexpr (MODE == MODE_RESIDUAL) {
    const __amdgpu_buffer_rsrc_t rh = ch_rsrc(st.out), rb = ch_rsrc(st.mirror);
    for (int e = threadIdx.x; e < NT * 256; e += CH_THREADS) {
      const int c = e & 15, m = (e >> 4) & 15, t = e >> 8;
      const int ln = (m >> 2) * 16 + c, i = m & 3;
      const int tile = nt0 + t;
      if (m >= M || tile >= NTT) continue;
      const float v = reduced(t, ln, i);
      const int idx = m * N + tile * 16 + c;
      const float nv = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rh, idx * 4, 0, CH_SC1)) + v;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(nv), rh, idx * 4, 0, CH_SC1);
      __builtin_amdgcn_raw_buffer_store_b16(f2bf(nv), rb, idx * 2, 0, CH_SC1);
    }
  } else {  // MODE_QKV: consumed by the next launch (attention): plain stores
    const QKVArgs& qa = st.qa;
    for (int e = threadIdx.x; e < NT * 256; e += CH_THREADS) {
      const int c = e & 15, m = (e >> 4) & 15, t = e >> 8;
      const int ln = (m >> 2) * 16 + c, i = m & 3;
      const int tile = nt0 + t;
      if (m >= M || tile >= NTT) continue;
      const float v = reduced(t, ln, i) * inv_rms[m];
      const int col = tile * 16 + c;
      const int head = col / qa.Dh, d = col - head * qa.Dh;
      const int b = m / qa.S, sq = m - b * qa.S;
      float r = v;
      if (head < qa.H + qa.Hkv) {  // RoPE pairs (d, d^1) are both in this 16-column tile
        const float pv = reduced(t, ln ^ 1, i) * inv_rms[m];
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
  }

  // ---- publish: every storing wave drains its write-through stores, then one arrival per workgroup
  if (st.publish) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_fetch_add(a.counters + (s * 8 + (blockIdx.x & 7)) * CH_LINE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (stamp && threadIdx.x == 0) stamp[3] = wall_clock64();
}

// Stage order is fixed: 0 = wo (residual), 1 = w1|w3 (SwiGLU), 2 = w2 (residual), 3 = next wqkv (optional)
__global__ void __launch_bounds__(CH_THREADS) decode_chain_kernel(const ChainArgs a) {
  extern __shared__ float smem[];
  const int b = blockIdx.x;
  const unsigned epoch = *a.epoch;
  if (b < a.st[1].wg_begin) {
    chain_stage<1, MODE_RESIDUAL, 8>(a, a.st[0], 0, b, epoch, smem);
  } else if (b < a.st[2].wg_begin) {
    chain_stage<2, MODE_SWIGLU, 4>(a, a.st[1], 1, b - a.st[1].wg_begin, epoch, smem);
  } else if (a.nstages == 3 || b < a.st[3].wg_begin) {
    chain_stage<1, MODE_RESIDUAL, 8>(a, a.st[2], 2, b - a.st[2].wg_begin, epoch, smem);
  } else {
    chain_stage<2, MODE_QKV, 4>(a, a.st[3], 3, b - a.st[3].wg_begin, epoch, smem);
  }
}

__global__ void chain_epoch_bump_kernel(unsigned* epoch) {
  if (threadIdx.x == 0) *epoch = *epoch + 1;
}

static int chain_tiles(int mode) { return (mode == MODE_RESIDUAL) ? 1 : 2; }

int decode_chain(ChainArgs a, hipStream_t s) {
  if (a.M <= 0 || a.M > 16 || (a.nstages != 3 && a.nstages != 4)) return -1;
  const int modes[4] = {MODE_RESIDUAL, MODE_SWIGLU, MODE_RESIDUAL, MODE_QKV};
  int total = 0;
  for (int i = 0; i < a.nstages; ++i) {
    ChainStage& st = a.st[i];
    if (st.mode != modes[i] || (st.N & 31) || (st.K & 31) || st.K <= 0 || st.N <= 0) return -1;
    if (i == 3 && (st.qa.Dh % 16 || a.M % st.qa.S)) return -1;
    const int nt = chain_tiles(st.mode);
    const int wgs = ((st.N >> 4) + nt - 1) / nt;
    st.wg_begin = total;
    st.wg_count = wgs;
    st.dep = i - 1;
    st.publish = i + 1 < a.nstages;
    total += wgs;
  }
  for (int i = 1; i < a.nstages; ++i) {  // arrivals of stage i-1 per shard (blockIdx % 8)
    const ChainStage& p = a.st[i - 1];
    for (int t = 0; t < 8; ++t) {
      int c = 0;
      for (int g = p.wg_begin; g < p.wg_begin + p.wg_count; ++g) c += (g & 7) == t;
      a.st[i].expect[t] = c;
    }
  }
  if (a.nstages == 3) a.st[3].wg_begin = total;
  const size_t lds = sizeof(float) * (CH_NW * 2 * 256 + CH_NW * 16 + 16);
  decode_chain_kernel<<<total, CH_THREADS, lds, s>>>(a);
  JLA_CHECK_LAUNCH();
  return 0;
}

int chain_epoch_bump(unsigned* epoch, hipStream_t s) {
  chain_epoch_bump_kernel<<<1, 64, 0, s>>>(epoch);
  JLA_CHECK_LAUNCH();
  return 0;
}

JLA_BOUNDS_ACCESSOR(chain)

}  // namespace jla
