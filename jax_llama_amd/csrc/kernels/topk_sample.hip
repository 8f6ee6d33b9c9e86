// On-device top-k / top-p sampler (replaces HF FlaxTemperatureLogitsWarper ->
// FlaxTopKLogitsWarper -> FlaxTopPLogitsWarper -> categorical that the reference inherits through
// generation.py:28-41 with do_sample = temperature != 0, top_k = 50).
//
// Two kernels, no host sync, hipGraph-capturable:
//   topk_chunk:  grid (ceil(V/4096), B). A 256-thread workgroup holds a 4096-logit chunk in
//                registers (16 keys per thread, order-preserving uint32 of the fp32 logit) and finds
//                the chunk's K-th largest key by 4-pass LDS radix select (8 bits per pass, one wave
//                scans the 256-bin histogram with DPP-free shuffles). It emits exactly K candidates:
//                everything above the threshold plus the lowest-index ties.
//   topk_merge:  one workgroup per row merges the C = chunks*K candidates the same way, sorts the K
//                survivors in one wave (64-lane bitonic network on (key, -index)), and either writes
//                them (vocab-parallel TP: each rank's top-K is all-gathered, 400 B per rank per row,
//                then merged again -- exact, since the global top-K is inside the union) or samples:
//                temperature, top-p over the sorted survivors (HF keep rule: a token survives if the
//                probability mass strictly before it is < top_p; the first always survives), then
//                Gumbel-max with counter-based Philox4x32-10 keyed by (seed, step, row, rank) -- every
//                TP rank draws the same token from the same candidates without communicating.
// Ties: lower vocabulary index first (lax.top_k order).
#include "common.h"
#include "launchers.h"

namespace jla {

constexpr int TK_THREADS = 256, TK_E = 64, TK_CHUNK = TK_THREADS * TK_E;

JLA_DEV uint32_t fkey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
JLA_DEV float kfloat(uint32_t k) { return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k); }

struct TkShared {
  uint32_t hist[256];
  uint32_t wsum[TK_THREADS / 64];
  uint32_t sel[2];
  uint32_t sk[64];  // merge: compacted survivors
  int32_t si[64];
  uint32_t ck[TK_THREADS];  // chunk: prefiltered candidates (key, element index), in element order
  int32_t cj[TK_THREADS];
  uint32_t total;
};

// Block-wide radix select over TK_E keys per thread: T = the K-th largest key; need_eq = how many
// keys equal to T are part of the top K (all keys > T are). Requires K <= number of keys.
// last_shift 16: two passes only, T = the K-th largest key with its low 16 bits cleared (a lower bound with at least K
// keys >= T; need_eq is then meaningless).
template <int E>
JLA_DEV void radix_select(const uint32_t (&key)[E], int K, TkShared& sh, uint32_t& T, int& need_eq,
                          int last_shift = 0) {
  uint32_t prefix = 0, mask = 0;
  int kr = K;
  for (int shift = 24; shift >= last_shift; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += TK_THREADS) sh.hist[i] = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < E; ++j)
      if ((key[j] & mask) == prefix) atomicAdd(&sh.hist[(key[j] >> shift) & 255u], 1u);
    __syncthreads();
    if (threadIdx.x < 64) {
      const int l = threadIdx.x;
      uint32_t c[4], s = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // lane l owns bins 255-4l .. 252-4l (descending)
        c[q] = sh.hist[255 - 4 * l - q];
        s += c[q];
      }
      uint32_t incl = s;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if (l >= o) incl += t;
      }
      uint32_t above = incl - s;
      if (above < (uint32_t)kr && (uint32_t)kr <= incl) {  // exactly one lane
        for (int q = 0; q < 4; ++q) {
          if ((uint32_t)kr <= above + c[q]) {
            sh.sel[0] = 255 - 4 * l - q;
            sh.sel[1] = above;
            break;
          }
          above += c[q];
        }
      }
    }
    __syncthreads();
    prefix |= sh.sel[0] << shift;
    mask |= 255u << shift;
    kr -= (int)sh.sel[1];
    __syncthreads();
  }
  T = prefix;
  need_eq = kr;
}

// exclusive block scan of one uint32 per thread (256 threads)
JLA_DEV uint32_t block_excl_scan(uint32_t v, TkShared& sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) sh.wsum[w] = incl;
  __syncthreads();
  uint32_t base = 0;
  for (int i = 0; i < w; ++i) base += sh.wsum[i];
  __syncthreads();
  return base + incl - v;
}

// Emit exactly K (key, index) pairs: keys > T in thread-major order, then the first need_eq keys == T.
template <int E, typename F>
JLA_DEV void emit_topk(const uint32_t (&key)[E], uint32_t T, int need_eq, int K, TkShared& sh, F&& put) {
  uint32_t ngt = 0, neq = 0;
#pragma unroll
  for (int j = 0; j < E; ++j) {
    ngt += key[j] > T;
    neq += key[j] == T;
  }
  const uint32_t ex = block_excl_scan((ngt << 16) | neq, sh);
  int gpos = ex >> 16, epos = ex & 0xffff;
  const int count_gt = K - need_eq;
#pragma unroll
  for (int j = 0; j < E; ++j) {
    if (key[j] > T) {
      put(gpos++, j);
    } else if (key[j] == T) {
      if (epos < need_eq) put(count_gt + epos, j);
      ++epos;
    }
  }
}

// Exact top K of the block's TK_CHUNK keys (thread t holds elements base .. base + TK_E - 1; key 0 = padding past
// n_valid), calling put(slot, key, element) once per slot 0..K-1 (ties at the threshold keep the lowest elements).
// Prefilter: T0 = the K-th largest of the 256 per-thread maxima (bound_shift 16: its top 16 bits). At least K keys are >= T0, so the top
// K are all >= T0; on logits only ~K keys survive, and the exact select runs on the survivors, one per thread (256
// LDS-histogram adds per radix pass instead of TK_CHUNK that pile onto the few hot exponent bins). More survivors
// than threads (flat, tied or clustered keys): the full TK_E-keys-per-thread select.
template <int E, typename F>
JLA_DEV void select_topk(const uint32_t (&key)[E], int base, int n_valid, int K, TkShared& sh, F&& put,
                         int bound_shift = 0) {
  uint32_t tmax = 0;
#pragma unroll
  for (int j = 0; j < E; ++j) tmax = max(tmax, key[j]);
  uint32_t T0;
  int ne0;
  {
    const uint32_t k1[1] = {tmax};
    radix_select(k1, K, sh, T0, ne0, bound_shift);  // a bound is enough
  }
  uint32_t ns = 0;
#pragma unroll
  for (int j = 0; j < E; ++j) ns += key[j] >= T0;
  const uint32_t pos = block_excl_scan(ns, sh);
  if (threadIdx.x == TK_THREADS - 1) sh.total = pos + ns;
  __syncthreads();
  const uint32_t S = sh.total;
  uint32_t T;
  int need_eq;
  if (S <= (uint32_t)TK_THREADS) {
    uint32_t r = pos;
#pragma unroll
    for (int j = 0; j < E; ++j)
      if (key[j] >= T0) {  // compacted in element order (thread-major, j ascending): ties keep index order
        sh.ck[r] = key[j];
        sh.cj[r] = base + j;
        ++r;
      }
    __syncthreads();
    const bool have = threadIdx.x < S;
    const uint32_t k1[1] = {have ? sh.ck[threadIdx.x] : 0u};
    const int e1 = have ? sh.cj[threadIdx.x] : n_valid;
    radix_select(k1, K, sh, T, need_eq);
    emit_topk(k1, T, need_eq, K, sh, [&](int slot, int) { put(slot, k1[0], e1); });
    return;
  }
  radix_select(key, K, sh, T, need_eq);
  emit_topk(key, T, need_eq, K, sh, [&](int slot, int j) { put(slot, key[j], base + j); });
}

__global__ void __launch_bounds__(TK_THREADS)
    topk_chunk_kernel(const float* __restrict__ logits, int V, int K, int idx_offset, float* __restrict__ cv,
                      int32_t* __restrict__ ci) {
  __shared__ TkShared sh;
  const int b = blockIdx.y, c = blockIdx.x, nch = gridDim.x;
  const int base = c * TK_CHUNK + threadIdx.x * TK_E;
  const float* x = logits + (size_t)b * V;
  uint32_t key[TK_E];
  if ((V & 3) == 0 && base + TK_E <= V) {
#pragma unroll
    for (int q = 0; q < TK_E / 4; ++q) {
      const float4 v = reinterpret_cast<const float4*>(x + base)[q];
      key[4 * q] = fkey(v.x);
      key[4 * q + 1] = fkey(v.y);
      key[4 * q + 2] = fkey(v.z);
      key[4 * q + 3] = fkey(v.w);
    }
  } else {
#pragma unroll
    for (int j = 0; j < TK_E; ++j) key[j] = base + j < V ? fkey(x[base + j]) : 0u;  // 0 < key(-inf)
  }
  float* ov = cv + ((size_t)b * nch + c) * K;
  int32_t* oi = ci + ((size_t)b * nch + c) * K;
  // logits: the top 16 bits (sign, exponent, 7 mantissa bits) of the bound admit ~K survivors; two radix passes saved
  select_topk(key, base, V, K, sh, [&](int slot, uint32_t k, int e) {
    const bool valid = e < V;
    ov[slot] = valid ? kfloat(k) : -INFINITY;
    oi[slot] = valid ? idx_offset + e : 0x7fffffff;
  }, 16);
}

JLA_DEV uint4 philox4x32_10(uint4 ctr, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * ctr.x, hi0 = __umulhi(0xD2511F53u, ctr.x);
    const uint32_t lo1 = 0xCD9E8D57u * ctr.z, hi1 = __umulhi(0xCD9E8D57u, ctr.z);
    ctr = make_uint4(hi1 ^ ctr.y ^ k.x, lo1, hi0 ^ ctr.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return ctr;
}

// mode 0: write the sorted top-K (out_v/out_i [B, K]); mode 1: sample one token per row into nxt[B].
// E candidates per thread: the smallest that covers C, so the candidates spread over most threads and the
// per-thread-maximum prefilter of select_topk compacts them (with TK_E per thread, 16 chunks x 50 candidates sat
// in 25 threads and every merge fell back to the full select)
template <int E>
__global__ void __launch_bounds__(TK_THREADS)
    topk_merge_kernel(const float* __restrict__ cv, const int32_t* __restrict__ ci, int C, int K, int mode,
                      float* __restrict__ out_v, int32_t* __restrict__ out_i, int32_t* __restrict__ nxt,
                      float inv_temp, float top_p, uint32_t seed_lo, uint32_t seed_hi,
                      const int32_t* __restrict__ step) {
  __shared__ TkShared sh;
  const int b = blockIdx.x;
  const int base = threadIdx.x * E;
  uint32_t key[E];
#pragma unroll
  for (int j = 0; j < E; ++j) key[j] = base + j < C ? fkey(cv[(size_t)b * C + base + j]) : 0u;
  select_topk(key, base, C, K, sh, [&](int slot, uint32_t k, int e) {
    sh.sk[slot] = k;
    sh.si[slot] = e < C ? ci[(size_t)b * C + e] : 0x7fffffff;
  });
  __syncthreads();
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  // composite sort key: value descending, then index ascending
  uint64_t v = lane < K ? ((uint64_t)sh.sk[lane] << 32) | (uint32_t)(0x7fffffff - sh.si[lane]) : 0ull;
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const uint32_t lo = __shfl_xor((uint32_t)v, j, 64), hi = __shfl_xor((uint32_t)(v >> 32), j, 64);
      const uint64_t o = ((uint64_t)hi << 32) | lo;
      const bool desc = (lane & k) == 0;  // final k = 64: whole wave descending
      const bool lower = (lane & j) == 0;
      const bool take_max = desc == lower;
      v = take_max ? (o > v ? o : v) : (o < v ? o : v);
    }
  }
  const float val = lane < K ? kfloat((uint32_t)(v >> 32)) : -INFINITY;
  const int32_t idx = lane < K ? 0x7fffffff - (int32_t)(uint32_t)v : 0x7fffffff;
  if (mode == 0) {
    if (lane < K) {
      out_v[(size_t)b * K + lane] = val;
      out_i[(size_t)b * K + lane] = idx;
    }
    return;
  }
  // temperature -> softmax over the survivors -> top-p keep mask
  const float l = lane < K ? val * inv_temp : -INFINITY;
  const float mx = __shfl(l, 0, 64);  // sorted: lane 0 holds the max
  float p = lane < K ? __expf(l - mx) : 0.f;
  float tot = p;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
  p /= tot;
  float incl = p;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  const bool keep = lane < K && (lane == 0 || (incl - p) < top_p);
  // Gumbel-max with Philox(seed; counter = (lane, row, step, 0))
  const uint4 r = philox4x32_10(make_uint4((uint32_t)lane, (uint32_t)b, (uint32_t)step[0], 0u),
                                make_uint2(seed_lo, seed_hi));
  const float u = ((float)(r.x >> 8) + 0.5f) * (1.0f / 16777216.0f);
  const float g = -__logf(-__logf(u));
  float score = keep ? l + g : -INFINITY;
  int best = lane;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float os = __shfl_xor(score, o, 64);
    const int ob = __shfl_xor(best, o, 64);
    if (os > score || (os == score && ob < best)) {
      score = os;
      best = ob;
    }
  }
  const int32_t tok = __shfl(idx, best, 64);
  if (lane == 0) nxt[b] = tok;
}

int topk_chunks(int V) { return (V + TK_CHUNK - 1) / TK_CHUNK; }

int topk_chunk(const float* logits, int B, int V, int K, int idx_offset, float* cv, int32_t* ci, hipStream_t s) {
  if (B <= 0) return 0;
  if (K < 1 || K > 64 || K > V) return -1;
  dim3 grid(topk_chunks(V), B);
  topk_chunk_kernel<<<grid, TK_THREADS, 0, s>>>(logits, V, K, idx_offset, cv, ci);
  JLA_CHECK_LAUNCH();
  return 0;
}

int topk_merge(const float* cv, const int32_t* ci, int B, int C, int K, int mode, float* out_v, int32_t* out_i,
               int32_t* nxt, float temperature, float top_p, uint64_t seed, const int32_t* step, hipStream_t s) {
  if (B <= 0) return 0;
  if (K < 1 || K > 64 || K > C || C > TK_CHUNK) return -1;
  if (mode == 1 && (!nxt || !step || !(temperature > 0.f))) return -2;
#define JLA_TKM(E)                                                                                          \
  topk_merge_kernel<E><<<B, TK_THREADS, 0, s>>>(cv, ci, C, K, mode, out_v, out_i, nxt, 1.0f / temperature, top_p, \
                                                (uint32_t)seed, (uint32_t)(seed >> 32), step)
  if (C <= 4 * TK_THREADS)
    JLA_TKM(4);
  else if (C <= 8 * TK_THREADS)
    JLA_TKM(8);
  else if (C <= 16 * TK_THREADS)
    JLA_TKM(16);
  else
    JLA_TKM(TK_E);
#undef JLA_TKM
  JLA_CHECK_LAUNCH();
  return 0;
}

}  // namespace jla
