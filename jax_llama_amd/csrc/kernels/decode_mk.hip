// Persistent decode step: every layer of one decode token (M <= 4 rows) in ONE launch.
//
// Why: at batch 1..4 a layer is five short kernels (qkv + RoPE/KV write, attention, wo + residual, w1|w3 + SwiGLU,
// w2 + residual) and each launch pays ~3-4 us of fill and drain around ~5-36 us of weight streaming
// (profiles/r3_decode_b1_step_sequence.txt: 88 us per Llama-3-8B layer against a 69 us HBM floor). Here one
// workgroup per CU walks the phases of every layer, separated by device-wide phase barriers, and -- the point of the
// design -- each wave issues the first MK_U weight loads of its NEXT phase before it waits at the barrier: weights do
// not depend on activations, so the weight stream overlaps the dependency wait instead of starting after it.
//
// GEMV phases (W packed [N/16][K/32][64 lanes x 16 B], common.h): the N/16 x K/32 fragment grid is one contiguous
// run in memory (tile-major). Wave gw of the P active waves streams fragments [W*gw/P, W*(gw+1)/P) of it -- the same
// bytes for every wave, one contiguous run each -- through a register ring of MK_U loads, with the x rows of the
// phase staged once per workgroup in LDS (whole K, M <= 4 rows). A run crosses at most MK_NSEG tiles; a tile whose
// whole K one wave streamed runs its epilogue directly, the others publish their 16 x 16 fp32 partial (write-through
// sc1 stores), take the tile's (SwiGLU: the gate/up pair's) agent-scope ticket, and the last arriver sums the
// partials in wave (= K) order -- deterministic -- and runs the epilogue: RoPE + q / KV-cache write, residual add +
// bf16 mirror + the per-16-column sums of squares of the new residual (the next RMSNorm statistic), or SwiGLU.
// Attention phase: (row, kv head, 64-key split) items over the workgroups; per split the K/V rows are loaded at once,
// scores by v_dot2, a per-wave softmax, one LDS merge of the 8 waves, (m, l, o) published with sc1 stores, and the
// last arriver of the (row, kv head) merges the splits in split order.
//
// Memory model: every value one workgroup writes and another reads within the launch (activations, partials, the
// new KV row, the norm statistic) is stored write-through (sc1) after which the writer waits vmcnt(0), and read with
// sc1 loads; counters are agent-scope atomics (the split-K ticket recipe of cdna_hip_programming.md Guideline 16,
// here also for the phase barrier). Co-residency: grid = one 512-thread workgroup per CU with ~144 KiB of LDS (one
// per CU fits), launched on an otherwise idle stream position; a barrier that has not completed after ~2^22 polls
// records the phase in the error word and lets the wave go on (wrong results, never a hang).
//
// Reference ops: jax_llama/model.py:383-398 (block), :210 / :294 / :338 (projections), :58-92 (RoPE),
// :169-199 (cache write), :236-291 (masked softmax attention), :28-48 (RMSNorm).
#include "common.h"
#include "launchers.h"

namespace jla {

constexpr int MK_NW = 8, MK_THREADS = MK_NW * 64;
constexpr int MK_U = 8;                 // weight ring: k-steps in flight per wave (8 x 1 KiB per wave)
constexpr int MK_NSEG = 3;              // tiles one wave's run may touch
constexpr int MK_MAXM = 4;              // rows
constexpr int MK_MINRUN = 8;            // fewest k-steps per active wave (tiny phases use fewer waves)
constexpr int MK_X_BYTES = 144 * 1024;  // x staging (M rows x K bf16, row pitch 2K + 16)
constexpr int MK_DH = 128;
constexpr int MK_KPG = 2;                         // keys per 16-lane group per attention split
constexpr int MK_CH = MK_NW * 4 * MK_KPG;         // keys per attention chunk (64)
constexpr int MK_ACH = 6;                         // chunks per attention split (384 keys: all loads issued at once)
constexpr int MK_SPK = MK_CH * MK_ACH;            // keys per attention split
constexpr unsigned MK_SC1 = 16;                   // cache-policy bits of a write-through / coherent buffer access

__device__ u32x4 g_mk_zero[64];  // zero fragment: past-the-end ring refills

JLA_DEV void mk_load(u32x4& r, const void* p) {
  asm volatile("global_load_dwordx4 %0, %1, off nt" : "+v"(r) : "v"(p) : "memory");
}
template <int N>
JLA_DEV void mk_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
JLA_DEV void mk_pin(u32x4& r) { asm volatile("" : "+v"(r)); }

JLA_DEV __amdgpu_buffer_rsrc_t mk_rsrc(const void* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)min(bytes, 0x7fffffffLL), 0x00020000);
}
JLA_DEV float ld1(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, MK_SC1));
}
JLA_DEV void st1(__amdgpu_buffer_rsrc_t r, int byte_off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, byte_off, 0, MK_SC1);
}
JLA_DEV void st_bf(__amdgpu_buffer_rsrc_t r, int byte_off, float v) {
  __builtin_amdgcn_raw_buffer_store_b16((unsigned short)f2bf(v), r, byte_off, 0, MK_SC1);
}

// Device-wide phase barrier, two levels so no counter sees more than ~32 arrivals per phase: each workgroup adds to
// its XCD group's counter (blockIdx % 8: the dispatcher's round-robin XCD), the group's last arriver adds to the
// global counter, and the overall last arriver raises every group's release flag; a workgroup polls only its own
// group's flag. Counters and flags are monotonic (phase number), each on its own 128-B line, zeroed by the host
// before the launch. The caller has drained its own write-through stores (vmcnt(0)) before anything it wants in
// flight across the barrier.
constexpr int MK_BAR_WORDS = 32 * 17;  // 8 group counters, 1 global counter, 8 release flags
JLA_DEV void mk_sync(unsigned* bar, unsigned epoch, int32_t* err) {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS reads are done before anyone restages
  __builtin_amdgcn_s_barrier();
  if (threadIdx.x == 0) {
    const int G = gridDim.x, ng = min(G, 8), x = blockIdx.x & 7;
    const unsigned nx = (unsigned)(G / 8 + (x < G % 8 ? 1 : 0));
    unsigned* flag = bar + 32 * (9 + x);
    const unsigned old = __hip_atomic_fetch_add(bar + 32 * x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == epoch * nx - 1) {  // last of its group
      const unsigned gold = __hip_atomic_fetch_add(bar + 32 * 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (gold == epoch * (unsigned)ng - 1)  // last group: release every group
        for (int i = 0; i < ng; ++i)
          __hip_atomic_store(bar + 32 * (9 + i), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    int spins = 0;
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < epoch) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1 << 22)) {
        __hip_atomic_store(err, (int)epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

struct MkLayer {
  const u32x4* wqkv;  // [(H + 2 Hkv) Dh / 16][D / 32][64], attention_norm folded in
  const u32x4* wo;    // [D / 16][H Dh / 32][64]
  const u32x4* wgu;   // [2F / 16][D / 32][64], gate / up tiles interleaved, ffn_norm folded in
  const u32x4* wdown; // [D / 16][F / 32][64]
  bf16_t* kc;         // [B][Hkv][T][Dh] of this layer
  bf16_t* vc;
};

struct MkArgs {
  const MkLayer* layers;
  int L, M, D, H, Hkv, F, T;
  float eps, scale;        // RMSNorm eps, 1 / sqrt(Dh)
  float* h;                // [M][D] fp32 residual
  bf16_t* hb;              // [M][D] its bf16 mirror (the next projection's A operand)
  bf16_t* q;               // [M][H Dh] rotated queries
  bf16_t* att;             // [M][H Dh] attention output
  bf16_t* act;             // [M][F] SwiGLU output
  float* ssq;              // [D / 16][4] per-16-column sums of squares of hb (RMSNorm statistic)
  const float2* rope;      // [rope_len][Dh / 2] (cos, sin)
  int rope_len;
  const int32_t* positions;  // [M]
  const int32_t* slot;       // device int32[1]: cache slot of this token
  const int32_t* kv_start;   // [M]: first valid key (left padding)
  float* slab;             // [grid * MK_NW][MK_NSEG][64][4] partial tiles
  int32_t* tickets;        // [max groups][32] (one per 128-B line), zero-initialised once, self-resetting
  unsigned* bar;           // phase-barrier counter, zeroed before every launch
  int32_t* err;            // barrier timeout -> phase tag
  float* aws;              // attention partials [M][Hkv][max_splits][REP][132]
  int32_t* atk;            // [M][Hkv] attention tickets (self-resetting)
  int max_splits;
  int prefetch_late;          // A/B: 1 = issue the ring prologue after the phase barrier instead of before
  unsigned long long* trace;  // optional [MK_TRACE_PH][MK_TRACE_EV][grid] s_memrealtime stamps (100 MHz), else null
};

// the first two layers, per wave (lane 0); events: entry, released, ready, streamed, done
constexpr int MK_TRACE_PH = 10, MK_TRACE_EV = 5;
JLA_DEV void mk_mark(const MkArgs& a, unsigned epoch, int ev) {
  const int ph = (int)epoch - 1;
  if (a.trace != nullptr && ph < MK_TRACE_PH && (threadIdx.x & 63) == 0)
    a.trace[((ph * MK_TRACE_EV + ev) * gridDim.x + blockIdx.x) * MK_NW + (threadIdx.x >> 6)] =
        __builtin_amdgcn_s_memrealtime();
}

// Run bounds in double precision: a 64-bit integer division is a ~100-instruction software routine (the last
// arriver evaluates these per contributor); the operands stay below 2^33 and the divisor below 2^13, so a
// non-integral quotient sits >= 2^-13 from the next integer, far above the double rounding error (exact floors).
JLA_DEV long long mk_lo(int w, long long W, int P) { return (long long)floor((double)W * (double)w / (double)P); }
JLA_DEV int mk_owner(long long it, long long W, int P) {
  return (int)floor(((double)(it + 1) * (double)P - 1.0) / (double)W);
}

// ---- one GEMV phase: y = epilogue([inv_rms *] x @ W^T), N / 16 tiles x K / 32 k-steps over the active waves
template <int MODE>
__device__ __attribute__((noinline)) void mk_gemv(const MkArgs& a, const MkLayer& ly, const u32x4* __restrict__ W, int N,
                                                  int K, const bf16_t* x, bool rms, unsigned epoch, char* lds,
                                                  float* inv_s) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int KS = K >> 5, NT = N >> 4;
  const long long Wt = (long long)NT * KS;
  const int GW = gridDim.x * MK_NW;
  const int P = (int)min((long long)GW, max(1LL, Wt / MK_MINRUN));
  const int gw = blockIdx.x * MK_NW + w;
  const int lo = gw < P ? (int)mk_lo(gw, Wt, P) : 0, hi = gw < P ? (int)mk_lo(gw + 1, Wt, P) : 0;

  // ring prologue: this wave's first MK_U fragments, issued BEFORE the barrier (no dependence on activations)
  u32x4 ring[MK_U];
  const u32x4* zf = g_mk_zero + lane;
  const u32x4* wp = W + lane;
  // (A/B: prefetch_late issues them after the barrier instead; one code path either way)
  const bool late = a.prefetch_late != 0;
  if (late) {
    mk_mark(a, epoch, 0);
    mk_sync(a.bar, epoch, a.err);
    mk_mark(a, epoch, 1);
  }
#pragma unroll
  for (int u = 0; u < MK_U; ++u) {
    ring[u] = u32x4{0u, 0u, 0u, 0u};
    mk_load(ring[u], lo + u < hi ? (const void*)(wp + (size_t)(lo + u) * 64) : (const void*)zf);
  }
  if (!late) {
    mk_mark(a, epoch, 0);
    mk_sync(a.bar, epoch, a.err);
    mk_mark(a, epoch, 1);
  }

  // ---- stage x [M][K] (sc1: written by other workgroups of this launch) and the norm statistic
  const int M = a.M;
  const int pitch = 2 * K + 16;  // bytes per staged row (the 16-B pad spreads rows over the banks)
  {
    const __amdgpu_buffer_rsrc_t xr = mk_rsrc(x, (long long)M * K * 2);
    const int cpr = K >> 3, chunks = M * cpr;  // 16-B chunks
    // the norm statistic's loads first (wave m < M: row m's K / 16 per-tile sums), so they share the x loads' round trip
    const int nt = K >> 4;
    const __amdgpu_buffer_rsrc_t sr = mk_rsrc(a.ssq, (long long)nt * 16);
    float sv[8];
    const bool do_rms = rms && w < M;
#pragma unroll
    for (int e = 0; e < 8; ++e) sv[e] = do_rms ? ld1(sr, (min(lane + 64 * e, nt - 1) * 4 + w) * 4) : 0.f;
    for (int c0 = threadIdx.x; c0 < chunks; c0 += 8 * MK_THREADS) {  // 8 loads in flight per thread
      u32x4 v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = min(c0 + e * MK_THREADS, chunks - 1);
        const int m = c / cpr, kc = c - m * cpr;
        v[e] = __builtin_amdgcn_raw_buffer_load_b128(xr, (m * K + 8 * kc) * 2, 0, MK_SC1);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = c0 + e * MK_THREADS;
        if (c < chunks) {
          const int m = c / cpr, kc = c - m * cpr;
          *reinterpret_cast<u32x4*>(lds + m * pitch + 16 * kc) = v[e];
        }
      }
    }
    if (do_rms) {  // fixed order: lane-strided partials, then the wave's xor tree
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (lane + 64 * e < nt) s += sv[e];
      for (int t0 = lane + 512; t0 < nt; t0 += 64) s += ld1(sr, (t0 * 4 + w) * 4);  // (D > 8192 only)
      s = wave_sum(s);
      if (lane == 0) inv_s[w] = rsqrtf(s / (float)K + a.eps);
    }
  }
  __syncthreads();
  mk_mark(a, epoch, 2);

  // ---- stream: fragment i = (tile i / KS, k-step i % KS); the A operand is row (lane & 15) of the staged x
  const int xrow = min(lane & 15, M - 1);
  const char* xl = lds + xrow * pitch + 16 * (lane >> 4);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f}, sa0 = acc, sa1 = acc;
  int nseg = 0, k = hi > lo ? lo % KS : 0;
  for (int j0 = lo; j0 < hi; j0 += MK_U) {
#pragma unroll
    for (int u = 0; u < MK_U; ++u) {
      const int idx = j0 + u;
      mk_wait<MK_U - 1>();
      mk_pin(ring[u]);
      if (idx < hi) {
        const u32x4 af = *reinterpret_cast<const u32x4*>(xl + 64 * k);
        acc = mfma16x16x32(af, ring[u], acc);
        ++k;
        if (k == KS || idx + 1 == hi) {  // end of a tile segment (wave-uniform, rare)
          if (nseg == 0) sa0 = acc;
          else if (nseg == 1) sa1 = acc;
          ++nseg;
          if (idx + 1 < hi) acc = f32x4{0.f, 0.f, 0.f, 0.f};
          if (k == KS) k = 0;
        }
      }
      const int nx = idx + MK_U;
      mk_load(ring[u], nx < hi ? (const void*)(wp + (size_t)nx * 64) : (const void*)zf);
    }
  }
  mk_wait<0>();
#pragma unroll
  for (int u = 0; u < MK_U; ++u) mk_pin(ring[u]);
  mk_mark(a, epoch, 3);

  // ---- epilogues. Accumulator layout: lane holds rows 4 (lane >> 4) + i, column lane & 15 (M <= 4: lanes 0..15)
  const int c = lane & 15, r0 = 4 * (lane >> 4);
  const __amdgpu_buffer_rsrc_t slr = mk_rsrc(a.slab, (long long)GW * MK_NSEG * 1024);
  auto scale_rows = [&](f32x4 v) {
    if (rms) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] *= inv_s[min(r0 + i, MK_MAXM - 1)];
    }
    return v;
  };
  // the epilogue of one finished tile group (sums already in K order)
  auto epilogue = [&](int t, f32x4 v0, f32x4 v1) {
    if constexpr (MODE == MODE_RESIDUAL) {
      const __amdgpu_buffer_rsrc_t hr = mk_rsrc(a.h, (long long)M * N * 4);
      const __amdgpu_buffer_rsrc_t br = mk_rsrc(a.hb, (long long)M * N * 2);
      const __amdgpu_buffer_rsrc_t qr = mk_rsrc(a.ssq, (long long)NT * 16);
      const int col = t * 16 + c;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = r0 + i;
        float sq = 0.f;
        if (m < M) {
          const float nv = ld1(hr, (m * N + col) * 4) + v0[i];
          st1(hr, (m * N + col) * 4, nv);
          st_bf(br, (m * N + col) * 2, nv);
          const float bv = bf2f(f2bf(nv));
          sq = bv * bv;
        }
        sq = row16_sum(sq);
        if (m < M && c == 0) st1(qr, (t * 4 + m) * 4, sq);
      }
    } else if constexpr (MODE == MODE_SWIGLU) {
      const __amdgpu_buffer_rsrc_t ar = mk_rsrc(a.act, (long long)M * (N >> 1) * 2);
      v0 = scale_rows(v0);
      v1 = scale_rows(v1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = r0 + i;
        if (m < M) st_bf(ar, (m * (N >> 1) + (t >> 1) * 16 + c) * 2, silu(v0[i]) * v1[i]);
      }
    } else {  // MODE_QKV
      v0 = scale_rows(v0);
      const int Dq = a.H * MK_DH;
      const int slot = a.slot[0];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = r0 + i;
        const float v = v0[i];
        const float pv = __shfl_xor(v, 1, 64);  // RoPE partner column (d ^ 1) lives in lane ^ 1
        if (m < M) {
          const int col = t * 16 + c;
          const int head = col / MK_DH, d = col - head * MK_DH;
          float r = v;
          if (head < a.H + a.Hkv) {
            int pos = a.positions[m];
            pos = pos < 0 ? 0 : (pos >= a.rope_len ? a.rope_len - 1 : pos);
            const float2 cs = a.rope[(size_t)pos * (MK_DH >> 1) + (d >> 1)];
            r = (d & 1) ? (pv * cs.y + v * cs.x) : (v * cs.x - pv * cs.y);
          }
          if (head < a.H) {
            st_bf(mk_rsrc(a.q, (long long)M * Dq * 2), (m * Dq + col) * 2, r);
          } else if (slot < a.T) {
            const bool is_k = head < a.H + a.Hkv;
            const int kh = is_k ? head - a.H : head - a.H - a.Hkv;
            bf16_t* cache = is_k ? ly.kc : ly.vc;
            const int off = ((m * a.Hkv + kh) * a.T + slot) * MK_DH + d;
            st_bf(mk_rsrc(cache, (long long)M * a.Hkv * a.T * MK_DH * 2), off * 2, r);
          }
        }
      }
    }
  };

  // Batched over the run's (<= MK_NSEG) segments so the round trips overlap: (1) direct epilogues of whole tiles and
  // the write-through partials of the others, one vmcnt(0); (2) every ticket add issued before any result is used;
  // (3) each group this wave completed: all contributors' partials loaded together, summed in wave (= K) order.
  const int t_first = hi > lo ? lo / KS : 0;
  auto seg_v = [&](int s) { return s == 0 ? sa0 : (s == 1 ? sa1 : acc); };
  auto is_direct = [&](int s) {
    const int kb = s == 0 ? lo % KS : 0, ke = s == nseg - 1 ? (hi - 1) % KS + 1 : KS;
    return MODE != MODE_SWIGLU && kb == 0 && ke == KS;
  };
  int pend = 0;  // bit s: segment s published a partial
  for (int s = 0; s < nseg; ++s) {
    if (is_direct(s)) {
      const f32x4 v = seg_v(s);
      epilogue(t_first + s, v, v);
    } else {
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, seg_v(s)), slr,
                                             ((gw * MK_NSEG + s) * 64 + lane) * 16, 0, MK_SC1);
      pend |= 1 << s;
    }
  }
  if (pend) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    auto group_of = [&](int s) { return MODE == MODE_SWIGLU ? ((t_first + s) >> 1) : (t_first + s); };
    auto count_of = [&](int g) {
      const int g0 = MODE == MODE_SWIGLU ? 2 * g : g, gn = MODE == MODE_SWIGLU ? 2 : 1;
      int count = 0;
      for (int q = 0; q < gn; ++q) {
        const long long b0 = (long long)(g0 + q) * KS;
        count += mk_owner(b0 + KS - 1, Wt, P) - mk_owner(b0, Wt, P) + 1;
      }
      return count;
    };
    int lastm = 0;
    if (lane == 0) {
      int prev[MK_NSEG];
#pragma unroll
      for (int s = 0; s < MK_NSEG; ++s)
        if (pend >> s & 1)
          prev[s] = __hip_atomic_fetch_add(a.tickets + 32 * group_of(s), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int s = 0; s < MK_NSEG; ++s)
        if ((pend >> s & 1) && prev[s] == count_of(group_of(s)) - 1) {
          lastm |= 1 << s;
          __hip_atomic_store(a.tickets + 32 * group_of(s), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    lastm = __shfl(lastm, 0, 64);
    for (int s = 0; s < nseg; ++s) {
      if (!(lastm >> s & 1)) continue;
      const int g = group_of(s);
      const int g0 = MODE == MODE_SWIGLU ? 2 * g : g, gn = MODE == MODE_SWIGLU ? 2 : 1;
      f32x4 sum[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        sum[q] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (q >= gn) continue;
        const int tt = g0 + q;
        const long long b0 = (long long)tt * KS;
        const int cw0 = mk_owner(b0, Wt, P), cw1 = mk_owner(b0 + KS - 1, Wt, P);
        for (int e0 = 0; cw0 + e0 <= cw1; e0 += 12) {  // 12 contributors' loads in flight per round
          u32x4 part[12];
#pragma unroll
          for (int e = 0; e < 12; ++e) {
            const int cw = min(cw0 + e0 + e, cw1);
            const int sidx = tt - (int)(mk_lo(cw, Wt, P) / KS);
            part[e] = __builtin_amdgcn_raw_buffer_load_b128(slr, ((cw * MK_NSEG + sidx) * 64 + lane) * 16, 0, MK_SC1);
          }
#pragma unroll
          for (int e = 0; e < 12; ++e)
            if (cw0 + e0 + e <= cw1) sum[q] += __builtin_bit_cast(f32x4, part[e]);
        }
      }
      epilogue(g0, sum[0], sum[1]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this phase's write-through stores have landed
  mk_mark(a, epoch, 4);
}

// ---- attention phase: (row, kv head, 64-key split) items; REP query heads share each K / V row
template <int REP>
__device__ __forceinline__ void mk_attn(const MkArgs& a, const MkLayer& ly, unsigned epoch, char* lds,
                                                  int* flag_s) {
  constexpr int HS = MK_DH + 4, PS = REP * HS;
  float (*sm_m)[REP] = reinterpret_cast<float (*)[REP]>(lds);
  float (*sm_l)[REP] = reinterpret_cast<float (*)[REP]>(lds + MK_NW * REP * 4);
  float (*sm_o)[REP][MK_DH] = reinterpret_cast<float (*)[REP][MK_DH]>(lds + 2 * MK_NW * REP * 4);
  mk_mark(a, epoch, 0);
  mk_sync(a.bar, epoch, a.err);
  mk_mark(a, epoch, 1);

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int slot = a.slot[0];
  const int hi = min(slot + 1, a.T);
  const int nsp = min((hi + MK_SPK - 1) / MK_SPK, a.max_splits);
  const int Dq = a.H * MK_DH;
  const int items = a.M * a.Hkv * nsp;
  const __amdgpu_buffer_rsrc_t qr = mk_rsrc(a.q, (long long)a.M * Dq * 2);
  const __amdgpu_buffer_rsrc_t orr = mk_rsrc(a.att, (long long)a.M * Dq * 2);
  for (int item = blockIdx.x; item < items; item += gridDim.x) {
    const int split = item % nsp, pair = item / nsp;
    const int kvh = pair % a.Hkv, b = pair / a.Hkv;
    const int lo = a.kv_start[b];
    const int s_lo = lo / MK_SPK, s_hi = hi > lo ? (hi + MK_SPK - 1) / MK_SPK : s_lo;
    const int n_act = s_hi - s_lo;
    const int h0 = kvh * REP;
    auto store_out = [&](int hh, int d, const float* v) {
      const int off = (b * Dq + (h0 + hh) * MK_DH + d) * 2;
      __builtin_amdgcn_raw_buffer_store_b64(u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])}, orr, off, 0, MK_SC1);
    };
    if (n_act <= 0) {
      if (split == 0)
        for (int it = threadIdx.x; it < REP * 32; it += MK_THREADS) {
          const float z[4] = {0.f, 0.f, 0.f, 0.f};
          store_out(it >> 5, 4 * (it & 31), z);
        }
      continue;
    }
    if (split < s_lo || split >= s_hi) continue;  // (workgroup-uniform)

    const int c0 = split * MK_SPK;
    const long long cache_bytes = (long long)MK_DH * 2 * a.T;
    const size_t head = ((size_t)b * a.Hkv + kvh) * a.T * MK_DH;
    const __amdgpu_buffer_rsrc_t kr_ = mk_rsrc(ly.kc + head, cache_bytes), vr_ = mk_rsrc(ly.vc + head, cache_bytes);
    // every K / V row of the split at once (one memory round trip); key of (chunk c, r) for this lane group:
    // c0 + 64 c + 32 r + 4 w + g (rows past the valid range re-read a valid one and are masked)
    const int nch = min(MK_ACH, (hi - c0 + MK_CH - 1) / MK_CH);  // chunks of this split holding keys
    u32x4 kr[MK_ACH][MK_KPG], vr[MK_ACH][MK_KPG], qv[REP];
#pragma unroll
    for (int c = 0; c < MK_ACH; ++c)
#pragma unroll
      for (int r = 0; r < MK_KPG; ++r) {
        const int jc = min(max(c0 + MK_CH * c + 4 * MK_NW * r + 4 * w + g, lo), hi - 1);
        if (c < nch) {
          kr[c][r] = __builtin_amdgcn_raw_buffer_load_b128(kr_, (jc * MK_DH + 8 * li) * 2, 0, MK_SC1);
          vr[c][r] = __builtin_amdgcn_raw_buffer_load_b128(vr_, (jc * MK_DH + 8 * li) * 2, 0, MK_SC1);
        }
      }
#pragma unroll
    for (int hh = 0; hh < REP; ++hh)
      qv[hh] = __builtin_amdgcn_raw_buffer_load_b128(qr, (b * Dq + (h0 + hh) * MK_DH + 8 * li) * 2, 0, MK_SC1);

    // per wave and head: online softmax over the chunks -- the running max wave-uniform, (l, o) lane-partial over the
    // lane group's keys, summed over the 4 groups once at the end
#pragma unroll
    for (int hh = 0; hh < REP; ++hh) {
      float mr = -INFINITY, l = 0.f, o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < MK_ACH; ++c) {
        if (c >= nch) continue;  // (wave-uniform)
        float sc[MK_KPG];
        float mx = -INFINITY;
#pragma unroll
        for (int r = 0; r < MK_KPG; ++r) {
          const int j = c0 + MK_CH * c + 4 * MK_NW * r + 4 * w + g;
          const float d = row16_sum(dot8_bf16(qv[hh], kr[c][r], 0.f)) * a.scale;
          sc[r] = (j >= lo && j < hi) ? d : -INFINITY;
          mx = fmaxf(mx, sc[r]);
        }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        if (mx == -INFINITY) continue;  // no valid key in this chunk (wave-uniform)
        const float mn = fmaxf(mr, mx);
        const float al = mr == -INFINITY ? 0.f : __expf(mr - mn);
        l *= al;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] *= al;
        mr = mn;
#pragma unroll
        for (int r = 0; r < MK_KPG; ++r) {
          const float p = sc[r] == -INFINITY ? 0.f : __expf(sc[r] - mn);
          l += p;
          float vf[8];
          unpack8(vr[c][r], vf);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] += p * vf[e];
        }
      }
      const float mx = mr;
      l += __shfl_xor(l, 16, 64);
      l += __shfl_xor(l, 32, 64);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        o[e] += __shfl_xor(o[e], 16, 64);
        o[e] += __shfl_xor(o[e], 32, 64);
      }
      if (g == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) sm_o[w][hh][8 * li + e] = o[e];
        if (li == 0) {
          sm_m[w][hh] = mx;
          sm_l[w][hh] = l;
        }
      }
    }
    __syncthreads();

    const __amdgpu_buffer_rsrc_t wr = mk_rsrc(a.aws + ((size_t)b * a.Hkv + kvh) * a.max_splits * PS,
                                              (long long)a.max_splits * PS * 4);
    for (int it = threadIdx.x; it < REP * 32; it += MK_THREADS) {
      const int hh = it >> 5, d = 4 * (it & 31);
      float Mx = -INFINITY;
#pragma unroll
      for (int ww = 0; ww < MK_NW; ++ww) Mx = fmaxf(Mx, sm_m[ww][hh]);
      float num[4] = {0.f, 0.f, 0.f, 0.f}, den = 0.f;
      if (Mx != -INFINITY) {
#pragma unroll
        for (int ww = 0; ww < MK_NW; ++ww) {
          const float mw = sm_m[ww][hh];
          const float f = mw == -INFINITY ? 0.f : __expf(mw - Mx);
          den += f * sm_l[ww][hh];
#pragma unroll
          for (int e = 0; e < 4; ++e) num[e] += f * sm_o[ww][hh][d + e];
        }
      }
      if (n_act == 1) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = den > 0.f ? num[e] / den : 0.f;
        store_out(hh, d, v);
      } else {
        const int off = (split * PS + hh * HS) * 4;
        __builtin_amdgcn_raw_buffer_store_b128(
            u32x4{__float_as_uint(num[0]), __float_as_uint(num[1]), __float_as_uint(num[2]), __float_as_uint(num[3])},
            wr, off + (4 + d) * 4, 0, MK_SC1);
        if (d == 0)
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(Mx), __float_as_uint(den), 0u, 0u}, wr, off, 0,
                                                 MK_SC1);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // LDS scores consumed; every storing wave drained
    if (n_act == 1) continue;
    if (threadIdx.x == 0) {
      int32_t* tk = a.atk + 32 * ((size_t)b * a.Hkv + kvh);
      const int prev = __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == n_act - 1;
      if (last) __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag_s = last;
    }
    __syncthreads();
    const int last = *flag_s;
    __syncthreads();  // flag read before the next item rewrites it
    if (!last) continue;
    for (int it = threadIdx.x; it < REP * 32; it += MK_THREADS) {
      const int hh = it >> 5, d = 4 * (it & 31);
      float Mr = -INFINITY, Lr = 0.f, Or[4] = {0.f, 0.f, 0.f, 0.f};
      for (int s = s_lo; s < s_hi; s += 4) {
        u32x4 ml[4], ov[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int off = (min(s + u, s_hi - 1) * PS + hh * HS) * 4;
          ml[u] = __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, MK_SC1);
          ov[u] = __builtin_amdgcn_raw_buffer_load_b128(wr, off + (4 + d) * 4, 0, MK_SC1);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (s + u >= s_hi) continue;
          const float ms = __uint_as_float(ml[u][0]);
          if (ms == -INFINITY) continue;
          const float mn = fmaxf(Mr, ms);
          const float al = Mr == -INFINITY ? 0.f : __expf(Mr - mn), f = __expf(ms - mn);
          Lr = Lr * al + f * __uint_as_float(ml[u][1]);
#pragma unroll
          for (int e = 0; e < 4; ++e) Or[e] = Or[e] * al + f * __uint_as_float(ov[u][e]);
          Mr = mn;
        }
      }
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = Lr > 0.f ? Or[e] / Lr : 0.f;
      store_out(hh, d, v);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  mk_mark(a, epoch, 4);
}

template <int REP>
__global__ void __launch_bounds__(MK_THREADS, 1) decode_mk_kernel(MkArgs args) {
  __shared__ __attribute__((aligned(16))) char lds[MK_X_BYTES];
  __shared__ float inv_s[4];
  __shared__ int flag_s;
  // the phases are separate (non-inlined) functions, each with its own register allocation; they read the
  // arguments and the layer's pointers from LDS copies (a reference to the kernel argument would copy it to scratch)
  __shared__ MkArgs a;
  __shared__ MkLayer ly;
  if (threadIdx.x == 0) a = args;
  __syncthreads();
  const int Dq = a.H * MK_DH, Dkv = a.Hkv * MK_DH;
  unsigned epoch = 0;
  for (int l = 0; l < a.L; ++l) {
    if (threadIdx.x == 0) ly = a.layers[l];
    __syncthreads();
    mk_gemv<MODE_QKV>(a, ly, ly.wqkv, Dq + 2 * Dkv, a.D, a.hb, true, ++epoch, lds, inv_s);
    mk_attn<REP>(a, ly, ++epoch, lds, &flag_s);
    mk_gemv<MODE_RESIDUAL>(a, ly, ly.wo, a.D, Dq, a.att, false, ++epoch, lds, inv_s);
    mk_gemv<MODE_SWIGLU>(a, ly, ly.wgu, 2 * a.F, a.D, a.hb, true, ++epoch, lds, inv_s);
    mk_gemv<MODE_RESIDUAL>(a, ly, ly.wdown, a.D, a.F, a.act, false, ++epoch, lds, inv_s);
    __syncthreads();  // every wave is past this layer's pointers before thread 0 rewrites them
  }
}

// the first layer's norm statistic: per-16-column sums of squares of hb (same order as the residual epilogue)
__global__ void __launch_bounds__(64) decode_mk_ssq_kernel(const bf16_t* __restrict__ hb, float* __restrict__ ssq,
                                                           int M, int D) {
  const int t = blockIdx.x, lane = threadIdx.x;
  const int c = lane & 15, m = lane >> 4;
  float v = 0.f;
  if (m < M) {
    const float x = bf2f(hb[(size_t)m * D + t * 16 + c]);
    v = x * x;
  }
  v = row16_sum(v);
  if (c == 0) ssq[t * 4 + m] = m < M ? v : 0.f;
}

// ------------------------------------------------------------------------------------------------------------
static int mk_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    if (n <= 0) n = 256;
  }
  return n;
}

int decode_mk_grid() { return mk_num_cus(); }
size_t decode_mk_slab_floats() { return (size_t)mk_num_cus() * MK_NW * MK_NSEG * 256; }
int decode_mk_max_splits(int T) { return (T + MK_SPK - 1) / MK_SPK; }
int decode_mk_bar_words() { return MK_BAR_WORDS; }
int decode_mk_trace_words() { return MK_TRACE_PH * MK_TRACE_EV * mk_num_cus() * MK_NW; }

// Whether one GEMV phase fits the kernel's plan: <= MK_NSEG tiles per wave run, x rows in the LDS staging area.
static bool mk_phase_ok(int M, int N, int K, int G) {
  if ((N & 15) || (K & 31)) return false;
  const long long KS = K >> 5, Wt = (long long)(N >> 4) * KS;
  const long long P = min((long long)G * MK_NW, max(1LL, Wt / MK_MINRUN));  // as mk_gemv
  const long long per = (Wt + P - 1) / P;                               // longest run
  if ((per + KS - 1) / KS + 1 > MK_NSEG) return false;                   // tiles one run touches
  return (long long)M * (2 * K + 16) <= MK_X_BYTES;
}

int decode_mk_supported(int M, int D, int H, int Hkv, int Dh, int F) {
  if (M < 1 || M > 4 || Dh != MK_DH || H % Hkv) return 0;
  const int rep = H / Hkv;
  if (rep != 1 && rep != 2 && rep != 4 && rep != 8) return 0;
  const int G = mk_num_cus();
  const int Dq = H * Dh, Dkv = Hkv * Dh;
  return mk_phase_ok(M, Dq + 2 * Dkv, D, G) && mk_phase_ok(M, D, Dq, G) && mk_phase_ok(M, 2 * F, D, G) &&
         mk_phase_ok(M, D, F, G) && (F & 15) == 0;
}

int decode_mk(const void* layers, int L, int M, int D, int H, int Hkv, int F, int T, float eps, float* h, bf16_t* hb,
              bf16_t* q, bf16_t* att, bf16_t* act, float* ssq, const float2* rope, int rope_len,
              const int32_t* positions, const int32_t* slot, const int32_t* kv_start, float* slab, size_t slab_floats,
              int32_t* tickets, int n_tickets, unsigned* bar, int32_t* err, float* aws, size_t aws_floats, int32_t* atk,
              unsigned long long* trace, int prefetch_late, hipStream_t s) {
  if (!decode_mk_supported(M, D, H, Hkv, MK_DH, F)) return -1;
  const int rep = H / Hkv;
  const int max_splits = decode_mk_max_splits(T);
  const int NTmax = max((H + 2 * Hkv) * MK_DH, max(2 * F, D)) >> 4;
  if (slab_floats < decode_mk_slab_floats() || n_tickets < 32 * NTmax ||
      aws_floats < (size_t)M * Hkv * max_splits * rep * (MK_DH + 4))
    return -3;
  MkArgs a{};
  a.layers = static_cast<const MkLayer*>(layers);
  a.L = L;
  a.M = M;
  a.D = D;
  a.H = H;
  a.Hkv = Hkv;
  a.F = F;
  a.T = T;
  a.eps = eps;
  a.scale = 1.f / sqrtf((float)MK_DH);
  a.h = h;
  a.hb = hb;
  a.q = q;
  a.att = att;
  a.act = act;
  a.ssq = ssq;
  a.rope = rope;
  a.rope_len = rope_len;
  a.positions = positions;
  a.slot = slot;
  a.kv_start = kv_start;
  a.slab = slab;
  a.tickets = tickets;
  a.bar = bar;
  a.err = err;
  a.aws = aws;
  a.atk = atk;
  a.max_splits = max_splits;
  a.trace = trace;
  a.prefetch_late = prefetch_late;
  if (hipMemsetAsync(bar, 0, MK_BAR_WORDS * sizeof(unsigned), s) != hipSuccess) return -2;
  decode_mk_ssq_kernel<<<D / 16, 64, 0, s>>>(hb, ssq, M, D);
  JLA_CHECK_LAUNCH();
  const int G = mk_num_cus();
  switch (rep) {
    case 1: decode_mk_kernel<1><<<G, MK_THREADS, 0, s>>>(a); break;
    case 2: decode_mk_kernel<2><<<G, MK_THREADS, 0, s>>>(a); break;
    case 4: decode_mk_kernel<4><<<G, MK_THREADS, 0, s>>>(a); break;
    default: decode_mk_kernel<8><<<G, MK_THREADS, 0, s>>>(a); break;
  }
  JLA_CHECK_LAUNCH();
  return 0;
}

}  // namespace jla
