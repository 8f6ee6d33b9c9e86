// Custom xGMI collectives for decode-sized tensor-parallel messages (the
// row-parallel wo / w2 outputs, 2 per layer per token, and the vocab-parallel sampler gathers;
// reference partition.py:67,70,77 where XLA's GSPMD inserts the NCCL collectives).
//
// Memory: every rank owns ONE uncached allocation, exported by IPC handle and mapped by every peer:
//   [A: 2 parities][world slots][max_bytes]     scatter / one-shot receive slots
//   [R: 2 parities][2 * max_bytes]              two-shot fp32 result region
// plus a small uncached signal allocation: flags [CAR_BLOCKS][CAR_MAX_WORLD], then per-block barrier
// and call counters and the error word (local use only).
//
// Coherence protocol (independent of the MTYPE the importing GPU maps the peer memory with):
//   * every byte handed to a peer is stored with sc0 sc1 (system-scope write-through) and every byte
//     handed over is loaded with sc0 sc1 (system scope, bypasses the non-coherent caches);
//   * producer: payload stores -> each wave s_waitcnt vmcnt(0) -> __syncthreads -> one lane per peer
//     stores the flag (relaxed, system scope = sc0 sc1 store);
//   * consumer: one lane per peer polls its flag (relaxed system-scope load, bounded by a wall-clock
//     timeout that raises the error word instead of hanging), __syncthreads, then the payload loads.
//   No release/acquire fences, and why none is needed (gfx950 memory model, peer-mapped memory):
//   - a release fence exists to write back dirty cache lines before the flag becomes visible; here no handed-off
//     byte is ever cached dirty: the buffers are uncached allocations and every hand-off store is sc0 sc1
//     (system-scope write-through), so it leaves the CU's caches and the XCD L2 immediately;
//   - s_waitcnt vmcnt(0) after the payload stores returns only once each store is acknowledged by the memory side
//     it targets (for a peer's buffer: across xGMI), and the flag store is issued after that wait, on the same
//     path -- so a peer that reads the flag's new value reads after the payload landed;
//   - an acquire fence exists to invalidate stale cached copies before the payload loads; here every load of
//     handed-off bytes is sc0 sc1 (system scope: it bypasses the non-coherent caches), so nothing stale is read;
//   - the granule protocol (below) needs no ordering at all: data and tag travel in one 8-byte store.
//   A fence would add the slow L2 write-back and the compiler hazard where the vmcnt wait after buffer_wbl2 is
//   dropped (MI355X_MICROARCH.md). The argument is verified, not assumed, on every new set of links: before an
//   instance is used, parallel/custom_allreduce.py self_test() runs rounds of every path (granule, flag one-shot,
//   two-shot, pair gather, the GEMV-fused exchange) with rank-dependent data checked word by word on the host, and
//   any mismatch moves every rank to RCCL.
//
// Block b of every rank handles chunks c == b (mod the instance grid, d.grid) of every message, so block b only ever
// pairs with block b of its peers; barriers count per block and flags are monotonic. Every kernel maps
// chunk c to the SAME bytes of a slot -- [c * CAR_CHUNK, (c + 1) * CAR_CHUNK) of A, and
// [c * 2 * CAR_CHUNK, (c + 1) * 2 * CAR_CHUNK) of R whatever the element type -- so a block's slot bytes are
// only ever touched by that block (and the same block of the peers), whichever kernel runs. The parity
// buffers make one barrier per round enough: block b's parity slot is overwritten two of ITS calls
// later, and by then the writer has passed a block-b barrier that every peer's block b reached after
// finishing its reads of that slot. (Blocks past a message's chunk count skip the call entirely, so
// block b's parity counts block b's calls only; with the byte mapping above that is all it needs.)
// Failure: a wait that times out sets the error word; every later wait sees it and gives up at once (no
// hang, results invalid), and the host refuses further calls once it has read the error.
// Graph-capturable: all state (pointers, counters) lives in device memory.
//
// Kernels
//   car_reduce_kernel<OP, TWO_SHOT>   sum of every rank's [n] input (bf16 or fp32, fp32 accumulation
//       in rank order -> bit-identical on every rank and between one-shot and two-shot):
//         OP_SUM    out = sum
//         OP_RESID  h (fp32) += sum; hb (bf16) = h     (the residual add + bf16 mirror of the decode
//                   step, fused: the row-parallel GEMM writes only its partial)
//       one-shot: push the input into slot `rank` of every peer, barrier, sum the local slots;
//       two-shot (reduce-scatter + all-gather): chunk c is owned by rank c % world; push it to the
//       owner only, barrier, the owner sums and pushes the fp32 sum to every rank, barrier, apply OP.
//   car_pairs_kernel<MODE>    all-gather of (fp32 value, int32 index) pairs (8-byte granules):
//         MODE_ARGMAX  per row the first max in rank order (vocab-parallel greedy token)
//         MODE_TOPK    per-rank top-k candidates laid out [B][world * k] for the final merge/sample
#include "car.h"
#include "common.h"
#include "launchers.h"

namespace jla {

// chunk c -> block c % d.grid on every call (fixed mapping per instance): 63 blocks while ranks share a device, 255 with
// one rank per GPU -- a 4 MiB message (the row-parallel partial of Llama-3-70B at MP 8, B = 256) then spreads over
// every CU instead of 63 (profiles/r3_car_grid_ab.jsonl)
static_assert(CAR_GRID_MAX <= CAR_BLOCKS && CAR_GRID_SHARED <= CAR_GRID_MAX && 2 * CAR_BLOCKS * 4 + 64 <= CAR_TAIL_BYTES,
              "signal layout");
constexpr int CAR_THREADS = 256;
constexpr int CAR_CHUNK = CAR_THREADS * 16;  // input bytes per block iteration
constexpr int CAR_PAIR_CHUNK = CAR_CHUNK / 8;  // pairs per block iteration: the same slot bytes as a reduce chunk
constexpr int CAR_PAIRS_PER_THREAD = CAR_PAIR_CHUNK / CAR_THREADS;

enum { OP_SUM = 0, OP_RESID = 1 };
enum { PAIRS_ARGMAX = 0, PAIRS_TOPK = 1 };

// Per-call state of block b, in LDS: the call and barrier counters are read once at the start (uncached memory:
// every access is a memory round trip) and written back once at the end.
struct CarCalls {
  int calls, bars;
};

// Start of a call for block b: read the counters, bump the call counter (parity).
JLA_DEV int car_begin(const CarDevice& d, int b, CarCalls* st) {
  if (threadIdx.x == 0) {
    const int2 c = d.ctr[b];
    st->calls = c.x + 1;
    st->bars = c.y;
  }
  __syncthreads();
  return st->calls & 1;
}
JLA_DEV void car_end(const CarDevice& d, int b, const CarCalls* st) {
  if (threadIdx.x == 0) d.ctr[b] = make_int2(st->calls, st->bars);
}

// Barrier of block b with block b of every peer. Every wave of the block must have issued its
// hand-off stores before calling.
JLA_DEV void car_barrier(const CarDevice& d, int b, CarCalls* st) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int e = st->bars + 1;
  if (threadIdx.x < d.world) {
    __hip_atomic_store(d.sig[threadIdx.x] + b * CAR_MAX_WORLD + d.rank, e, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    const int* f = d.sig[d.rank] + b * CAR_MAX_WORLD + threadIdx.x;
    const long long t0 = (long long)wall_clock64();
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      // an earlier wait already gave up: the protocol state is out of step, do not wait again
      if (__hip_atomic_load(d.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
      if ((long long)wall_clock64() - t0 > d.timeout_ticks) {
        __hip_atomic_store(d.error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) st->bars = e;
}

// fp32 values of one 16-byte input piece (8 bf16 or 4 fp32)
template <bool BF16>
struct Piece {
  static constexpr int N = BF16 ? 8 : 4;
  float v[N];
  JLA_DEV void set(const u32x4 x) {
    if constexpr (BF16) {
      unpack8(x, v);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = __uint_as_float(x[i]);
    }
  }
  JLA_DEV void add(const u32x4 x) {
    Piece<BF16> t;
    t.set(x);
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += t.v[i];
  }
};

// Apply the op to element range [e0, e0 + N) given the fp32 sum
// hb_pack (optional, OP_RESID): packed-layout copy (common.h pack_off) of hb, rows of pack_cols elements -- the
// next projection's packed-x input on the decode path
template <int OP, bool BF16>
JLA_DEV void car_epilogue(const float* sum, long long e0, void* out, float* h, bf16_t* hb, bf16_t* hb_pack,
                          int pack_cols, bool pre, f32x4 pre0, f32x4 pre1) {
  constexpr int N = BF16 ? 8 : 4;
  if constexpr (OP == OP_SUM) {
    if constexpr (BF16) {
      *reinterpret_cast<u32x4*>(static_cast<bf16_t*>(out) + e0) = pack8(sum);
    } else {
      *reinterpret_cast<f32x4*>(static_cast<float*>(out) + e0) = f32x4{sum[0], sum[1], sum[2], sum[3]};
    }
  } else {
    float r[N];
#pragma unroll
    for (int q = 0; q < N / 4; ++q) {
      f32x4 hv = pre ? (q == 0 ? pre0 : pre1) : *reinterpret_cast<const f32x4*>(h + e0 + 4 * q);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        r[4 * q + i] = hv[i] + sum[4 * q + i];
        hv[i] = r[4 * q + i];
      }
      *reinterpret_cast<f32x4*>(h + e0 + 4 * q) = hv;
    }
    if constexpr (BF16) {
      *reinterpret_cast<u32x4*>(hb + e0) = pack8(r);
    } else {
      u32x2 p;
      p[0] = pack2bf(r[0], r[1]);
      p[1] = pack2bf(r[2], r[3]);
      *reinterpret_cast<u32x2*>(hb + e0) = p;
    }
    if (hb_pack) {
      // N consecutive elements of one row (pack_cols % 32 == 0, e0 % N == 0): 8 (or 4) contiguous packed bf16
      const int m = (int)(e0 / pack_cols), c = (int)(e0 - (long long)m * pack_cols);
      bf16_t* dst = hb_pack + pack_off(m, c, pack_cols);
      if constexpr (BF16) {
        *reinterpret_cast<u32x4*>(dst) = pack8(r);
      } else {
        u32x2 p;
        p[0] = pack2bf(r[0], r[1]);
        p[1] = pack2bf(r[2], r[3]);
        *reinterpret_cast<u32x2*>(dst) = p;
      }
    }
  }
}

template <int OP, bool BF16, bool TWO_SHOT>
__global__ void __launch_bounds__(CAR_THREADS)
    car_reduce_kernel(const char* __restrict__ in, void* __restrict__ out, float* __restrict__ h,
                      bf16_t* __restrict__ hb, long long nbytes, const CarDevice* __restrict__ dev,
                      bf16_t* __restrict__ hb_pack, int pack_cols) {
  const CarDevice& d = *dev;  // by reference: a by-value copy indexed with runtime p lives in scratch
  constexpr int ESZ = BF16 ? 2 : 4;
  constexpr int N = 16 / ESZ;
  const int b = blockIdx.x;
  const long long nchunks = (nbytes + CAR_CHUNK - 1) / CAR_CHUNK;
  if (b >= nchunks) return;
  __shared__ CarCalls st;
  // the first chunk's input (and, one-shot OP_RESID, its residual rows) are loaded before the counters come back:
  // independent of the hand-off, so their latency hides behind the counter read
  const long long off0 = (long long)b * CAR_CHUNK + (long long)threadIdx.x * 16;
  const bool have0 = off0 < nbytes;
  u32x4 in0 = {0u, 0u, 0u, 0u};
  f32x4 h0a = {0.f, 0.f, 0.f, 0.f}, h0b = {0.f, 0.f, 0.f, 0.f};
  if (have0) in0 = *reinterpret_cast<const u32x4*>(in + off0);
  if constexpr (OP == OP_RESID && !TWO_SHOT) {
    if (have0) {
      h0a = *reinterpret_cast<const f32x4*>(h + off0 / ESZ);
      if constexpr (N == 8) h0b = *reinterpret_cast<const f32x4*>(h + off0 / ESZ + 4);
    }
  }
  const int parity = car_begin(d, b, &st);
  const long long slot = d.max_bytes;
  const long long a_off = (long long)parity * d.world * slot;
  const long long r_off = 2 * (long long)d.world * slot + (long long)parity * 2 * slot;
  const __amdgpu_buffer_rsrc_t mine = rsrc(d.buf[d.rank]);

  // 1. push this rank's input: to every peer (one-shot) or to the chunk's owner (two-shot)
  for (long long c = b; c < nchunks; c += d.grid) {
    const long long off = c * CAR_CHUNK + (long long)threadIdx.x * 16;
    if (off >= nbytes) continue;
    const u32x4 v = c == b ? in0 : *reinterpret_cast<const u32x4*>(in + off);
    if (TWO_SHOT) {
      const int o = (int)(c % d.world);
      st_sys16(rsrc(d.buf[o]), a_off + (long long)d.rank * slot + off, v);
    } else {
      for (int p = 0; p < d.world; ++p) st_sys16(rsrc(d.buf[p]), a_off + (long long)d.rank * slot + off, v);
    }
  }
  car_barrier(d, b, &st);

  if (!TWO_SHOT) {
    // 2. sum the slots in rank order, apply the op
    for (long long c = b; c < nchunks; c += d.grid) {
      const long long off = c * CAR_CHUNK + (long long)threadIdx.x * 16;
      if (off >= nbytes) continue;
      Piece<BF16> acc;
      acc.set(ld_sys16(mine, a_off + off));
      for (int p = 1; p < d.world; ++p) acc.add(ld_sys16(mine, a_off + (long long)p * slot + off));
      car_epilogue<OP, BF16>(acc.v, off / ESZ, out, h, hb, hb_pack, pack_cols, OP == OP_RESID && c == b, h0a, h0b);
    }
    car_end(d, b, &st);
    return;
  }
  // 2. owner: sum its chunks in rank order, push the fp32 sum to every rank's R region
  for (long long c = b; c < nchunks; c += d.grid) {
    if ((int)(c % d.world) != d.rank) continue;
    const long long off = c * CAR_CHUNK + (long long)threadIdx.x * 16;
    if (off >= nbytes) continue;
    Piece<BF16> acc;
    acc.set(ld_sys16(mine, a_off + off));
    for (int p = 1; p < d.world; ++p) acc.add(ld_sys16(mine, a_off + (long long)p * slot + off));
    // fp32 result of element off / ESZ, in chunk c's own 2 * CAR_CHUNK bytes of R
    const long long roff = r_off + c * 2 * CAR_CHUNK + ((off - c * CAR_CHUNK) / ESZ) * 4;
#pragma unroll
    for (int q = 0; q < N / 4; ++q) {
      const u32x4 v = {__float_as_uint(acc.v[4 * q]), __float_as_uint(acc.v[4 * q + 1]),
                       __float_as_uint(acc.v[4 * q + 2]), __float_as_uint(acc.v[4 * q + 3])};
      for (int p = 0; p < d.world; ++p) st_sys16(rsrc(d.buf[p]), roff + 16 * q, v);
    }
  }
  car_barrier(d, b, &st);
  // 3. every rank: apply the op to every chunk from the gathered sums
  for (long long c = b; c < nchunks; c += d.grid) {
    const long long off = c * CAR_CHUNK + (long long)threadIdx.x * 16;
    if (off >= nbytes) continue;
    const long long roff = r_off + c * 2 * CAR_CHUNK + ((off - c * CAR_CHUNK) / ESZ) * 4;
    float s[N];
#pragma unroll
    for (int q = 0; q < N / 4; ++q) {
      const u32x4 v = ld_sys16(mine, roff + 16 * q);
#pragma unroll
      for (int i = 0; i < 4; ++i) s[4 * q + i] = __uint_as_float(v[i]);
    }
    car_epilogue<OP, BF16>(s, off / ESZ, out, h, hb, hb_pack, pack_cols, false, f32x4{}, f32x4{});
  }
  car_end(d, b, &st);
}

// ---- granule one-shot (decode-sized messages): no flag, no barrier -------------------------------------
// Every 4 payload bytes travel as one 8-byte granule {data, tag} written by ONE store (16-B sc0 sc1 stores = two
// granules, each observed untorn on gfx950; MI355X_MICROARCH.md handoff-1to1 vs handoff-flag), tag = the call's epoch
// (a quiet-NaN pattern, never a payload of a working model), so the consumer polls the data itself: one memory round
// trip instead of payload -> vmcnt(0) drain -> flag store -> flag poll -> payload load. The granules of payload chunk c
// (2 KiB of payload, 4 KiB of granules) occupy exactly the A-slot bytes of chunk c, so the block ownership and parity
// rules of the flag protocol hold unchanged (the kernels mix freely on one state).
constexpr int GRAN_THREADS = 128;
constexpr int GRAN_PAYLOAD = GRAN_THREADS * 16;  // payload bytes per chunk (4 KiB of granules)
static_assert(2 * GRAN_PAYLOAD == CAR_CHUNK, "a granule chunk covers one reduce chunk's bytes");


template <int OP, bool BF16>
__global__ void __launch_bounds__(GRAN_THREADS)
    car_gran_kernel(const char* __restrict__ in, void* __restrict__ out, float* __restrict__ h,
                    bf16_t* __restrict__ hb, long long nbytes, const CarDevice* __restrict__ dev,
                    bf16_t* __restrict__ hb_pack, int pack_cols) {
  const CarDevice& d = *dev;
  constexpr int ESZ = BF16 ? 2 : 4;
  constexpr int N = 16 / ESZ;
  const int b = blockIdx.x;
  const long long nchunks = (nbytes + GRAN_PAYLOAD - 1) / GRAN_PAYLOAD;
  if (b >= nchunks) return;
  __shared__ CarCalls st;
  const long long off0 = (long long)b * GRAN_PAYLOAD + (long long)threadIdx.x * 16;
  const bool have0 = off0 < nbytes;
  u32x4 in0 = {0u, 0u, 0u, 0u};
  f32x4 h0a = {0.f, 0.f, 0.f, 0.f}, h0b = {0.f, 0.f, 0.f, 0.f};
  if (have0) {
    in0 = *reinterpret_cast<const u32x4*>(in + off0);
    if constexpr (OP == OP_RESID) {
      h0a = *reinterpret_cast<const f32x4*>(h + off0 / ESZ);
      if constexpr (N == 8) h0b = *reinterpret_cast<const f32x4*>(h + off0 / ESZ + 4);
    }
  }
  const int parity = car_begin(d, b, &st);
  const unsigned tag = gran_tag(st.calls);
  const long long slot = d.max_bytes;
  const long long a_off = (long long)parity * d.world * slot;
  const __amdgpu_buffer_rsrc_t mine = rsrc(d.buf[d.rank]);
  // 1. push: granules of this rank's payload into slot `rank` of every peer
  for (long long c = b; c < nchunks; c += d.grid) {
    const long long off = c * GRAN_PAYLOAD + (long long)threadIdx.x * 16;
    if (off >= nbytes) continue;
    const u32x4 v = c == b ? in0 : *reinterpret_cast<const u32x4*>(in + off);
    const long long g = a_off + (long long)d.rank * slot + 2 * off;  // granule bytes: 2 x payload offset
    const u32x4 g0 = {v[0], tag, v[1], tag}, g1 = {v[2], tag, v[3], tag};
    for (int p = 0; p < d.world; ++p) {
      st_sys16(rsrc(d.buf[p]), g, g0);
      st_sys16(rsrc(d.buf[p]), g + 16, g1);
    }
  }
  // 2. per 16 payload bytes: poll every rank's two granule pairs until they carry this call's tag, sum in rank order
  // give_up: once any wait of any block (or an earlier call) has timed out, every later wait -- further peers, further
  // chunks of this block -- returns at once; the error word is re-read inside each poll loop and after a local timeout,
  // so one launch stalls for at most ~timeout_s however many peers are missing
  bool give_up = __hip_atomic_load(d.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
  for (long long c = b; c < nchunks; c += d.grid) {
    const long long off = c * GRAN_PAYLOAD + (long long)threadIdx.x * 16;
    if (off >= nbytes) continue;
    Piece<BF16> acc;
    for (int p = 0; p < d.world; ++p) {
      const long long g = a_off + (long long)p * slot + 2 * off;
      u32x4 g0 = ld_sys16(mine, g), g1 = ld_sys16(mine, g + 16);
      if (!give_up && (g0[1] != tag || g0[3] != tag || g1[1] != tag || g1[3] != tag)) {
        const long long t0 = (long long)wall_clock64();
        while (g0[1] != tag || g0[3] != tag || g1[1] != tag || g1[3] != tag) {
          if (__hip_atomic_load(d.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
            give_up = true;
            break;
          }
          if ((long long)wall_clock64() - t0 > d.timeout_ticks) {
            __hip_atomic_store(d.error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            give_up = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          g0 = ld_sys16(mine, g);
          g1 = ld_sys16(mine, g + 16);
        }
      }
      const u32x4 v = {g0[0], g0[2], g1[0], g1[2]};
      if (p == 0) acc.set(v); else acc.add(v);
    }
    car_epilogue<OP, BF16>(acc.v, off / ESZ, out, h, hb, hb_pack, pack_cols, OP == OP_RESID && c == b, h0a, h0b);
  }
  car_end(d, b, &st);
}

// (value, index) pairs: granule i = (a[i], b[i] + idx_offset)
template <int MODE>
__global__ void __launch_bounds__(CAR_THREADS)
    car_pairs_kernel(const float* __restrict__ a, const int32_t* __restrict__ bi, int idx_offset, long long n, int k,
                     float* __restrict__ out_a, int32_t* __restrict__ out_b, const CarDevice* __restrict__ dev) {
  const CarDevice& d = *dev;
  const int blk = blockIdx.x;
  const long long nchunks = (n + CAR_PAIR_CHUNK - 1) / CAR_PAIR_CHUNK;
  if (blk >= nchunks) return;
  __shared__ CarCalls st;
  const int parity = car_begin(d, blk, &st);
  const long long slot = d.max_bytes;
  const long long a_off = (long long)parity * d.world * slot;
  const __amdgpu_buffer_rsrc_t mine = rsrc(d.buf[d.rank]);
  for (long long c = blk; c < nchunks; c += d.grid) {
#pragma unroll
    for (int t = 0; t < CAR_PAIRS_PER_THREAD; ++t) {
      const long long i = c * CAR_PAIR_CHUNK + t * CAR_THREADS + threadIdx.x;
      if (i >= n) continue;
      const u32x2 v = {__float_as_uint(a[i]), (unsigned)(bi[i] + idx_offset)};
      for (int p = 0; p < d.world; ++p) st_sys8(rsrc(d.buf[p]), a_off + (long long)d.rank * slot + i * 8, v);
    }
  }
  car_barrier(d, blk, &st);
  for (long long c = blk; c < nchunks; c += d.grid) {
   for (int t = 0; t < CAR_PAIRS_PER_THREAD; ++t) {
    const long long i = c * CAR_PAIR_CHUNK + t * CAR_THREADS + threadIdx.x;
    if (i >= n) continue;
    if (MODE == PAIRS_ARGMAX) {
      u32x2 best = ld_sys8(mine, a_off + i * 8);
      for (int p = 1; p < d.world; ++p) {
        const u32x2 v = ld_sys8(mine, a_off + (long long)p * slot + i * 8);
        if (__uint_as_float(v[0]) > __uint_as_float(best[0])) best = v;  // first max in rank order
      }
      if (out_a) out_a[i] = __uint_as_float(best[0]);
      out_b[i] = (int32_t)best[1];
    } else {
      const long long row = i / k, j = i - row * k;
      for (int p = 0; p < d.world; ++p) {
        const u32x2 v = ld_sys8(mine, a_off + (long long)p * slot + i * 8);
        const long long o = row * (long long)d.world * k + (long long)p * k + j;
        out_a[o] = __uint_as_float(v[0]);
        out_b[o] = (int32_t)v[1];
      }
    }
   }
  }
  car_end(d, blk, &st);
}

// ---- host side -------------------------------------------------------------------------------
struct CarHost {
  CarDevice h;
  CarDevice* d;
  void* own_buf;
  void* own_sig;
  void* opened[2 * CAR_MAX_WORLD];
  int n_opened;
};

// A: 2 parities x world slots x max_bytes; R: 2 parities x 2 * max_bytes (max_bytes % CAR_CHUNK == 0, so chunk c's
// 2 * CAR_CHUNK bytes of R fit for every chunk of a max_bytes message)
size_t car_buffer_bytes(long long max_bytes, int world) {
  return (size_t)2 * world * max_bytes + (size_t)2 * 2 * max_bytes;
}
// flags [CAR_BLOCKS][CAR_MAX_WORLD], then ctr [CAR_BLOCKS] (int2), the error word, and the per-workgroup call counters
// of the fused row-parallel GEMV (gemv.hip MODE_TPRESID)
size_t car_signal_bytes() {
  return (size_t)CAR_BLOCKS * CAR_MAX_WORLD * sizeof(int) + CAR_TAIL_BYTES + (size_t)CAR_WG_COUNTERS * sizeof(int);
}

int car_alloc(long long max_bytes, int world, void** buf, void** sig, hipIpcMemHandle_t* hbuf,
              hipIpcMemHandle_t* hsig) {
  if (world < 1 || world > CAR_MAX_WORLD || max_bytes <= 0 || (max_bytes % CAR_CHUNK)) return -1;
  if (car_buffer_bytes(max_bytes, world) >= 0x7fffffffull) return -3;  // buffer-resource offsets are 31-bit
  *buf = *sig = nullptr;
  hipError_t e = hipExtMallocWithFlags(buf, car_buffer_bytes(max_bytes, world), hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipExtMallocWithFlags(sig, car_signal_bytes(), hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipMemset(*sig, 0, car_signal_bytes());
  // zeroed slots: no granule tag (car.h) can be a leftover of an earlier allocation at this address
  if (e == hipSuccess) e = hipMemset(*buf, 0, car_buffer_bytes(max_bytes, world));
  if (e == hipSuccess) e = hipIpcGetMemHandle(hbuf, *buf);
  if (e == hipSuccess) e = hipIpcGetMemHandle(hsig, *sig);
  if (e != hipSuccess) {
    car_free(*buf, *sig);
    *buf = *sig = nullptr;
  }
  return (int)e;
}

// frees car_alloc's buffers (a rank whose car_init failed, or every rank after a failed rendezvous)
void car_free(void* buf, void* sig) {
  if (buf) (void)hipFree(buf);
  if (sig) (void)hipFree(sig);
}

static void car_close_opened(CarHost* st) {
  for (int i = 0; i < st->n_opened; ++i) (void)hipIpcCloseMemHandle(st->opened[i]);
  st->n_opened = 0;
}

// handles[p] for p != rank are opened; own pointers are used for p == rank
int car_init(int rank, int world, long long max_bytes, void* own_buf, void* own_sig, const hipIpcMemHandle_t* hbufs,
             const hipIpcMemHandle_t* hsigs, double timeout_s, void** state) {
  if (world < 1 || world > CAR_MAX_WORLD || rank < 0 || rank >= world) return -1;
  CarHost* st = new CarHost();
  st->own_buf = own_buf;
  st->own_sig = own_sig;
  st->n_opened = 0;
  st->h.rank = rank;
  st->h.world = world;
  st->h.grid = CAR_GRID_SHARED;
  st->h.max_bytes = max_bytes;
  int dev = 0, rate_khz = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || rate_khz <= 0)
    rate_khz = 100000;
  st->h.timeout_ticks = (long long)(timeout_s * 1000.0 * rate_khz);
  for (int p = 0; p < world; ++p) {
    if (p == rank) {
      st->h.buf[p] = static_cast<char*>(own_buf);
      st->h.sig[p] = static_cast<int*>(own_sig);
      continue;
    }
    void* pb = nullptr;
    void* ps = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&pb, hbufs[p], hipIpcMemLazyEnablePeerAccess);
    if (e == hipSuccess) {
      st->opened[st->n_opened++] = pb;
      e = hipIpcOpenMemHandle(&ps, hsigs[p], hipIpcMemLazyEnablePeerAccess);
      if (e == hipSuccess) st->opened[st->n_opened++] = ps;
    }
    if (e != hipSuccess) {  // undo this rank's mappings; the caller still owns (and frees) its own buffers
      car_close_opened(st);
      delete st;
      return (int)e;
    }
    st->h.buf[p] = static_cast<char*>(pb);
    st->h.sig[p] = static_cast<int*>(ps);
  }
  // barrier / call counters and the error word live after the flags in the local signal allocation
  int* tail = reinterpret_cast<int*>(static_cast<char*>(own_sig) + CAR_BLOCKS * CAR_MAX_WORLD * sizeof(int));
  st->h.ctr = reinterpret_cast<int2*>(tail);  // [CAR_BLOCKS] {calls, barriers}
  st->h.error = tail + 2 * CAR_BLOCKS;
  st->h.wg_ctr = reinterpret_cast<int*>(static_cast<char*>(own_sig) + CAR_BLOCKS * CAR_MAX_WORLD * sizeof(int) +
                                        CAR_TAIL_BYTES);
  st->d = nullptr;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(&st->d), sizeof(CarDevice));
  if (e == hipSuccess) e = hipMemcpy(st->d, &st->h, sizeof(CarDevice), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    if (st->d) (void)hipFree(st->d);
    car_close_opened(st);
    delete st;
    return (int)e;
  }
  *state = st;
  return 0;
}

template <int OP, bool BF16>
static void launch_reduce(int two_shot, int grid, const void* in, void* out, float* h, bf16_t* hb, long long nbytes,
                          const CarDevice* d, hipStream_t s, bf16_t* hb_pack, int pack_cols) {
  if (two_shot)
    car_reduce_kernel<OP, BF16, true><<<grid, CAR_THREADS, 0, s>>>(static_cast<const char*>(in), out, h, hb, nbytes, d,
                                                                   hb_pack, pack_cols);
  else
    car_reduce_kernel<OP, BF16, false><<<grid, CAR_THREADS, 0, s>>>(static_cast<const char*>(in), out, h, hb, nbytes, d,
                                                                    hb_pack, pack_cols);
}

// granule one-shot up to this many payload bytes per rank (the granules take 2x the bytes of the A slot)
static long long g_car_gran_max = 256 << 10;
void car_set_gran_max(long long n) { g_car_gran_max = n; }

// op 0: out = sum(in) (same dtype); op 1: h += sum(in), hb = bf16(h) (h fp32, hb bf16, element count of in)
int car_reduce(void* state, int op, const void* in, void* out, float* h, bf16_t* hb, long long nbytes, int is_bf16,
               int two_shot, hipStream_t s, bf16_t* hb_pack, int pack_cols) {
  CarHost* st = static_cast<CarHost*>(state);
  if (!st || nbytes <= 0) return nbytes == 0 ? 0 : -1;
  if (nbytes > st->h.max_bytes || (nbytes & 15)) return -2;
  if (op == OP_RESID && (!h || !hb)) return -1;
  if (hb_pack && (op != OP_RESID || pack_cols <= 0 || (pack_cols & 31))) return -1;
  if (two_shot && st->h.world == 1) two_shot = 0;
  if (!two_shot && nbytes <= g_car_gran_max && 2 * nbytes <= st->h.max_bytes) {
    const long long gch = (nbytes + GRAN_PAYLOAD - 1) / GRAN_PAYLOAD;
    const int ggrid = (int)(gch < st->h.grid ? gch : st->h.grid);
    const char* ip = static_cast<const char*>(in);
#define JLA_GRAN(OPV, BFV)                                                                                          \
  car_gran_kernel<OPV, BFV><<<ggrid, GRAN_THREADS, 0, s>>>(ip, out, h, hb, nbytes, st->d, OPV == OP_RESID ? hb_pack : nullptr, \
                                                          OPV == OP_RESID ? pack_cols : 0)
    if (op == OP_SUM) {
      if (is_bf16) JLA_GRAN(OP_SUM, true); else JLA_GRAN(OP_SUM, false);
    } else {
      if (is_bf16) JLA_GRAN(OP_RESID, true); else JLA_GRAN(OP_RESID, false);
    }
#undef JLA_GRAN
    JLA_CHECK_LAUNCH();
    return 0;
  }
  const long long nchunks = (nbytes + CAR_CHUNK - 1) / CAR_CHUNK;
  const int grid = (int)(nchunks < st->h.grid ? nchunks : st->h.grid);
  if (op == OP_SUM) {
    if (is_bf16) launch_reduce<OP_SUM, true>(two_shot, grid, in, out, h, hb, nbytes, st->d, s, nullptr, 0);
    else launch_reduce<OP_SUM, false>(two_shot, grid, in, out, h, hb, nbytes, st->d, s, nullptr, 0);
  } else {
    if (is_bf16) launch_reduce<OP_RESID, true>(two_shot, grid, in, out, h, hb, nbytes, st->d, s, hb_pack, pack_cols);
    else launch_reduce<OP_RESID, false>(two_shot, grid, in, out, h, hb, nbytes, st->d, s, hb_pack, pack_cols);
  }
  JLA_CHECK_LAUNCH();
  return 0;
}

// mode 0 (argmax): out_b[i] = index of the first max over ranks of pair i (out_a: its value, optional)
// mode 1 (top-k):  n = rows * k; out_a/out_b[row][p * k + j] = rank p's pair (row, j)
int car_pairs(void* state, int mode, const float* a, const int32_t* b, int idx_offset, long long n, int k,
              float* out_a, int32_t* out_b, hipStream_t s) {
  CarHost* st = static_cast<CarHost*>(state);
  if (!st || n <= 0) return n == 0 ? 0 : -1;
  if (n * 8 > st->h.max_bytes) return -2;
  if (mode == PAIRS_TOPK && (k <= 0 || n % k || !out_a)) return -1;
  const long long nchunks = (n + CAR_PAIR_CHUNK - 1) / CAR_PAIR_CHUNK;
  const int grid = (int)(nchunks < st->h.grid ? nchunks : st->h.grid);
  if (mode == PAIRS_ARGMAX)
    car_pairs_kernel<PAIRS_ARGMAX><<<grid, CAR_THREADS, 0, s>>>(a, b, idx_offset, n, k, out_a, out_b, st->d);
  else
    car_pairs_kernel<PAIRS_TOPK><<<grid, CAR_THREADS, 0, s>>>(a, b, idx_offset, n, k, out_a, out_b, st->d);
  JLA_CHECK_LAUNCH();
  return 0;
}

// collective blocks per launch of this instance (every rank of the group must set the same value, before first use)
int car_set_grid(void* state, int grid) {
  CarHost* st = static_cast<CarHost*>(state);
  if (grid == 0) grid = CAR_GRID_MAX;
  if (!st || grid < 1 || grid > CAR_GRID_MAX) return -1;
  st->h.grid = grid;
  return (int)hipMemcpy(st->d, &st->h, sizeof(CarDevice), hipMemcpyHostToDevice);
}

int car_world(void* state) { return static_cast<CarHost*>(state)->h.world; }
const void* car_device(void* state) { return static_cast<CarHost*>(state)->d; }
long long car_max_bytes(void* state) { return static_cast<CarHost*>(state)->h.max_bytes; }

int car_error(void* state) {
  CarHost* st = static_cast<CarHost*>(state);
  int v = 0;
  if (hipMemcpy(&v, st->h.error, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return v;
}

void car_destroy(void* state) {
  CarHost* st = static_cast<CarHost*>(state);
  if (!st) return;
  car_close_opened(st);
  (void)hipFree(st->d);
  (void)hipFree(st->own_buf);
  (void)hipFree(st->own_sig);
  delete st;
}

}  // namespace jla
