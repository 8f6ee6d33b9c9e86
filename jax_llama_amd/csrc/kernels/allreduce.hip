// One-shot push all-reduce over xGMI for decode-sized tensor-parallel messages (SURVEY D1 / X1-X2:
// the row-parallel wo / w2 outputs, 2 per layer per token; reference partition.py:67,70 where XLA's
// GSPMD inserts the NCCL all-reduce).
//
// Every rank owns one uncached (MTYPE UC, hipDeviceMallocUncached) receive buffer
// [2 parities][world slots][max_bytes] and a signal array [64 blocks][world], both exported by
// IPC handle and mapped by every peer. A call:
//   1. block b copies its byte-chunks of the local input into slot `rank` of EVERY rank's buffer
//      (remote stores go straight over the rank<->peer xGMI link; uncached, so they land in the
//      peer's HBM), drains them (s_waitcnt vmcnt(0)), then writes its epoch into flag[b][rank] of
//      every peer;
//   2. waits until flag[b][p] >= epoch for every peer p (bounded spin: a missing peer sets the
//      error word instead of hanging the GPU);
//   3. sums slots 0..world-1 IN RANK ORDER from its local buffer -> bit-identical result on
//      every rank.
// Chunks map to blocks by byte offset (chunk c -> block c % 63) on every call and every rank, and
// epochs are per block, so block b of rank r only ever pairs with block b of its peers; the parity
// buffers make one barrier per call enough: block b overwrites a parity slot two calls later, and
// by then it has seen every peer's block b signal the call in between (after that peer's reads).
// Graph-capturable: all state (pointers, epochs) lives in device memory.
#include "common.h"
#include "launchers.h"

namespace jla {

constexpr int CAR_MAX_WORLD = 8;
constexpr int CAR_BLOCKS = 64;   // signal rows; blocks 0..62 carry data, word 63 of the tail = error
constexpr int CAR_GRID = 63;     // chunk c -> block c % CAR_GRID on every call (fixed mapping)
constexpr int CAR_THREADS = 256;
constexpr int CAR_CHUNK = CAR_THREADS * 16;  // bytes per block iteration

struct CarDevice {
  char* buf[CAR_MAX_WORLD];     // every rank's receive buffer, mapped here
  int* sig[CAR_MAX_WORLD];      // every rank's signal array [CAR_BLOCKS][CAR_MAX_WORLD]
  int* epoch;                   // this rank's per-block epochs [CAR_BLOCKS] (local)
  int* error;                   // set to 1 when a spin times out
  long long max_bytes;
  int rank, world;
};

JLA_DEV void st_uc(u32x4* p, u32x4 v) { __builtin_nontemporal_store(v, p); }
JLA_DEV u32x4 ld_uc(const u32x4* p) { return __builtin_nontemporal_load(p); }

JLA_DEV void add4f(u32x4& acc, const u32x4 v) {
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = __float_as_uint(__uint_as_float(acc[i]) + __uint_as_float(v[i]));
}

// bf16 messages accumulate the world slots in fp32 and round once.
__global__ void __launch_bounds__(CAR_THREADS)
    car_kernel(const char* __restrict__ in, char* __restrict__ out, long long nbytes, int is_bf16,
               const CarDevice* __restrict__ dev) {
  const CarDevice& d = *dev;  // by reference: a by-value copy indexed with runtime p lives in scratch
  const int b = blockIdx.x;
  const long long nchunks = (nbytes + CAR_CHUNK - 1) / CAR_CHUNK;
  if (b >= nchunks) return;
  __shared__ int s_epoch;
  if (threadIdx.x == 0) {
    const int e = d.epoch[b] + 1;
    d.epoch[b] = e;
    s_epoch = e;
  }
  __syncthreads();
  const int e = s_epoch;
  const int parity = e & 1;
  const long long slot_bytes = d.max_bytes;
  const long long par_off = (long long)parity * d.world * slot_bytes;

  // 1. push local input into slot `rank` of every rank's buffer
  for (long long c = b; c < nchunks; c += CAR_GRID) {
    const long long off = c * CAR_CHUNK + (long long)threadIdx.x * 16;
    if (off < nbytes) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(in + off);
      for (int p = 0; p < d.world; ++p)
        st_uc(reinterpret_cast<u32x4*>(d.buf[p] + par_off + (long long)d.rank * slot_bytes + off), v);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < d.world) {
    int* f = d.sig[threadIdx.x] + b * CAR_MAX_WORLD + d.rank;
    __hip_atomic_store(f, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 2. wait for every peer's block b
  if (threadIdx.x < d.world) {
    const int* f = d.sig[d.rank] + b * CAR_MAX_WORLD + threadIdx.x;
    int it = 0;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      if (++it > (1 << 24)) {
        __hip_atomic_store(d.error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  asm volatile("" ::: "memory");
  __syncthreads();
  // 3. sum the slots in rank order (identical on every rank)
  const char* mine = d.buf[d.rank] + par_off;
  for (long long c = b; c < nchunks; c += CAR_GRID) {
    const long long off = c * CAR_CHUNK + (long long)threadIdx.x * 16;
    if (off >= nbytes) continue;
    if (is_bf16) {
      float acc[8];
      unpack8(ld_uc(reinterpret_cast<const u32x4*>(mine + off)), acc);
      for (int p = 1; p < d.world; ++p) {
        float f[8];
        unpack8(ld_uc(reinterpret_cast<const u32x4*>(mine + (long long)p * slot_bytes + off)), f);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += f[i];
      }
      *reinterpret_cast<u32x4*>(out + off) = pack8(acc);
    } else {
      u32x4 acc = ld_uc(reinterpret_cast<const u32x4*>(mine + off));
      for (int p = 1; p < d.world; ++p)
        add4f(acc, ld_uc(reinterpret_cast<const u32x4*>(mine + (long long)p * slot_bytes + off)));
      *reinterpret_cast<u32x4*>(out + off) = acc;
    }
  }
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

size_t car_buffer_bytes(long long max_bytes, int world) { return (size_t)2 * world * max_bytes; }
size_t car_signal_bytes() { return (size_t)CAR_BLOCKS * CAR_MAX_WORLD * sizeof(int) + 256; }

int car_alloc(long long max_bytes, int world, void** buf, void** sig, hipIpcMemHandle_t* hbuf,
              hipIpcMemHandle_t* hsig) {
  if (world < 1 || world > CAR_MAX_WORLD || max_bytes <= 0 || (max_bytes & 15)) return -1;
  hipError_t e = hipExtMallocWithFlags(buf, car_buffer_bytes(max_bytes, world), hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipExtMallocWithFlags(sig, car_signal_bytes(), hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(*sig, 0, car_signal_bytes());
  if (e != hipSuccess) return (int)e;
  e = hipIpcGetMemHandle(hbuf, *buf);
  if (e != hipSuccess) return (int)e;
  e = hipIpcGetMemHandle(hsig, *sig);
  return (int)e;
}

// handles[p] for p != rank are opened; own pointers are used for p == rank
int car_init(int rank, int world, long long max_bytes, void* own_buf, void* own_sig, const hipIpcMemHandle_t* hbufs,
             const hipIpcMemHandle_t* hsigs, void** state) {
  if (world < 1 || world > CAR_MAX_WORLD || rank < 0 || rank >= world) return -1;
  CarHost* st = new CarHost();
  st->own_buf = own_buf;
  st->own_sig = own_sig;
  st->n_opened = 0;
  st->h.rank = rank;
  st->h.world = world;
  st->h.max_bytes = max_bytes;
  for (int p = 0; p < world; ++p) {
    if (p == rank) {
      st->h.buf[p] = static_cast<char*>(own_buf);
      st->h.sig[p] = static_cast<int*>(own_sig);
      continue;
    }
    void* pb = nullptr;
    void* ps = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&pb, hbufs[p], hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return (int)e;
    e = hipIpcOpenMemHandle(&ps, hsigs[p], hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return (int)e;
    st->opened[st->n_opened++] = pb;
    st->opened[st->n_opened++] = ps;
    st->h.buf[p] = static_cast<char*>(pb);
    st->h.sig[p] = static_cast<int*>(ps);
  }
  // per-block epochs and the error word live after the flags in the local signal allocation
  char* tail = static_cast<char*>(own_sig) + CAR_BLOCKS * CAR_MAX_WORLD * sizeof(int);
  st->h.epoch = reinterpret_cast<int*>(tail);       // [CAR_GRID] per-block epochs
  st->h.error = reinterpret_cast<int*>(tail) + CAR_GRID;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(&st->d), sizeof(CarDevice));
  if (e != hipSuccess) return (int)e;
  e = hipMemcpy(st->d, &st->h, sizeof(CarDevice), hipMemcpyHostToDevice);
  if (e != hipSuccess) return (int)e;
  *state = st;
  return 0;
}

int car_allreduce(void* state, const void* in, void* out, long long nbytes, int is_bf16, hipStream_t s) {
  CarHost* st = static_cast<CarHost*>(state);
  if (!st || nbytes <= 0) return nbytes == 0 ? 0 : -1;
  if (nbytes > st->h.max_bytes || (nbytes & 15)) return -2;
  const long long nchunks = (nbytes + CAR_CHUNK - 1) / CAR_CHUNK;
  const int grid = (int)(nchunks < CAR_GRID ? nchunks : CAR_GRID);
  car_kernel<<<grid, CAR_THREADS, 0, s>>>(static_cast<const char*>(in), static_cast<char*>(out), nbytes, is_bf16,
                                          st->d);
  JLA_CHECK_LAUNCH();
  return 0;
}

int car_error(void* state) {
  CarHost* st = static_cast<CarHost*>(state);
  int v = 0;
  if (hipMemcpy(&v, st->h.error, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return v;
}

void car_destroy(void* state) {
  CarHost* st = static_cast<CarHost*>(state);
  if (!st) return;
  for (int i = 0; i < st->n_opened; ++i) (void)hipIpcCloseMemHandle(st->opened[i]);
  (void)hipFree(st->d);
  (void)hipFree(st->own_buf);
  (void)hipFree(st->own_sig);
  delete st;
}

}  // namespace jla
