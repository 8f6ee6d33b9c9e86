// Custom xGMI collective state shared by the collective kernels (allreduce.hip) and the GEMV's fused row-parallel
// epilogue (gemv.hip MODE_TPRESID): every rank's IPC-mapped buffers, counters, the error word, and the system-scope
// (sc0 sc1) buffer accesses every hand-off byte goes through.
#pragma once
#include "common.h"
#include "launchers.h"

namespace jla {

constexpr int CAR_MAX_WORLD = 8;
constexpr int CAR_BLOCKS = 256;        // signal rows (one per collective block)
constexpr int CAR_TAIL_BYTES = 4096;   // after the flags: ctr [CAR_BLOCKS] (int2) and the error word
constexpr int CAR_GRID_SHARED = 63;    // ranks sharing one GPU (tests): 8 x 63 blocks stay co-resident
constexpr int CAR_GRID_MAX = 255;      // one rank per GPU: a 4 MiB message spreads over every CU

struct CarDevice {
  char* buf[CAR_MAX_WORLD];     // every rank's buffer (A then R), mapped here
  int* sig[CAR_MAX_WORLD];      // every rank's flags [CAR_BLOCKS][CAR_MAX_WORLD]
  int2* ctr;                    // [CAR_BLOCKS] {calls made, barriers passed} by block b (local): ONE 8-byte load
                                // at the start of a call gives both the parity and the flag epoch
  int* error;                   // 1 once a wait timed out
  int* wg_ctr;                  // [CAR_WG_COUNTERS] calls made by fused-GEMV workgroup w (local; parity + tag)
  long long max_bytes;          // A slot size; R holds 2 * max_bytes per parity
  long long timeout_ticks;      // wall-clock ticks (s_memrealtime, 100 MHz) before giving up
  int rank, world;
  int grid;                     // collective blocks per launch (chunk c -> block c % grid on every call, every rank):
                                // CAR_GRID_SHARED while ranks share a device (every rank's blocks co-resident), else
                                // CAR_GRID_MAX; fixed for the life of the instance
};

constexpr int SYS = 17;  // cache policy bits: sc0 | sc1

JLA_DEV __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
JLA_DEV void st_sys16(__amdgpu_buffer_rsrc_t r, long long off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, SYS);
}
JLA_DEV u32x4 ld_sys16(__amdgpu_buffer_rsrc_t r, long long off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, SYS);
}
JLA_DEV void st_sys8(__amdgpu_buffer_rsrc_t r, long long off, u32x2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)off, 0, SYS);
}
JLA_DEV u32x2 ld_sys8(__amdgpu_buffer_rsrc_t r, long long off) {
  return __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, SYS);
}

// granule tag of a call: a quiet-NaN pattern (never a payload of a working model) carrying the call count
JLA_DEV unsigned gran_tag(int calls) { return 0x7FC00000u | ((unsigned)calls & 0x003FFFFFu); }
// the fused GEMV's tags (gemv.hip MODE_TPRESID): the negative quiet NaNs, so granules the standalone kernels left in
// the same slots (the instance's self-test) never carry a fused call's tag
JLA_DEV unsigned gran_tag_fused(int calls) { return 0xFFC00000u | ((unsigned)calls & 0x003FFFFFu); }

// The fused epilogues' gather (gemv.hip MODE_TPRESID, gemm.hip gemm_reduce_tp_kernel): the 8-byte granule at `off` of
// this rank's buffer once it carries `tag`. One load in the common case; otherwise poll, bounded by the group's timeout
// (then the error word is set and the stale granule returned: the host raises at its next poll). give_up: another
// workgroup already timed out -- no second wait.
JLA_DEV u32x2 car_granule(const CarDevice& d, __amdgpu_buffer_rsrc_t mine, long long off, unsigned tag, bool give_up) {
  u32x2 r = ld_sys8(mine, off);
  if (r[1] != tag && !give_up) {
    const long long t0 = (long long)wall_clock64();
    while (r[1] != tag) {
      if ((long long)wall_clock64() - t0 > d.timeout_ticks) {
        __hip_atomic_store(d.error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      if (__hip_atomic_load(d.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
      __builtin_amdgcn_s_sleep(1);
      r = ld_sys8(mine, off);
    }
  }
  return r;
}

// The gather of a whole group: granule `off + p * stride` of this rank's buffer for every rank p, every load issued
// before any is checked -- one round trip for the group instead of one per rank (a check on each load before the next
// one serialised world round trips per element) -- then a granule still without its tag is polled alone. W: the
// loads issued (the world size, rounded up to 1 / 2 / 4 / 8; ranks past the world re-read rank 0's granule, never an
// address outside the buffer -- hipcc issues such predicated loads unconditionally).
template <int W>
JLA_DEV void car_gather8_w(const CarDevice& d, __amdgpu_buffer_rsrc_t mine, long long off, long long stride,
                           unsigned tag, bool give_up, u32x2 (&r)[CAR_MAX_WORLD]) {
#pragma unroll
  for (int p = 0; p < W; ++p) r[p] = ld_sys8(mine, off + (long long)(p < d.world ? p : 0) * stride);
#pragma unroll
  for (int p = 0; p < W; ++p)
    if (p < d.world && r[p][1] != tag) r[p] = car_granule(d, mine, off + (long long)p * stride, tag, give_up);
}
JLA_DEV void car_gather8(const CarDevice& d, __amdgpu_buffer_rsrc_t mine, long long off, long long stride,
                         unsigned tag, bool give_up, u32x2 (&r)[CAR_MAX_WORLD]) {
  if (d.world == 1)
    car_gather8_w<1>(d, mine, off, stride, tag, give_up, r);
  else if (d.world == 2)
    car_gather8_w<2>(d, mine, off, stride, tag, give_up, r);
  else if (d.world <= 4)
    car_gather8_w<4>(d, mine, off, stride, tag, give_up, r);
  else
    car_gather8_w<8>(d, mine, off, stride, tag, give_up, r);
}
// two adjacent granules per rank (16 bytes, one load; each 8-byte half carries its own tag), polled as a pair
template <int W>
JLA_DEV void car_gather16_w(const CarDevice& d, __amdgpu_buffer_rsrc_t mine, long long off, long long stride,
                            unsigned tag, bool give_up, u32x4 (&r)[CAR_MAX_WORLD]) {
#pragma unroll
  for (int p = 0; p < W; ++p) r[p] = ld_sys16(mine, off + (long long)(p < d.world ? p : 0) * stride);
#pragma unroll
  for (int p = 0; p < W; ++p) {
    if (p < d.world && (r[p][1] != tag || r[p][3] != tag) && !give_up) {
      const long long o = off + (long long)p * stride;
      const long long t0 = (long long)wall_clock64();
      do {
        if ((long long)wall_clock64() - t0 > d.timeout_ticks) {
          __hip_atomic_store(d.error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        if (__hip_atomic_load(d.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
        __builtin_amdgcn_s_sleep(1);
        r[p] = ld_sys16(mine, o);
      } while (r[p][1] != tag || r[p][3] != tag);
    }
  }
}
JLA_DEV void car_gather16(const CarDevice& d, __amdgpu_buffer_rsrc_t mine, long long off, long long stride,
                          unsigned tag, bool give_up, u32x4 (&r)[CAR_MAX_WORLD]) {
  if (d.world == 1)
    car_gather16_w<1>(d, mine, off, stride, tag, give_up, r);
  else if (d.world == 2)
    car_gather16_w<2>(d, mine, off, stride, tag, give_up, r);
  else if (d.world <= 4)
    car_gather16_w<4>(d, mine, off, stride, tag, give_up, r);
  else
    car_gather16_w<8>(d, mine, off, stride, tag, give_up, r);
}

}  // namespace jla
