// Token selection and decode-loop bookkeeping (replaces HF FlaxGenerationMixin's loop body that the
// reference inherits: generation.py:28-41 -> _greedy_search / _sample).
//
// argmax: first index of the row maximum (jnp.argmax semantics), also returns the max value so a
//   vocab-parallel (TP) caller can pick the global winner from one (value, index) pair per rank.
// decode_update: finished rows emit pad, is_sent_finished |= (token == eos), sequences[:, cur_len]
//   = token, positions += 1, cache slot += 1, cur_len += 1 -- all on the device so the whole decode
//   step (model + sampler + state) replays from one hipGraph without host round trips.
#include "common.h"
#include "launchers.h"

namespace jla {

__global__ void __launch_bounds__(1024)
    argmax_kernel(const float* __restrict__ logits, int V, int32_t* __restrict__ idx, float* __restrict__ val) {
  __shared__ float sv[16];
  __shared__ int si[16];
  const int row = blockIdx.x;
  const float* x = logits + (size_t)row * V;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    const float v = x[i];
    if (v > bv) {  // strictly greater: keeps the first index within a thread's stride
      bv = v;
      bi = i;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > bv || (ov == bv && oi < bi)) {
      bv = ov;
      bi = oi;
    }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    sv[wid] = bv;
    si[wid] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
    for (int w = 1; w < nw; ++w)
      if (sv[w] > bv || (sv[w] == bv && si[w] < bi)) {
        bv = sv[w];
        bi = si[w];
      }
    idx[row] = bi == 0x7fffffff ? 0 : bi;
    val[row] = bv;
  }
}

int argmax(const float* logits, int B, int V, int32_t* idx, float* val, hipStream_t s) {
  if (B <= 0) return 0;
  argmax_kernel<<<B, 1024, 0, s>>>(logits, V, idx, val);
  JLA_CHECK_LAUNCH();
  return 0;
}

__global__ void decode_update_kernel(const int32_t* __restrict__ nxt, int32_t* __restrict__ finished,
                                     int32_t* __restrict__ sequences, int32_t* __restrict__ cur_len,
                                     int32_t* __restrict__ tokens, int32_t* __restrict__ positions,
                                     int32_t* __restrict__ slot, int B, int L, int pad, int eos) {
  const int cl = cur_len[0];
  for (int b = threadIdx.x; b < B; b += blockDim.x) {  // one workgroup: any batch size
    int t = nxt[b];
    const int fin = finished[b];
    if (fin) t = pad;
    finished[b] = (fin || t == eos) ? 1 : 0;
    if (cl < L)
      sequences[(size_t)b * L + cl] = t;
    else
      JLA_FLAG(JLA_BOUNDS_SEQ);
    tokens[b] = t;
    positions[b] += 1;
  }
  __syncthreads();  // every thread has read cur_len before it advances
  if (threadIdx.x == 0) {
    cur_len[0] = cl + 1;
    slot[0] += 1;
  }
}

int decode_update(const int32_t* nxt, int32_t* finished, int32_t* sequences, int32_t* cur_len, int32_t* tokens,
                  int32_t* positions, int32_t* slot, int B, int L, int pad, int eos, hipStream_t s) {
  if (B <= 0) return -1;
  decode_update_kernel<<<1, min(1024, ((B + 63) / 64) * 64), 0, s>>>(nxt, finished, sequences, cur_len, tokens, positions, slot,
                                                          B, L, pad, eos);
  JLA_CHECK_LAUNCH();
  return 0;
}

JLA_BOUNDS_ACCESSOR(sample)

}  // namespace jla
