// CU placement: streams restricted to a set of CUs, and a census of where a launch's workgroups run.
//
// The large-batch decode step splits the chip between the memory-bound decode attention of one micro-batch and the
// MFMA-bound projections of the other (runtime/engine.py, the partitioned schedule). Sharing a CU does not work:
// with the attention's K / V stream co-resident beside a gemm4 workgroup, the GEMM's LDS-DMA K-tiles queue behind the
// stream's HBM misses in the CU's own memory pipeline and the GEMM takes 1.6x as long (profiles/r6_overlap_probe*.jsonl,
// kernel trace r6_overlap_trace_coresident.txt). Disjoint CU sets do not share that queue: each side gets a stream
// created with a CU mask (hipExtStreamCreateWithCUMask; bit i = CU i of the device's logical numbering).
#include <hip/hip_runtime.h>

#include <vector>

#include "common.h"

namespace jla {

// one record per workgroup: HW_ID (wave / SIMD / CU / SH / SE ids) and XCC_ID
__global__ void __launch_bounds__(64) cu_census_kernel(uint32_t* __restrict__ out) {
  if (threadIdx.x == 0) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
  }
}

int cu_census(uint32_t* out, int blocks, hipStream_t s) {
  if (blocks <= 0) return -1;
  cu_census_kernel<<<blocks, 64, 0, s>>>(out);
  JLA_CHECK_LAUNCH();
  return 0;
}

int cu_mask_stream_create(const uint32_t* mask, int words, hipStream_t* out) {
  if (words <= 0 || !out) return -1;
  return hipExtStreamCreateWithCUMask(out, (uint32_t)words, mask) == hipSuccess ? 0 : -2;
}

int cu_mask_stream_get(hipStream_t s, uint32_t* mask, int words) {
  return hipExtStreamGetCUMask(s, (uint32_t)words, mask) == hipSuccess ? 0 : -2;
}

int stream_destroy(hipStream_t s) { return hipStreamDestroy(s) == hipSuccess ? 0 : -2; }

// kernel launches recorded in a captured graph (torch.cuda.CUDAGraph.raw_cuda_graph()): the decode step's launch count
// as the hardware sees it (bench.py reports it per layer)
int graph_kernel_nodes(hipGraph_t g) {
  size_t n = 0;
  if (hipGraphGetNodes(g, nullptr, &n) != hipSuccess) return -2;
  if (n == 0) return 0;
  std::vector<hipGraphNode_t> nodes(n);
  if (hipGraphGetNodes(g, nodes.data(), &n) != hipSuccess) return -2;
  int k = 0;
  for (size_t i = 0; i < n; ++i) {
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nodes[i], &t) == hipSuccess && t == hipGraphNodeTypeKernel) ++k;
  }
  return k;
}

}  // namespace jla
