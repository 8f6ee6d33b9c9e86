// Diagnostic: where a gemm2 ping-pong K-tile spends its cycles (s_memtime stamps per phase per wave).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -DJLA_GEMM_STAMPS \
//     -I jax_llama_amd/csrc/kernels tools/debug/gemm_stamps.hip -o tools/debug/gemm_stamps
//   ./tools/debug/gemm_stamps M N K
// Prints mean per-wave cycles per K-tile of: L phase (issue + LDS reads + waits), barrier 1 wait,
// M phase (32 MFMA issue), barrier 2 wait -- for each wave row (ping-pong group). Read the SHARES, not
// the total: the stamps' own waits forbid some overlap.
#include "../../jax_llama_amd/csrc/kernels/gemm.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096, N = argc > 2 ? atoi(argv[2]) : 28672,
            K = argc > 3 ? atoi(argv[3]) : 4096;
  std::vector<uint16_t> hx((size_t)M * K), hw((size_t)N * K);
  for (auto& v : hx) v = 0x3f80 ^ (rand() & 0x807f);  // random-ish bf16 around +-1
  for (auto& v : hw) v = 0x3c00 ^ (rand() & 0x807f);
  uint16_t *x, *w, *out;
  hipMalloc(&x, hx.size() * 2);
  hipMalloc(&w, hw.size() * 2);
  hipMalloc(&out, (size_t)M * N * 2);
  hipMemcpy(x, hx.data(), hx.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(w, hw.data(), hw.size() * 2, hipMemcpyHostToDevice);
  for (int it = 0; it < 3; ++it)
    jla::gemm(x, w, out, M, N, K, MODE_STORE, 0, 0, nullptr, nullptr, nullptr, 0, 1, 0, -1.f, 1);
  hipDeviceSynchronize();
  const int tm = (M + 255) / 256, tn = (N + 255) / 256, nwg = tm * tn;
  std::vector<unsigned long long> st((size_t)nwg * 8 * 6);
  hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(jla::g_gemm_stamps), st.size() * 8);
  const int KT = K / 32;
  for (int grp = 0; grp < 2; ++grp) {
    double acc[6] = {0, 0, 0, 0, 0, 0};
    for (int b = 0; b < nwg; ++b)
      for (int wv = grp * 4; wv < grp * 4 + 4; ++wv)
        for (int q = 0; q < 6; ++q) acc[q] += st[((size_t)b * 8 + wv) * 6 + q];
    const double n = (double)nwg * 4 * KT;
    const double tot = acc[0] + acc[1] + acc[2] + acc[3];
    printf("  L split: glds issue %.0f, ds_reads (issued+landed) %.0f, vmcnt wait %.0f\n", acc[4] / n, acc[5] / n,
           acc[0] / n);
    acc[0] += acc[4] + acc[5];
    printf("group %d cycles/K-tile: L %.0f  bar1 %.0f  M %.0f  bar2 %.0f  (total %.0f; L %.0f%% bar1 %.0f%% M %.0f%% bar2 %.0f%%)\n",
           grp, acc[0] / n, acc[1] / n, acc[2] / n, acc[3] / n, tot / n, 100 * acc[0] / tot, 100 * acc[1] / tot,
           100 * acc[2] / tot, 100 * acc[3] / tot);
  }
  return 0;
}
