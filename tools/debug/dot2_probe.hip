#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__global__ void k(const unsigned* a, const unsigned* b, const float* c, float* o) {
  int i = threadIdx.x;
  o[i] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a[i]), __builtin_bit_cast(bf16x2_t, b[i]), c[i], false);
}
static unsigned bf(float f) { unsigned u; u = __builtin_bit_cast(unsigned, f); return u >> 16; }
int main() {
  const int n = 4;
  float av[n][2] = {{1.5f, 2.f}, {1.f, 0.f}, {0.f, 1.f}, {0.3f, -0.7f}};
  float bv[n][2] = {{3.f, .5f}, {2.f, 5.f}, {2.f, 5.f}, {1.1f, 2.3f}};
  float cv[n] = {0.f, 0.f, 0.f, 0.25f};
  unsigned ha[n], hb[n];
  for (int i = 0; i < n; ++i) { ha[i] = bf(av[i][0]) | (bf(av[i][1]) << 16); hb[i] = bf(bv[i][0]) | (bf(bv[i][1]) << 16); }
  unsigned *da, *db; float *dc, *dout; float out[n];
  hipMalloc(&da, 16); hipMalloc(&db, 16); hipMalloc(&dc, 16); hipMalloc(&dout, 16);
  hipMemcpy(da, ha, 16, hipMemcpyHostToDevice); hipMemcpy(db, hb, 16, hipMemcpyHostToDevice); hipMemcpy(dc, cv, 16, hipMemcpyHostToDevice);
  k<<<1, n>>>(da, db, dc, dout);
  hipMemcpy(out, dout, 16, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; ++i) printf("dot2 %d: got %f expect %f\n", i, out[i], av[i][0]*bv[i][0] + av[i][1]*bv[i][1] + cv[i]);
  return 0;
}
