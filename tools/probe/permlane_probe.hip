// Semantics of gfx950 v_permlane32_swap / v_permlane16_swap with the same
// register as both operands: prints, per lane, where each result came from.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned *o) {
  const unsigned v = threadIdx.x;
  auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  auto s = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  o[4 * threadIdx.x + 0] = r[0];
  o[4 * threadIdx.x + 1] = r[1];
  o[4 * threadIdx.x + 2] = s[0];
  o[4 * threadIdx.x + 3] = s[1];
}
int main() {
  unsigned *d, h[256];
  hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) printf("lane %2d: p32 {%2u %2u} p16 {%2u %2u}\n", l, h[4 * l], h[4 * l + 1], h[4 * l + 2], h[4 * l + 3]);
  return 0;
}
