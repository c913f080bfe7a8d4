// Diagnostic only: streams the n=16, m=32 QP inputs with the solver kernel's
// exact load pattern (H, A: two rows per dwordx4 instruction per QP; f, b)
// and writes a per-QP checksum, at a forced occupancy (LDS padding).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

template <int LDS_DOUBLES>
__global__ __launch_bounds__(64) void probe(const double* __restrict__ Hg, const double* __restrict__ fg,
                                            const double* __restrict__ Ag, const double* __restrict__ bg,
                                            double* __restrict__ xg, long long batch) {
  __shared__ double pad[LDS_DOUBLES];
  const int l = threadIdx.x & 15;
  const long long g = (long long)blockIdx.x * 4 + (threadIdx.x >> 4);
  if (g >= batch) return;
  const double* Hq = Hg + g * 256;
  const double* Aq = Ag + g * 512;
  const int hr = l >> 3, hc = 2 * (l & 7);
  double acc = 0;
#pragma unroll
  for (int t = 0; t < 8; ++t) { double2 v = *reinterpret_cast<const double2*>(&Hq[(2 * t + hr) * 16 + hc]); acc += v.x + v.y; }
#pragma unroll
  for (int t = 0; t < 16; ++t) { double2 v = *reinterpret_cast<const double2*>(&Aq[(2 * t + hr) * 16 + hc]); acc += v.x + v.y; }
  acc += fg[g * 16 + l] + bg[g * 32 + l] + bg[g * 32 + 16 + l];
  pad[threadIdx.x] = acc;
  __builtin_amdgcn_wave_barrier();
  acc += pad[(threadIdx.x + 1) & 63];
  xg[g * 16 + l] = acc;
}

template <int L>
float run(const double* H, const double* f, const double* A, const double* b, double* x, long long B) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(probe<L>, dim3(B / 4), dim3(64), 0, 0, H, f, A, b, x, B);
  hipEventRecord(e0);
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(probe<L>, dim3(B / 4), dim3(64), 0, 0, H, f, A, b, x, B);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / 10;
}

int main() {
  const long long B = 262144;
  double *H, *f, *A, *b, *x;
  hipMalloc(&H, B * 256 * 8); hipMalloc(&A, B * 512 * 8); hipMalloc(&f, B * 16 * 8); hipMalloc(&b, B * 32 * 8); hipMalloc(&x, B * 16 * 8);
  hipMemset(H, 0, B * 256 * 8); hipMemset(A, 0, B * 512 * 8); hipMemset(f, 0, B * 128); hipMemset(b, 0, B * 256);
  const double bytes = B * (256 + 512 + 16 + 32 + 16) * 8.0;
  // LDS per block -> waves per CU: 64 doubles (~32/CU), 2560 (20 KB, 8/CU), 5120 (40 KB, 4/CU)
  float t;
  t = run<64>(H, f, A, b, x, B);   printf("occ=max   %.3f ms  %.0f GB/s\n", t, bytes / t / 1e6);
  t = run<1400>(H, f, A, b, x, B); printf("occ=14/CU %.3f ms  %.0f GB/s\n", t, bytes / t / 1e6);
  t = run<2560>(H, f, A, b, x, B); printf("occ=8/CU  %.3f ms  %.0f GB/s\n", t, bytes / t / 1e6);
  t = run<5120>(H, f, A, b, x, B); printf("occ=4/CU  %.3f ms  %.0f GB/s\n", t, bytes / t / 1e6);
  return 0;
}
