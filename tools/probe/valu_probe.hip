// Diagnostic only: VALU issue rates and dependent-chain latencies on gfx950
// for the instruction classes of the active-set kernels (fp64 FMA / mul,
// fp32 FMA, v_mov_b64_dpp, v_mov_b32_dpp, v_cndmask, ds_read/ds_write round
// trip).  Prints cycles per wave-instruction (throughput, many waves per SIMD)
// and cycles per dependent instruction (latency, one wave per SIMD).
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int ITERS = 4096;

// throughput: 8 independent chains per lane
template <int KIND>
__global__ __launch_bounds__(64) void thr_kernel(double *out, double seed, long long *clk) {
  double a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  float fa[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) fa[i] = (float)a[i];
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 pk[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) pk[i] = (f2){fa[i], fa[i] + 1.0f};
  const f2 pkm = {0.999f, 0.999f}, pka = {1e-3f, 1e-3f};
  const long long t0 = wall_clock64();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (KIND == 0) a[i] = __builtin_fma(a[i], 0.999, 1e-3);
      if constexpr (KIND == 1) a[i] = a[i] * 0.999;
      if constexpr (KIND == 2) fa[i] = __builtin_fmaf(fa[i], 0.999f, 1e-3f);
      if constexpr (KIND == 3) a[i] = __builtin_amdgcn_mov_dpp(a[i], 0x151, 0xF, 0xF, true);  // row_newbcast:1
      if constexpr (KIND == 4) a[i] = __builtin_amdgcn_mov_dpp(a[i], 0x121, 0xF, 0xF, true);  // row_ror:1
      if constexpr (KIND == 5) a[i] = __builtin_amdgcn_rcp(a[i]);
      if constexpr (KIND == 6)  // v_fmac_f64 with a row_newbcast DPP source (a[i] written 7 instructions earlier)
        asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(a[i]), "v"(0.999));
      if constexpr (KIND == 7)  // v_pk_fma_f32 (two fp32 FMAs per lane), 8 independent packed chains
        asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(pk[i]) : "v"(pkm), "v"(pka));
      if constexpr (KIND == 8)  // the unfused pair: v_mov_b64_dpp + v_fmac_f64
        a[i] = __builtin_fma(__builtin_amdgcn_mov_dpp(a[i], 0x151, 0xF, 0xF, true), 0.999, a[i]);
    }
    asm volatile("" ::: "memory");
  }
  const long long t1 = wall_clock64();
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += a[i] + fa[i] + pk[i].x + pk[i].y;
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
}

// latency: one dependent chain
template <int KIND>
__global__ __launch_bounds__(64) void lat_kernel(double *out, double seed, long long *clk) {
  double a = seed + threadIdx.x;
  __shared__ double sh[64];
  const long long t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (KIND == 0) a = __builtin_fma(a, 0.999, 1e-3);
    if constexpr (KIND == 1) a = __builtin_amdgcn_mov_dpp(a, 0x151, 0xF, 0xF, true);
    if constexpr (KIND == 2) a = __builtin_fmin(a, __builtin_amdgcn_mov_dpp(a, 0x121, 0xF, 0xF, true));
    if constexpr (KIND == 3) {
      sh[threadIdx.x] = a;
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      a = sh[(threadIdx.x + 1) & 63] + 1.0;
    }
    if constexpr (KIND == 4) a = __builtin_amdgcn_rcp(a);
    if constexpr (KIND == 5)  // accumulator chain of v_fmac_f64_dpp (the DPP source is a fixed register)
      asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf" : "+v"(a) : "v"(seed), "v"(0.999));
    if constexpr (KIND == 6)  // the same chain on plain v_fmac_f64
      asm volatile("v_fmac_f64 %0, %1, %2" : "+v"(a) : "v"(seed), "v"(0.999));
  }
  const long long t1 = clock64();
  out[blockIdx.x * 64 + threadIdx.x] = a;
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
}

// accuracy of the raw hardware estimates v_rcp_f64 / v_rsq_f64 (relative to
// IEEE division / sqrt) over inputs spread across many binades
__global__ void acc_kernel(double *err) {
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long z = 0x9E3779B97F4A7C15ull * (t + 1);
  double er = 0.0, es = 0.0;
  for (int i = 0; i < 256; ++i) {
    z ^= z >> 33; z *= 0xff51afd7ed558ccdull; z ^= z >> 33;
    const double m = 1.0 + (double)(z >> 12) * 0x1p-52;
    const double x = __builtin_ldexp(m, (int)((z >> 3) % 200) - 100);
    const double r = __builtin_amdgcn_rcp(x), q = __builtin_amdgcn_rsq(x);
    er = fmax(er, fabs(r * x - 1.0));
    es = fmax(es, fabs(q * sqrt(x) - 1.0));
  }
  atomicMax((unsigned long long *)&err[0], __double_as_longlong(er));
  atomicMax((unsigned long long *)&err[1], __double_as_longlong(es));
}

int main() {
  double *out;
  long long *clk;
  const int blocks = 256 * 4 * 8;  // 8 waves per SIMD
  hipMalloc(&out, sizeof(double) * blocks * 64);
  hipMalloc(&clk, sizeof(long long));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char *tn[] = {"fma_f64", "mul_f64", "fma_f32", "mov_b64_dpp_bcast", "mov_dpp_ror_f64", "rcp_f64",
                      "fmac_f64_dpp_bcast", "pk_fma_f32", "mov_b64_dpp+fma_f64"};
  auto thr = [&](auto kern, const char *name) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, out, 1.0, clk);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, out, 1.0, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    // cycles per wave-instruction per SIMD at 2.4 GHz
    const double insts = (double)blocks * ITERS * 8;  // wave-instructions
    const double cyc = ms * 1e-3 * 2.4e9 * 1024 / insts;
    printf("{\"probe\": \"throughput\", \"op\": \"%s\", \"ms\": %.3f, \"cycles_per_wave_inst_per_simd\": %.2f}\n", name,
           ms, cyc);
  };
  thr(thr_kernel<0>, tn[0]);
  thr(thr_kernel<1>, tn[1]);
  thr(thr_kernel<2>, tn[2]);
  thr(thr_kernel<3>, tn[3]);
  thr(thr_kernel<4>, tn[4]);
  thr(thr_kernel<5>, tn[5]);
  thr(thr_kernel<6>, tn[6]);
  thr(thr_kernel<7>, tn[7]);
  thr(thr_kernel<8>, tn[8]);
  const char *ln[] = {"fma_f64_dep", "mov_b64_dpp_dep", "dpp_ror+min_f64_dep", "ds_write+ds_read_f64_dep",
                      "rcp_f64_dep", "fmac_f64_dpp_acc_dep", "fmac_f64_acc_dep"};
  auto lat = [&](auto kern, const char *name) {
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, out, 1.0, clk);
    hipDeviceSynchronize();
    long long c;
    hipMemcpy(&c, clk, sizeof c, hipMemcpyDeviceToHost);
    printf("{\"probe\": \"latency\", \"op\": \"%s\", \"cycles_per_step\": %.2f}\n", name, (double)c / ITERS);
  };
  lat(lat_kernel<0>, ln[0]);
  lat(lat_kernel<1>, ln[1]);
  lat(lat_kernel<2>, ln[2]);
  lat(lat_kernel<3>, ln[3]);
  lat(lat_kernel<4>, ln[4]);
  lat(lat_kernel<5>, ln[5]);
  lat(lat_kernel<6>, ln[6]);
  double *err;
  hipMalloc(&err, 2 * sizeof(double));
  hipMemset(err, 0, 2 * sizeof(double));
  hipLaunchKernelGGL(acc_kernel, dim3(4096), dim3(256), 0, 0, err);
  double he[2];
  hipMemcpy(he, err, sizeof he, hipMemcpyDeviceToHost);
  printf("{\"probe\": \"accuracy\", \"rcp_f64_max_rel_err\": %.3e, \"rsq_f64_max_rel_err\": %.3e, \"log2\": [%.2f, %.2f]}\n",
         he[0], he[1], log2(he[0]), log2(he[1]));
  return 0;
}
