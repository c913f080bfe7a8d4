// occupancy_probe.hip -- how many one-wave workgroups a CU holds at once, for
// a given static LDS size and VGPR count (the wave-timeline finding of round
// 5: gi_dense held at most 11 waves per CU).
//
//   hipcc --offload-arch=gfx950 -O2 -std=c++20 tools/probe/occupancy_probe.hip -o /tmp/occ
//   /tmp/occ            -> one JSON line per (LDS bytes, VGPRs) case
//
// Every wave spins ~20 us on s_memrealtime, recording its start, end and
// HW_ID / XCC_ID; the host sweeps each CU's intervals for the largest number
// resident at once.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>

#define CHECK(x)                                                          \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                           \
    }                                                                     \
  } while (0)

__device__ __forceinline__ unsigned long long rtime() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// VG: force the allocation up to v[VG-1] (an asm clobber of that register)
template <int LDSB, int VG>
__global__ __launch_bounds__(64) void spin(unsigned long long *rec, int ticks) {
  __shared__ double lds[LDSB / 8];
  const unsigned long long t0 = rtime();
  unsigned hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  if constexpr (VG == 128) asm volatile("v_mov_b32 v127, 0" ::: "v127");
  if constexpr (VG == 168) asm volatile("v_mov_b32 v167, 0" ::: "v167");
  if constexpr (VG == 176) asm volatile("v_mov_b32 v175, 0" ::: "v175");
  lds[threadIdx.x] = (double)threadIdx.x;
  __builtin_amdgcn_wave_barrier();
  double acc = lds[(threadIdx.x + 1) & 63];
  unsigned long long t1 = rtime();
  while (t1 - t0 < (unsigned long long)ticks) {
    __builtin_amdgcn_s_sleep(2);
    t1 = rtime();
  }
  if (threadIdx.x == 0) {
    unsigned long long *r = rec + 4ull * blockIdx.x;
    r[0] = t0;
    r[1] = t1;
    r[2] = hw | ((unsigned long long)xcc << 32);
    r[3] = (unsigned long long)acc;
  }
}

// launch rate: `blocks` one-wave workgroups that each live `ticks` x 10 ns;
// kernel time by events, waves per microsecond over the whole chip
template <int LDSB, int VG>
int rate(unsigned long long *d, int blocks, int ticks) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((spin<LDSB, VG>), dim3(blocks), dim3(64), 0, 0, d, ticks);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((spin<LDSB, VG>), dim3(blocks), dim3(64), 0, 0, d, ticks);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, ms);
  }
  printf("{\"rate\": true, \"lds_bytes\": %d, \"vgprs\": %d, \"blocks\": %d, \"wave_us\": %.2f, \"kernel_ms\": %.4f, "
         "\"waves_per_us\": %.1f}\n",
         LDSB, VG, blocks, ticks / 100.0, best, blocks / (best * 1e3));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return 0;
}

template <int LDSB, int VG>
int run(unsigned long long *d, std::vector<unsigned long long> &h, int blocks) {
  hipLaunchKernelGGL((spin<LDSB, VG>), dim3(blocks), dim3(64), 0, 0, d, 2000);  // 20 us at 100 MHz
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  hipLaunchKernelGGL((spin<LDSB, VG>), dim3(blocks), dim3(64), 0, 0, d, 2000);
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
  std::map<unsigned long long, std::vector<std::pair<unsigned long long, int>>> ev;  // per CU
  std::map<unsigned long long, std::vector<std::pair<unsigned long long, int>>> evs;  // per SIMD
  for (int b = 0; b < blocks; ++b) {
    const unsigned long long t0 = h[4 * b], t1 = h[4 * b + 1], w = h[4 * b + 2];
    const unsigned hw = (unsigned)w, xcc = (unsigned)(w >> 32) & 15;
    const unsigned long long cu = ((unsigned long long)xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 7) |
                                  (((hw >> 8) & 15) << 2);
    const unsigned long long simd = cu | ((hw >> 4) & 3);
    ev[cu].push_back({t0, 1});
    ev[cu].push_back({t1, -1});
    evs[simd].push_back({t0, 1});
    evs[simd].push_back({t1, -1});
  }
  auto maxc = [](std::map<unsigned long long, std::vector<std::pair<unsigned long long, int>>> &m, int &lo, int &hi) {
    lo = 1 << 30;
    hi = 0;
    for (auto &kv : m) {
      auto &v = kv.second;
      std::sort(v.begin(), v.end(), [](auto &a, auto &b) { return a.first < b.first || (a.first == b.first && a.second < b.second); });
      int c = 0, mx = 0;
      for (auto &e : v) mx = std::max(mx, c += e.second);
      lo = std::min(lo, mx);
      hi = std::max(hi, mx);
    }
  };
  int clo, chi, slo, shi;
  maxc(ev, clo, chi);
  maxc(evs, slo, shi);
  printf("{\"lds_bytes\": %d, \"vgprs\": %d, \"cus\": %zu, \"cu_max_min\": %d, \"cu_max_max\": %d, "
         "\"simd_max_min\": %d, \"simd_max_max\": %d}\n",
         LDSB, VG, ev.size(), clo, chi, slo, shi);
  return 0;
}

int main() {
  const int blocks = 256 * 24;
  unsigned long long *d;
  CHECK(hipMalloc(&d, (size_t)blocks * 32));
  std::vector<unsigned long long> h((size_t)blocks * 4);
  int rc = 0;
  rc |= run<1024, 168>(d, h, blocks);
  rc |= run<12288, 168>(d, h, blocks);
  rc |= run<12544, 168>(d, h, blocks);
  rc |= run<12800, 168>(d, h, blocks);
  rc |= run<13056, 168>(d, h, blocks);
  rc |= run<13120, 168>(d, h, blocks);
  rc |= run<13312, 168>(d, h, blocks);
  rc |= run<13632, 168>(d, h, blocks);
  rc |= run<13632, 128>(d, h, blocks);
  rc |= run<1024, 128>(d, h, blocks);
  rc |= run<1024, 176>(d, h, blocks);
  CHECK(hipFree(d));
  // dispatch rate, in the kernel's own configuration and without LDS
  const int rb = 1 << 18;
  CHECK(hipMalloc(&d, (size_t)rb * 32));
  rc |= rate<13632, 168>(d, rb, 0);
  rc |= rate<13632, 168>(d, rb, 200);
  rc |= rate<13632, 168>(d, rb, 1800);
  rc |= rate<12288, 168>(d, rb, 1800);
  rc |= rate<1024, 128>(d, rb, 0);
  rc |= rate<1024, 128>(d, rb, 200);
  CHECK(hipFree(d));
  return rc;
}
