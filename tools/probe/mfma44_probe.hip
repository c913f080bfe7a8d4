// gfx950 v_mfma_f64_4x4x4_4b_f64: operand / result lane layout and issue cost.
// Layout: random A, B per lane, one MFMA; every hypothesis of where A(i,k),
// B(k,j) and C(i,j) sit inside a 16-lane block is checked on the host.
// Cost: s_memtime cycles of chains of independent / dependent MFMAs, and of
// MFMAs interleaved with independent v_fma_f64 in the same wave.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>

__global__ void layout_k(const double *a, const double *b, double *c) {
  const int l = threadIdx.x;
  double acc = 0.0;
  acc = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], acc, 0, 0, 0);
  c[l] = acc;
}

template <int MODE>
__global__ void cost_k(const double *in, double *out, long long *cyc, int iters) {
  const int l = threadIdx.x;
  double x = in[l], y = in[l + 64];
  double c0 = 0, c1 = 0, c2 = 0, c3 = 0, v0 = x, v1 = y, v2 = x + 1, v3 = y + 1;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    if constexpr (MODE == 0) {  // 4 independent accumulators
      c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, c3, 0, 0, 0);
    } else if constexpr (MODE == 1) {  // one dependent chain
      c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, c0, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, c0, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, c0, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, c0, 0, 0, 0);
    } else if constexpr (MODE == 2) {  // 4 independent MFMAs + 8 independent v_fma_f64
      c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, c0, 0, 0, 0);
      v0 = __builtin_fma(v0, x, y); v1 = __builtin_fma(v1, x, y);
      c1 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, c1, 0, 0, 0);
      v2 = __builtin_fma(v2, x, y); v3 = __builtin_fma(v3, x, y);
      c2 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, c2, 0, 0, 0);
      v0 = __builtin_fma(v0, x, y); v1 = __builtin_fma(v1, x, y);
      c3 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, c3, 0, 0, 0);
      v2 = __builtin_fma(v2, x, y); v3 = __builtin_fma(v3, x, y);
    } else {  // the 8 v_fma_f64 alone
      v0 = __builtin_fma(v0, x, y); v1 = __builtin_fma(v1, x, y);
      v2 = __builtin_fma(v2, x, y); v3 = __builtin_fma(v3, x, y);
      v0 = __builtin_fma(v0, x, y); v1 = __builtin_fma(v1, x, y);
      v2 = __builtin_fma(v2, x, y); v3 = __builtin_fma(v3, x, y);
    }
  }
  long long t1 = clock64();
  out[l] = c0 + c1 + c2 + c3 + v0 + v1 + v2 + v3;
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

// Pipe sharing: 8 waves per workgroup (two per SIMD: waves w and w + 4 share
// one); waves 0-3 run independent 4x4x4 f64 MFMAs, waves 4-7 independent
// v_fma_f64 chains.  MODE 0: MFMA waves only, 1: FMA waves only, 2: both.
// Concurrent time ~ max of the two: separate pipes; ~ their sum: shared.
template <int MODE>
__global__ __launch_bounds__(512) void share_k(const double *in, double *out, long long *cyc, int iters) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  double x = in[l], y = in[l + 64];
  double c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0, c6 = 0, c7 = 0;
  const bool mf = w < 4;
  const bool run = MODE == 2 || (MODE == 0 && mf) || (MODE == 1 && !mf);
  long long t0 = clock64();
  if (run) {
    if (mf) {
      for (int i = 0; i < iters; ++i) {
        c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, c3, 0, 0, 0);
      }
    } else {
      for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          c0 = __builtin_fma(c0, x, y); c1 = __builtin_fma(c1, x, y); c2 = __builtin_fma(c2, x, y);
          c3 = __builtin_fma(c3, x, y); c4 = __builtin_fma(c4, x, y); c5 = __builtin_fma(c5, x, y);
          c6 = __builtin_fma(c6, x, y); c7 = __builtin_fma(c7, x, y);
        }
      }
    }
  }
  long long t1 = clock64();
  out[threadIdx.x] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
  if (l == 0) cyc[w] = run ? t1 - t0 : 0;
}

int main() {
  double ha[64], hb[64], hc[64];
  srand(7);
  for (int i = 0; i < 64; ++i) {
    ha[i] = (rand() % 1000) / 100.0 - 5;
    hb[i] = (rand() % 1000) / 100.0 - 5;
  }
  double *da, *db, *dc;
  hipMalloc(&da, 512 * 2);
  hipMalloc(&db, 512);
  hipMalloc(&dc, 512);
  hipMemcpy(da, ha, 512, hipMemcpyHostToDevice);
  hipMemcpy(db, hb, 512, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(layout_k, dim3(1), dim3(64), 0, 0, da, db, dc);
  hipMemcpy(hc, dc, 512, hipMemcpyDeviceToHost);
  // lane of (block, r, c) when the three 2-bit fields occupy lane bits
  // (0-1, 2-3, 4-5) in the order given by permutation p of {block, r, c}
  const int perms[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};
  const char *fld[3] = {"blk", "r", "c"};
  auto pos = [&](int p, int blk, int r, int c) {
    const int v[3] = {blk, r, c};
    return v[perms[p][0]] + 4 * v[perms[p][1]] + 16 * v[perms[p][2]];
  };
  int found = 0;
  for (int oa = 0; oa < 6; ++oa)
    for (int ob = 0; ob < 6; ++ob)
      for (int oc = 0; oc < 6; ++oc) {
        double err = 0;
        for (int blk = 0; blk < 4; ++blk)
          for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
              double s = 0;
              for (int k = 0; k < 4; ++k) s += ha[pos(oa, blk, i, k)] * hb[pos(ob, blk, k, j)];
              err = fmax(err, fabs(s - hc[pos(oc, blk, i, j)]));
            }
        if (err < 1e-9) {
          printf("MATCH: lane bits (0-1,2-3,4-5) = A(i,k): %s,%s,%s  B(k,j): %s,%s,%s  C(i,j): %s,%s,%s\n",
                 fld[perms[oa][0]], fld[perms[oa][1]], fld[perms[oa][2]], fld[perms[ob][0]], fld[perms[ob][1]],
                 fld[perms[ob][2]], fld[perms[oc][0]], fld[perms[oc][1]], fld[perms[oc][2]]);
          ++found;
        }
      }
  for (int l = 0; l < 64; ++l) printf("lane %2d a %6.2f b %6.2f c %9.4f\n", l, ha[l], hb[l], hc[l]);
  printf("layout hypotheses matching: %d\n", found);
  long long *dcyc, hcyc[4];
  hipMalloc(&dcyc, 64);
  const int iters = 4096;
  const char *mn[4] = {"4 independent MFMA", "4 dependent MFMA", "4 indep MFMA + 8 indep v_fma_f64", "8 v_fma_f64 alone"};
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(cost_k<0>, dim3(1), dim3(64), 0, 0, da, dc, dcyc + 0, iters);
    hipLaunchKernelGGL(cost_k<1>, dim3(1), dim3(64), 0, 0, da, dc, dcyc + 1, iters);
    hipLaunchKernelGGL(cost_k<2>, dim3(1), dim3(64), 0, 0, da, dc, dcyc + 2, iters);
    hipLaunchKernelGGL(cost_k<3>, dim3(1), dim3(64), 0, 0, da, dc, dcyc + 3, iters);
    hipDeviceSynchronize();
    hipMemcpy(hcyc, dcyc, 32, hipMemcpyDeviceToHost);
    if (rep == 1)
      for (int m = 0; m < 4; ++m) printf("cost: %-36s %.2f cycles per loop trip\n", mn[m], (double)hcyc[m] / iters);
  }
  {
    long long *dc8, h8[8];
    double *dout;
    hipMalloc(&dc8, 64);
    hipMalloc(&dout, 512 * 8);
    const int it2 = 2048;
    const char *nm2[3] = {"MFMA waves alone (4 x 4x4x4 f64 per trip)", "FMA waves alone (16 v_fma_f64 per trip)",
                          "both, one of each per SIMD"};
    for (int rep = 0; rep < 2; ++rep)
      for (int m = 0; m < 3; ++m) {
        if (m == 0) hipLaunchKernelGGL(share_k<0>, dim3(1), dim3(512), 0, 0, da, dout, dc8, it2);
        if (m == 1) hipLaunchKernelGGL(share_k<1>, dim3(1), dim3(512), 0, 0, da, dout, dc8, it2);
        if (m == 2) hipLaunchKernelGGL(share_k<2>, dim3(1), dim3(512), 0, 0, da, dout, dc8, it2);
        hipDeviceSynchronize();
        hipMemcpy(h8, dc8, 64, hipMemcpyDeviceToHost);
        if (rep == 1)
          printf("share: %-44s MFMA waves %.1f, FMA waves %.1f cycles per trip\n", nm2[m],
                 (double)(h8[0] + h8[1] + h8[2] + h8[3]) / 4 / it2, (double)(h8[4] + h8[5] + h8[6] + h8[7]) / 4 / it2);
      }
  }
  return 0;
}
