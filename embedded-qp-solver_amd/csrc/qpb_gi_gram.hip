// qpb_gi_gram.hip -- active-set QP kernel for 32 < n <= 128, m <= 256 (gfx950).
//
// BASELINE configs[3] (n = 128, m = 256).  The same dual active-set method as
// qpb_gi.hip (Goldfarb & Idnani) with D = A L^{-T} fixed after the setup and
// the active set's factorisation kept beside it:
//
//   setup   H = L L^T (blocked, right-looking, 16 x 16 tiles: trailing updates
//           and panel solves on the fp64 matrix cores, v_mfma_f64_16x16x4_f64),
//           D = A L^{-T} (blocked forward substitution, every tile product and
//           the diagonal-tile solves on the matrix cores), y = L^{-1} f,
//           s = b + D y (the slack of the unconstrained minimiser,
//           test/qp_ref.py:35's answer).
//   iterate for the selected row p (most violated normalised slack), with
//           D_W^T = Q1^T R (Q1: orthonormal rows, R upper triangular, kept as
//           Z = R^{-1}):
//           u = D[p,:], d = Q1 u, w = u - Q1^T d (|w|^2 = |d2|^2 of G-I),
//           r = Z d, slack direction D w, partial step t1 (ratio test on the
//           multipliers), full step t2 = -s_p / |w|^2, s += t D w.
//           ADD p: Q1 gains the row w / |w|, Z the column [-r / |w|; 1 / |w|].
//           DROP k: Givens rotations zero row k of Z (columns k .. q-1), the
//           same rotations on Q1's rows, row k of Z goes.  Every phase is a
//           parallel pass; no triangular solve and nothing O(q^2) per ADD.
//   finish  x = -L^{-T} (y + D^T lam) (KKT stationarity, lam by row), L
//           restored from the scratch.
//
// Replaces, batched, the reference's dense kernels on this path: matrix_mult
// (matrix_ops.c:235-271) as the MFMA tile products and the GEMVs, the LU /
// explicit inverse (:487-630) by the Cholesky and the triangular solves, the
// vector ops (:158-411) fused into the iteration.
//
// One QP per 512-thread workgroup (8 wavefronts, two per SIMD), one
// workgroup per CU; the workgroups pull QP indices from an atomic queue, so
// QPs with long iteration counts do not hold up a static partition.
// Registers: wave w owns rows 32w..32w+31 of D as two 16-row tiles (t) of
// eight 16 x 16 column tiles (k) in the matrix cores' C/D layout, which is
// also their B-operand layout: lane (g = l >> 4, j = l & 15) holds
// D[32w + 16t + j][16k + g + 4r] (element r), i.e. in each row tile row j,
// the 32 columns congruent to g mod 4.  A row dot product is 32 FMAs and two
// cross-group butterfly steps.
// LDS (160 KiB): the packed triangle (L in setup and finish, Z = R^{-1} by
// columns in the loop), the diagonal-tile inverses (setup) / the rows of Q1
// (loop; rows past QL live in a per-workgroup global scratch), vectors.
#include "qpb_common.h"
#include "qpb.h"

namespace qpb {
namespace gram {

constexpr int NB = 128;                // max (padded) n
constexpr int MB = 256;                // max m: 16 rows per wavefront
constexpr int NT = 512;   // 8 wavefronts, two per SIMD (256 VGPRs each)
constexpr int NWV = NT / 64;
constexpr int RT = MB / 16 / NWV;  // 16-row tiles of D per wavefront (2)
constexpr int LP = NB * (NB + 1) / 2;  // packed triangle, 8256 doubles
constexpr int LDS_D = 20480;           // 160 KiB
constexpr int PV = 4 * 34;  // a padded permuted vector (see pad())
constexpr int NBUF = 2136;
constexpr int OFF_TRI = 0;
constexpr int OFF_ROWS = LP;  // diagonal-tile inverses (setup) / D_W rows (loop)
constexpr int OFF_BUF = LDS_D - NBUF;
// Q1 rows in LDS at stride QS: 2 QS = 32 mod 64 dwords, so the row-adjacent
// lane groups of one b64 read (the d and w phases) hit opposite bank halves
constexpr int QS = 144;
constexpr int QL = (OFF_BUF - OFF_ROWS) / QS;  // Q1 rows in LDS (70)
// Permuted vectors (u, w, y) keep lane group g's 32 entries at 34 g: the four
// groups' b128 reads then start 4 banks apart instead of on the same banks.
constexpr int B_CAND = OFF_BUF;                // per wave: its most violated row of D (PV each)
constexpr int B_CSP = B_CAND + NWV * PV;       // per wave: that row's slack
constexpr int B_W = B_CSP + NWV;               // w (padded permuted)
constexpr int B_V = B_W + PV;                  // per-wave candidate row norms (NWV) and DROP scratch (row k of Z, at NB); lambda scatter at the end
constexpr int B_R = B_V + MB;                  // r by position
constexpr int B_CB = B_R + NB;                 // d = Q1 u by position
constexpr int B_LAM = B_CB + NB;               // multipliers by position
constexpr int B_Y = B_LAM + NB;                // y (padded permuted), then y + D_W^T lam
constexpr int B_RED = B_Y + PV;                // selection keys, partial reductions, scalars
constexpr int B_INT = B_RED + 32;              // ints: flags, queue slot, mask words (64)
constexpr int B_IAM = B_INT + 32;              // ints: constraint index by position (128)
static_assert(B_IAM + 64 == LDS_D, "LDS layout");
// diagonal-tile inverses (setup): 16 x 16 at row stride LIS = 17, so the
// lanes of a b64 read, one row each, start 34 dwords apart (conflict-free);
// at stride 16 every read was an 8-way bank conflict
constexpr int LIS = 17;
constexpr int LIT = 16 * LIS;  // doubles per tile
static_assert(OFF_ROWS + 8 * LIT <= OFF_BUF, "diagonal-tile inverses fit the row area");
// B_RED slots
constexpr int R_KEY = 0;    // per-wave selection keys (NWV)
constexpr int R_T1 = 8;     // per-wave (ratio min, argmin position) pairs (2 NWV)
constexpr int R_ND2 = 24;   // per-wave partial |w|^2 (NWV)
constexpr double kDepTol = 1e-24;
constexpr long long SCRATCH = LP + (long long)(NB - QL) * NB;  // doubles per workgroup

using d4 = __attribute__((__vector_size__(4 * sizeof(double)))) double;

__device__ __forceinline__ int tri(int i, int j) { return ((i * (i + 1)) >> 1) + j; }
// column c -> its place in the permuted vector layout (lane group c & 3 reads
// a contiguous 32-double block in the order of its registers)
__device__ __forceinline__ int perm(int c) { return ((c & 3) << 5) + ((c >> 4) << 2) + ((c >> 2) & 3); }
// a permuted index 0..127 -> its slot in the padded layout
__device__ __forceinline__ int pad(int c) { return c + 2 * (c >> 5); }
__device__ __forceinline__ double mfma(double a, double b, d4 &c) {
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  return 0.0;
}
__device__ __forceinline__ double readlane_d(double v, int lane) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const int lo = __builtin_amdgcn_readlane((int)(unsigned)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(unsigned)(b >> 32), lane);
  return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double pack_key256(double v, int idx) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  return __builtin_bit_cast(double, (b & ~255ull) | (unsigned long long)idx);
}
__device__ __forceinline__ int key_index256(double k) { return (int)(__builtin_bit_cast(unsigned long long, k) & 255ull); }
// min over the 64 lanes of a wave (exact), on every lane
__device__ __forceinline__ double wave_min(double v) {
  v = row_min(v);
  return __builtin_fmin(__builtin_fmin(readlane_d(v, 0), readlane_d(v, 16)),
                        __builtin_fmin(readlane_d(v, 32), readlane_d(v, 48)));
}
__device__ __forceinline__ double wave_sum(double v) {
  v = row_sum(v);
  return (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
}
// sum over the four lane groups (lanes j, j+16, j+32, j+48): the same value,
// bitwise, on all four.  gfx950's v_permlane32_swap / v_permlane16_swap with
// one register as both operands hand every lane the pair {value of the lower
// partner, value of the upper partner} (lanes l, l ^ 32, resp. l, l ^ 16;
// tools/probe/permlane_probe.hip), so both partners add the same two numbers
// in the same order.
__device__ __forceinline__ double pair32(double v) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
  const double x = __builtin_bit_cast(double, ((unsigned long long)hi[0] << 32) | lo[0]);
  const double y = __builtin_bit_cast(double, ((unsigned long long)hi[1] << 32) | lo[1]);
  return x + y;
}
__device__ __forceinline__ double pair16(double v) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
  const double x = __builtin_bit_cast(double, ((unsigned long long)hi[0] << 32) | lo[0]);
  const double y = __builtin_bit_cast(double, ((unsigned long long)hi[1] << 32) | lo[1]);
  return x + y;
}
__device__ __forceinline__ double group_sum(double v) { return pair16(pair32(v)); }
// this lane's rows of D (one per tile) against a permuted vector in LDS
__device__ __forceinline__ void row_dot(const double (&E)[RT][8][4], const double *vp, double (&out)[RT]) {
  // the 16 lanes of a group need the same 32 entries: lane j reads entries
  // 2j, 2j + 1 (one b128 instead of sixteen), and the FMAs take entry 4k + c
  // from lane 2k + c / 2 by a fused row_newbcast (same products, same order)
  const double2 u = *reinterpret_cast<const double2 *>(&vp[2 * (threadIdx.x & 15)]);
  double a[RT][4];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) a[t][r] = 0.0;
  unroll<8>([&](auto K) {
    constexpr int k = K;
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      fmac_bc<2 * k>(a[t][0], u.x, E[t][k][0]);
      fmac_bc<2 * k>(a[t][1], u.y, E[t][k][1]);
      fmac_bc<2 * k + 1>(a[t][2], u.x, E[t][k][2]);
      fmac_bc<2 * k + 1>(a[t][3], u.y, E[t][k][3]);
    }
  });
#pragma unroll
  for (int t = 0; t < RT; ++t) out[t] = group_sum((a[t][0] + a[t][1]) + (a[t][2] + a[t][3]));
}
// symmetric packed access
__device__ __forceinline__ double sym(const double *P, int i, int j) { return i >= j ? P[tri(i, j)] : P[tri(j, i)]; }

// ---------------------------------------------------------------- Cholesky
// H (n x n, padded to 16 T with the identity) from global memory into the
// packed lower triangle, factorised in place: blocked right-looking over
// 16 x 16 tiles.  The diagonal tile is factorised by wavefront 0 (lane i owns
// row i, pivot rows by DPP broadcast as in qpb_gi.hip) and inverted (lane j
// solves column j); the panel below it is multiplied by that inverse and the
// trailing tiles updated on the matrix cores.  Returns false if a pivot <= 0.
template <class CLK>
__device__ __forceinline__ bool cholesky(double *lds, const double *__restrict__ Hq, int n, int T, int tid, CLK &clk) {
  double *Lp = lds + OFF_TRI;
  double *LI = lds + OFF_ROWS;
  int *flags = reinterpret_cast<int *>(lds + B_INT);
  const int l = tid & 63, wv = tid >> 6;  // tid: the caller's opaque thread id
  const int nb = 16 * T;
  {
    // rows wv, wv + 8, ... (lanes along the columns: coalesced); every load
    // is issued before the first store, one memory round trip per QP.  The
    // loads are unconditional (addresses clamped into the row, so no extra
    // lines): a guarded load becomes a branch with its own wait.
    double h[NB / NWV][2];
#pragma unroll
    for (int u = 0; u < NB / NWV; ++u) {
      const int r = wv + NWV * u;
      const int rr = r < n ? r : n - 1;
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int c = l + 64 * h2;
        const double v = Hq[rr * n + (c <= rr ? c : rr)];
        h[u][h2] = (r < n && c <= r) ? v : (r == c ? 1.0 : 0.0);
      }
    }
#pragma unroll
    for (int u = 0; u < NB / NWV; ++u) {
      const int r = wv + NWV * u;
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int c = l + 64 * h2;
        if (r < nb && c <= r) Lp[tri(r, c)] = h[u][h2];
      }
    }
  }
  if (tid == 0) flags[0] = 0;
  __syncthreads();
  clk.tick(11);
  // the diagonal tile K, on wavefront 0
  auto factor_diag = [&](int K) {
    int i = l & 15;
    asm volatile("" : "+v"(i));  // opaque per step: nothing lane-dependent is hoisted and kept live
    const int r0 = 16 * K;
    // lane i: row i of the tile (a, the full symmetric row) and row i of
    // the identity (e): the sweep turns e into row i of L^{-T}, i.e.
    // column i of the tile inverse, alongside the factorisation
    double a[16], e[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      a[j] = j <= i ? Lp[tri(r0 + i, r0 + j)] : Lp[tri(r0 + j, r0 + i)];
      e[j] = j == i ? 1.0 : 0.0;
    }
    bool ok = true;
    unroll<16>([&](auto Kc) {
      constexpr int k = Kc;
      // a step boundary the scheduler keeps (as qpb_gi.hip's sweep): the
      // previous step's writes of a[j] (and, at k = 0, the selects above)
      // stay ahead of this step's broadcast and rsq chain, well over the two
      // wait states the v_fmac_f64_dpp reads of a[j] need (hipcc does not pad
      // inline asm; tests/test_dpp_hazards.py checks the built objects)
      __builtin_amdgcn_sched_barrier(0);
      // pivot row k of the Schur complement = column k (symmetry): lane k's
      // entries, broadcast by DPP
      const double akk = bc<k>(a[k]);
      ok = ok && (akk > 0.0);
      const double ik = rsq1(akk);  // hardware estimate + one Newton step (qpb_common.h)
      const double ik2 = ik * ik;
      const double c = a[k] * ik2;
      const double ne2 = -(e[k] * ik2);
      e[k] *= ik;
      const double nc = -c;
      // broadcasts fused into v_fmac_f64_dpp (the pivot row read straight
      // from lane k); the e update reads lane k's a[j] before the a update of
      // the same j writes it (volatile asm keeps the order); a[j] was last
      // written in the previous step, well over two instructions before (the
      // DPP read hazard)
      unroll<15 - k>([&](auto J) {
        constexpr int j = k + 1 + J;
        fmac_bc<k>(e[j], a[j], ne2);
        fmac_bc<k>(a[j], a[j], nc);
      });
      a[k] *= ik;
    });
    if (l < 16) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if (j <= i) Lp[tri(r0 + i, r0 + j)] = a[j];
        LI[K * LIT + j * LIS + i] = e[j];
      }
    }
    if (l == 0 && !ok) flags[0] = 1;
      };
  const int li = l & 15, lk = l >> 4;
  // one tile update (I, J) -= L[I, K] L[J, K]^T on the matrix cores (two
  // tiles at a time: independent MFMA chains); `on` masks the second one
  auto tile_update2 = [&](int K, const int (&I)[2], const int (&J)[2], const bool (&on)[2]) {
    d4 acc[2];
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * I[h2] + lk + 4 * r, col = 16 * J[h2] + li;
        acc[h2][r] = row >= col ? Lp[tri(row, col)] : 0.0;
      }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2)
        mfma(-Lp[tri(16 * I[h2] + li, 16 * K + 4 * s + lk)], Lp[tri(16 * J[h2] + li, 16 * K + 4 * s + lk)], acc[h2]);
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * I[h2] + lk + 4 * r, col = 16 * J[h2] + li;
        if (on[h2] && row >= col) Lp[tri(row, col)] = acc[h2][r];
      }
  };
  if (wv == 0) factor_diag(0);
  __syncthreads();
  for (int K = 0; K < T; ++K) {
    clk.tick(12);
    // panel: L[I, K] = H~[I, K] Linv_K^T, one tile per wavefront
    if (wv < T - K - 1) {
      const int I = K + 1 + wv;
      d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < 4; ++s)
        mfma(Lp[tri(16 * I + li, 16 * K + 4 * s + lk)], LI[K * LIT + li * LIS + 4 * s + lk], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) Lp[tri(16 * I + lk + 4 * r, 16 * K + li)] = acc[r];
    }
    __syncthreads();
    clk.tick(13);
    if (K + 1 < T) {
      // look-ahead: wavefront 0 updates the next diagonal tile and factorises
      // it while the others update the rest of the trailing matrix
      const int nr = T - K - 1, ntile = nr * (nr + 1) / 2 - 1;  // all but (K+1, K+1)
      if (wv == 0) {
        const int I[2] = {K + 1, K + 1}, J[2] = {K + 1, K + 1};
        const bool on[2] = {true, false};
        tile_update2(K, I, J, on);
        wave_lds_sync();
        factor_diag(K + 1);
      } else if (wv != 4) {
        // waves 1-3, 5-7: wave 4 shares wavefront 0's SIMD and stays idle, so
        // the diagonal factorisation (the critical path) keeps its issue slots
        const int wr = wv < 4 ? wv - 1 : wv - 2;
        constexpr int NTW = NWV - 2;
        for (int t0 = wr; t0 < ntile; t0 += 2 * NTW) {
          int I[2], J[2];
          bool on[2];
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            const int t = t0 + NTW * h2;
            on[h2] = t < ntile;
            // tiles in row-major lower order after (K+1, K+1): index t + 1
            const int tt = (on[h2] ? t : t0) + 1;
            int i = (int)((__builtin_sqrt(8.0 * tt + 1.0) - 1.0) * 0.5);
            if (tri(i + 1, 0) <= tt) ++i;
            if (tri(i, 0) > tt) --i;
            J[h2] = tt - tri(i, 0) + K + 1;
            I[h2] = i + K + 1;
          }
          tile_update2(K, I, J, on);
        }
      }
      __syncthreads();
    }
    clk.tick(14);
  }
  return flags[0] == 0;
}

// Lane-parallel triangular solves with the packed L on one wavefront: lane l
// owns entries l and l + 64 (a0, a1: right-hand side in, solution out).
// Step i broadcasts the finished entry i (v_readlane with a constant lane) and
// every later entry takes its update; the steps are unrolled over the whole
// padded size (entries past nb have zero rows), L prefetched 16 steps at a
// time, so only the broadcast chain is serial.  A finished entry is never
// touched again (its later coefficients are zero), so the solution is the
// accumulator times 1 / L_ii at the end.
__device__ __forceinline__ void solve_lower(const double *Lp, int nb, int l, double &a0, double &a1) {
  const double id0 = l < nb ? rcp(Lp[tri(l, l)]) : 0.0;
  const double id1 = l + 64 < nb ? rcp(Lp[tri(l + 64, l + 64)]) : 0.0;
  unroll<8>([&](auto C) {
    constexpr int i0 = 16 * C;
    double L0[16], L1[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
      const int i = i0 + jj;
      L0[jj] = (i0 < 64 && l > i && l < nb) ? Lp[tri(l, i)] : 0.0;
      L1[jj] = (l + 64 > i && l + 64 < nb) ? Lp[tri(l + 64, i)] : 0.0;
    }
    unroll<16>([&](auto J) {
      constexpr int i = i0 + J;
      if constexpr (i < 64) {
        const double yi = readlane_d(a0 * id0, i);
        a0 = __builtin_fma(-L0[J], yi, a0);
        a1 = __builtin_fma(-L1[J], yi, a1);
      } else {
        const double yi = readlane_d(a1 * id1, i - 64);
        a1 = __builtin_fma(-L1[J], yi, a1);
      }
    });
  });
  a0 *= id0;
  a1 *= id1;
}
// L^T x = v (backward)
__device__ __forceinline__ void solve_upper(const double *Lp, int nb, int l, double &a0, double &a1) {
  const double id0 = l < nb ? rcp(Lp[tri(l, l)]) : 0.0;
  const double id1 = l + 64 < nb ? rcp(Lp[tri(l + 64, l + 64)]) : 0.0;
  unroll<8>([&](auto C) {
    constexpr int i1 = 112 - 16 * C;
    double L0[16], L1[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
      const int i = i1 + jj;
      L0[jj] = (l < i && i < nb) ? Lp[tri(i, l)] : 0.0;
      L1[jj] = (i1 >= 64 && l + 64 < i && i < nb) ? Lp[tri(i, l + 64)] : 0.0;
    }
    unroll<16>([&](auto J) {
      constexpr int i = i1 + 15 - J;
      if constexpr (i >= 64) {
        const double xi = readlane_d(a1 * id1, i - 64);
        a0 = __builtin_fma(-L0[15 - J], xi, a0);
        a1 = __builtin_fma(-L1[15 - J], xi, a1);
      } else {
        const double xi = readlane_d(a0 * id0, i);
        a0 = __builtin_fma(-L0[15 - J], xi, a0);
      }
    });
  });
  a0 *= id0;
  a1 *= id1;
}

// ------------------------------------------------------- Q1 row storage
struct Rows {
  double *lds;  // rows 0..QL-1, stride QS
  double *gl;   // rows QL.. (per-workgroup global scratch), stride NB
  __device__ __forceinline__ double *row(int j) const { return j < QL ? lds + j * QS : gl + (j - QL) * NB; }
};

// ------------------------------------------------------------------ kernel
// BOX: lb <= x <= ub with A = [I; -I] implicit (qpb_solve_box for 32 < n <= 128):
// Ag = lb, bg = ub (n per QP, either may be NULL: absent bounds), m = 2n; the
// rows of A are generated where they are loaded (D = A L^{-T} is formed as for
// a dense A; nothing else reads A)
template <bool STAMP, bool BOX = false>
__global__ __launch_bounds__(NT, 1) void gi_gram_kernel(
    const double *__restrict__ Hg, const double *__restrict__ fg, const double *__restrict__ Ag,
    const double *__restrict__ bg, double *__restrict__ xg, double *__restrict__ lamg, uint32_t *__restrict__ actg,
    int32_t *__restrict__ statg, int32_t *__restrict__ itg, int n, int m, long long batch, int max_iter,
    double feas_tol, int *__restrict__ queue, double *__restrict__ scratch, unsigned long long *__restrict__ dbg) {
  __shared__ double lds[LDS_D];
  // diagnostic build: s_memrealtime section stamps (0 Cholesky, 1 D, 2 y and
  // s, 3 select + v, 4 r + ratio, 5 w, 6 step + update, 7 outputs, 8 L again,
  // 9 x, 10 queue)
  SectionClock<STAMP> clk;
  double *Lp = lds + OFF_TRI;  // L, then Z = R^{-1} (packed by columns)
  double *LI = lds + OFF_ROWS;
  double *wb = lds + B_W, *vb = lds + B_V, *rb = lds + B_R, *lamb = lds + B_LAM, *yb = lds + B_Y;
  double *red = lds + B_RED;
  int *flags = reinterpret_cast<int *>(lds + B_INT);
  int *iamb = reinterpret_cast<int *>(lds + B_IAM);
  // per-workgroup scratch: L (packed), then the Q1 rows past QL
  double *Lgl = scratch + (long long)blockIdx.x * SCRATCH;
  const Rows QR{lds + OFF_ROWS, Lgl + LP};
  const int T = (n + 15) >> 4, nb = 16 * T;
  for (;;) {
    // lane ids re-derived opaquely per QP: lane-dependent values are not
    // hoisted out of the QP loop (they would stay live across it)
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int l = tid & 63, wv = tid >> 6;
    const int li = l & 15, lk = l >> 4;  // lane: row li of each of the wave's tiles, column group lk
    int row[RT];
    bool rowok[RT];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      row[t] = 16 * (RT * wv + t) + li;
      rowok[t] = row[t] < m;
    }
    // the next QP index from the queue.  (Rounds 2-3 also read the QP after
    // it and touched one dword per line of its H and A during this QP's
    // iterations; the six prefetch registers lived across the loop, spilled
    // there and made the loop wait on the loads: 3.3-3.9 % slower than no
    // prefetch, profiles/r04/ab/ab128_nopf_*.json.)
    if (tid == 0) flags[1] = atomicAdd(queue, 1);
    __syncthreads();
    const long long g = flags[1];
    if (g >= batch) break;
    const double *Hq = Hg + g * (long long)n * n;
    const double *Aq = BOX ? Hq : Ag + g * (long long)m * n;

    // ------------------------------------------------------------ setup
    clk.tick(10);
    const bool spd = cholesky(lds, Hq, n, T, tid, clk);
#ifdef GRAM_ONLY_CHOL
    if (tid == 0) statg[g] = spd;
    continue;
#endif
    // L kept in the workgroup's scratch for the final solve (the triangle
    // holds Z = R^{-1} during the loop); the loads back come after several
    // barriers on the same CU
#pragma unroll
    for (int u = 0; u < (LP + NT - 1) / NT; ++u) {
      const int e = tid + NT * u;
      if (e < tri(nb, 0)) Lgl[e] = Lp[e];
    }
    clk.tick(0);
    // y = L^{-1} f on wavefront 0, into yb (permuted), before D is live
    if (wv == 0) {
      double a0 = l < n ? fg[g * n + l] : 0.0, a1 = l + 64 < n ? fg[g * n + l + 64] : 0.0;
      solve_lower(Lp, nb, l, a0, a1);
      yb[pad(perm(l))] = a0;
      yb[pad(perm(l + 64))] = a1;
    }
    // this lane's entries of A and b, all issued before the first use: one
    // memory round trip.  Loads are unconditional (masked lanes read a
    // clamped address): a guarded load becomes a branch with its own wait.
    // A's entries land in the registers of D, which the blocked substitution
    // overwrites in place.
    double E[RT][8][4];
    double bl[RT];
    if constexpr (BOX) {
      // row r < n: x_r <= ub_r (a = e_r); row n + i: -x_i <= -lb_i (a = -e_i);
      // an absent bound (NULL array, NaN) is +inf: the row is never violated
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        const int rr = row[t], c0 = rr < n ? rr : rr - n;
        const double sg = rr < n ? 1.0 : -1.0;
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
          for (int r = 0; r < 4; ++r) E[t][k][r] = (rowok[t] && 16 * k + lk + 4 * r == c0) ? sg : 0.0;
        const double *bnd = rr < n ? bg : Ag;
        const double v = (rowok[t] && bnd) ? bnd[g * n + c0] : (rr < n ? kInf : -kInf);
        const double bv = rr < n ? v : -v;
        bl[t] = rowok[t] ? (bv == bv ? bv : kInf) : 0.0;
      }
    } else if (m > 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int col = 16 * k + lk + 4 * r;
            const bool ok = rowok[t] && col < n;
            const double v = Aq[ok ? row[t] * n + col : 0];
            E[t][k][r] = ok ? v : 0.0;
          }
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        const double v = bg[g * m + (rowok[t] ? row[t] : 0)];
        bl[t] = rowok[t] ? v : 0.0;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) E[t][k][r] = 0.0;
#pragma unroll
      for (int t = 0; t < RT; ++t) bl[t] = 0.0;
    }

    // D = A L^{-T} on the matrix cores: tile k of D^T (16 columns of D x 16
    // rows) = (A^T's tile - sum_{j<k} L[k, j] D^T[j]) times Linv_k; the two
    // row tiles of the wave share every L operand
    double na2[RT] = {};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k < T) {
        d4 C[RT];
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            C[t][r] = E[t][k][r];
            na2[t] = __builtin_fma(C[t][r], C[t][r], na2[t]);
          }
#pragma unroll
        for (int j = 0; j < k; ++j)
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const double a = -Lp[tri(16 * k + li, 16 * j + 4 * s + lk)];
#pragma unroll
            for (int t = 0; t < RT; ++t) mfma(a, E[t][j][s], C[t]);
          }
        d4 Z[RT];
#pragma unroll
        for (int t = 0; t < RT; ++t) Z[t] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const double a = LI[k * LIT + li * LIS + 4 * s + lk];
#pragma unroll
          for (int t = 0; t < RT; ++t) mfma(a, C[t][s], Z[t]);
        }
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) E[t][k][r] = Z[t][r];
      }
    }
    clk.tick(1);
    // |D[row,:]|^2 of the lane's rows (the dependency test's scale, published
    // with the selection key: no |u|^2 reduction in the loop)
    double dn2[RT];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      double a0 = 0.0, a1 = 0.0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        a0 = __builtin_fma(E[t][k][0], E[t][k][0], a0);
        a1 = __builtin_fma(E[t][k][1], E[t][k][1], a1);
        a0 = __builtin_fma(E[t][k][2], E[t][k][2], a0);
        a1 = __builtin_fma(E[t][k][3], E[t][k][3], a1);
      }
      dn2[t] = group_sum(a0 + a1);
    }
    double invn[RT], thr[RT], s[RT];
    bool zero_bad = false, act[RT];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      const double nn2 = group_sum(na2[t]);
      invn[t] = nn2 > 0.0 ? rsq(nn2) : 0.0;
      thr[t] = (rowok[t] && nn2 > 0.0) ? -feas_tol * (1.0 + __builtin_fabs(bl[t]) * invn[t]) : -kInf;
      zero_bad = zero_bad || (rowok[t] && nn2 == 0.0 && bl[t] < -feas_tol * (1.0 + __builtin_fabs(bl[t])));
      act[t] = false;
    }
    if (tid == 0) flags[20] = 0;
    __syncthreads();
    if (zero_bad && lk == 0) flags[20] = 1;
    {
      double dy[RT];
      row_dot(E, yb + 34 * lk, dy);  // s = b + D y
#pragma unroll
      for (int t = 0; t < RT; ++t) s[t] = bl[t] + dy[t];
    }
    __syncthreads();
    int status = !spd ? QPB_NOT_SPD : (flags[20] ? QPB_INFEASIBLE : QPB_MAX_ITER);
    bool done = status != QPB_MAX_ITER;
    clk.tick(2);
    // ------------------------------------------------------- active set
    // G-I's J = L^{-T} [Q1^T Q2] in the form D_W^T = Q1^T R, with R kept as
    // its inverse Z = R^{-1}: the orthonormal rows Q1 (q x n, permuted column
    // order; LDS rows at stride QS, rows past QL in the scratch) and the upper
    // triangular Z (q x q, packed by columns in the triangle: Z[i][j] at
    // tri(j, i)), positions 0 .. q-1 in the order of the active set.  For the
    // selected row u = D[p,:] one iteration is
    //   d = Q1 u                        (G-I's d1 = J1^T n+)
    //   w = u - Q1^T d, |w|^2, r = Z d  (J2 J2^T n+, |d2|^2, R^{-1} d1; one
    //                                    phase: w and r do not wait for each other)
    //   D w, the step; ADD: Q1 gains the row w / |w|, Z the column
    //   [-r / |w|; 1 / |w|] (the bordered inverse); DROP k: Givens rotations
    //   on Z's columns j, j+1 (j = k .. q-2) chosen to zero row k of Z, the
    //   same rotations on Q1's rows, then row k of Z and the last column and
    //   row go (R with column k removed, re-triangularised, inverted).
    // Every phase is a parallel pass: nothing is O(q^2) per ADD, and no
    // triangular solve runs in the loop.
    int it = 0, p = 0, q = 0;
    bool selecting = true;
    double up = 0.0, dd = 0.0;
    const double *ub = lds + B_CAND;  // u = D[p,:]: the winning wave's candidate row
    double *db = lds + B_CB;          // d by position
    // each wave offers its most violated row: the key (normalised slack, row
    // in the low mantissa bits) and its slack
    auto publish_key = [&]() {
      double key = kBig;
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        const double v = s[t] * invn[t];
        key = (!act[t] && v < thr[t]) ? __builtin_fmin(key, pack_key256(v, row[t])) : key;
      }
      key = row_min(key);  // the 16 rows of each tile pair, on every lane group
      if (l == 0) red[R_KEY + wv] = key;
      const int pw = key_index256(key);
      // the row itself is written after the selection, by its wave only
      if (key < kBig) {
#pragma unroll
        for (int t = 0; t < RT; ++t)
          if (row[t] == pw && lk == 0) {
            lds[B_CSP + wv] = s[t];
            vb[wv] = dn2[t];  // B_V is free during the loop below NB
          }
      }
    };
    if (tid < NB) {
      iamb[tid] = -1;
      db[tid] = 0.0;
    }
    if (!done) publish_key();
    __syncthreads();
    while (!done && it < max_iter) {
      ++it;
      // lane ids re-derived opaquely per iteration: the addresses built from
      // them are recomputed in the iteration instead of hoisted out of the
      // loop, where they lived across it and spilled
      int tid = threadIdx.x;
      asm volatile("" : "+v"(tid));
      const int l = tid & 63, li = l & 15, lk = l >> 4;
      if (selecting) {
        double kmin = red[R_KEY];
#pragma unroll
        for (int w = 1; w < NWV; ++w) kmin = __builtin_fmin(kmin, red[R_KEY + w]);
        if (!(kmin < kBig)) {
          status = QPB_OK;
          break;
        }
        p = key_index256(kmin);
        up = 0.0;
        selecting = false;
        // u = D[p,:] from the one wave that holds row p
        if (wv == p / (16 * RT)) {
#pragma unroll
          for (int t = 0; t < RT; ++t)
            if (row[t] == p) {
              double *dst = lds + B_CAND + 34 * lk;
#pragma unroll
              for (int k = 0; k < 8; ++k) {
                *reinterpret_cast<double2 *>(&dst[4 * k]) = make_double2(E[t][k][0], E[t][k][1]);
                *reinterpret_cast<double2 *>(&dst[4 * k + 2]) = make_double2(E[t][k][2], E[t][k][3]);
              }
            }
        }
        __syncthreads();
        // |u|^2 (the dependency test's scale), published with the key
        dd = vb[p / (16 * RT)];
      }
      clk.tick(3);
      // ---- d = Q1 u: lane (lk, li) of wave w takes position 32 j + 4 w + lk
      // over the columns li + 16 i (row sums over the 16 lanes finish it)
      for (int t0 = 4 * wv; t0 < q; t0 += 4 * NWV) {
        const int t = t0 + lk;
        const int tt = t < q ? t : t0;
        // all eight Q1 entries and u entries in flight before the FMAs; rows
        // in LDS (the usual case, wave-uniform test) are read as LDS, not
        // through generic pointers (flat loads, each waited for)
        double qv[8], uv[8];
        if (t0 + 3 < QL) {
          const __attribute__((address_space(3))) double *qr =
              (const __attribute__((address_space(3))) double *)(QR.lds + tt * QS);
#pragma unroll
          for (int i = 0; i < 8; ++i) qv[i] = qr[li + 16 * i];
        } else {
          const double *qr = QR.row(tt);
#pragma unroll
          for (int i = 0; i < 8; ++i) qv[i] = qr[li + 16 * i];
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) uv[i] = ub[pad(li + 16 * i)];
        double a0 = 0.0, a1 = 0.0;
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
          a0 = __builtin_fma(qv[i], uv[i], a0);
          a1 = __builtin_fma(qv[i + 1], uv[i + 1], a1);
        }
        const double dv = row_sum(a0 + a1);
        if (li == 0 && t < q) db[t] = dv;
      }
      __syncthreads();
      clk.tick(4);
      // ---- w = u - Q1^T d: lane (lk, li) of wave w takes (permuted) column
      // 16 w + li over the positions j = lk mod 4; |w|^2 per wave
      {
        const int c = 16 * wv + li;
        double acc0 = 0.0, acc1 = 0.0;
        const int qa = q < QL ? q : QL;
        int j = lk;
        // four positions per step, their eight reads in flight together
        for (; j + 12 < qa; j += 16) {
          const double d0 = db[j], d1 = db[j + 4], d2 = db[j + 8], d3 = db[j + 12];
          const double q0 = QR.lds[j * QS + c], q1 = QR.lds[(j + 4) * QS + c];
          const double q2 = QR.lds[(j + 8) * QS + c], q3 = QR.lds[(j + 12) * QS + c];
          acc0 = __builtin_fma(d0, q0, acc0);
          acc1 = __builtin_fma(d1, q1, acc1);
          acc0 = __builtin_fma(d2, q2, acc0);
          acc1 = __builtin_fma(d3, q3, acc1);
        }
        for (; j + 4 < qa; j += 8) {
          acc0 = __builtin_fma(db[j], QR.lds[j * QS + c], acc0);
          acc1 = __builtin_fma(db[j + 4], QR.lds[(j + 4) * QS + c], acc1);
        }
        if (j < qa) acc0 = __builtin_fma(db[j], QR.lds[j * QS + c], acc0);
        for (j = QL + lk; j < q; j += 4) acc1 = __builtin_fma(db[j], QR.gl[(j - QL) * NB + c], acc1);
        const double w = ub[pad(c)] - group_sum(acc0 + acc1);
        if (lk == 0) wb[pad(c)] = w;
        const double ws = wave_sum(lk == 0 ? w * w : 0.0);
        if (l == 0) red[R_ND2 + wv] = ws;
      }
      // ---- r = Z d over rows i = 16 w + li (lane group lk: the columns
      // c >= i, c = lk mod 4), then each wave's ratio minimum (first position
      // at the minimum; waves in position order)
      {
        const int i = 16 * wv + li;
        double ratio = kBig;
        if (16 * wv < q) {
          double acc = 0.0, acc1 = 0.0;
          int c = lk + ((i > lk) ? ((i - lk + 3) & ~3) : 0);
          // four columns per step, their eight reads in flight together
          for (; c + 12 < q; c += 16) {
            const double z0 = Lp[tri(c, i)], z1 = Lp[tri(c + 4, i)], z2 = Lp[tri(c + 8, i)], z3 = Lp[tri(c + 12, i)];
            const double d0 = db[c], d1 = db[c + 4], d2 = db[c + 8], d3 = db[c + 12];
            acc = __builtin_fma(z0, d0, acc);
            acc1 = __builtin_fma(z1, d1, acc1);
            acc = __builtin_fma(z2, d2, acc);
            acc1 = __builtin_fma(z3, d3, acc1);
          }
          for (; c < q; c += 4) acc = __builtin_fma(Lp[tri(c, i)], db[c], acc);
          const double rt = group_sum(acc + acc1);
          if (i < q) {
            if (lk == 0) rb[i] = rt;
            if (rt > 0.0) ratio = lamb[i] * rcp(rt);
          }
        }
        const double wmin = row_min(ratio);
        const double kpos = row_min((ratio == wmin && wmin < kBig) ? (double)i : 1e9);
        if (l == 0) {
          red[R_T1 + 2 * wv] = wmin;
          red[R_T1 + 2 * wv + 1] = kpos;
        }
      }
      // s_p, read before the barrier: an ADD's publish_key below rewrites the
      // candidate slacks while slower waves may still be in this step
      const double sp = lds[B_CSP + p / (16 * RT)];
      __syncthreads();
      clk.tick(5);
      // ---- slack direction D w (issued before the scalar chain below needs it)
      double ds[RT];
      row_dot(E, wb + 34 * lk, ds);
      // ---- step lengths (identical arithmetic on every wavefront)
      double nd2 = 0.0;
#pragma unroll
      for (int w = 0; w < NWV; ++w) nd2 += red[R_ND2 + w];
      double t1 = kBig;
      int kdrop = 0;
#pragma unroll
      for (int w = 0; w < NWV; ++w)  // waves in position order: ties keep the lowest position
        if (red[R_T1 + 2 * w] < t1) {
          t1 = red[R_T1 + 2 * w];
          kdrop = (int)red[R_T1 + 2 * w + 1];
        }
      const double t2 = (nd2 > kDepTol * dd) ? -sp * rcp(nd2) : kBig;
      const double tt = t1 < t2 ? t1 : t2;
      if (!(tt < kBig)) {
        status = QPB_INFEASIBLE;
        break;
      }
      clk.tick(15);
      if (t2 < kBig) {
#pragma unroll
        for (int t = 0; t < RT; ++t) s[t] = __builtin_fma(tt, ds[t], s[t]);
      }
      up += tt;
      clk.tick(16);
      if (tid < q) lamb[tid] = __builtin_fma(-tt, rb[tid], lamb[tid]);
      if (t2 <= t1) {
        // ---- ADD p at position q
        const double rn = rsq(nd2);  // 1 / |w|
        if (tid < NB) QR.row(q)[tid] = wb[pad(tid)] * rn;
        if (tid < q) Lp[tri(q, tid)] = -rb[tid] * rn;
        if (tid == q) Lp[tri(q, q)] = rn;
        if (tid == 0) {
          iamb[q] = p;
          lamb[q] = up;
        }
#pragma unroll
        for (int t = 0; t < RT; ++t)
          if (row[t] == p) act[t] = true;
        ++q;
        selecting = true;
      } else {
        // ---- DROP position k
        const int k = kdrop;
        const int cdrop = iamb[k];
#pragma unroll
        for (int t = 0; t < RT; ++t)
          if (row[t] == cdrop) act[t] = false;
        // row k of Z (columns k .. q-1) copied aside: the rotation chains of
        // waves 0-2 read it while wave 0 rewrites Z in place
        double *zrow = vb + NB;
        if (tid >= k && tid < q) zrow[tid] = Lp[tri(tid, k)];
        __syncthreads();  // the multiplier update above and zrow, before the shift
        // Rotation j (j = k .. q-2) on the pair (j, j+1) zeroes Z[k][j]: with
        // X_k = Z[k][k] and X_{j+1} = hypot(X_j, Z[k][j+1]) (the carried
        // entry of row k), c_j = Z[k][j+1] / X_{j+1}, s_j = -X_j / X_{j+1}.
        // Every wave that applies rotations runs this scalar chain itself.
        if (wv == 0) {
          // Z's columns: lane l carries rows l and l + 64; row i > k moves to
          // i - 1 (row k goes).  Step j reads column j+1 and writes column j;
          // one wave's DS instructions run in order, so the row moving into
          // i - 1 never overwrites an entry row i - 1 has still to read.
          double x0 = l <= k ? Lp[tri(k, l <= k ? l : 0)] : 0.0;  // rows' entries in column k
          double x1 = l + 64 <= k ? Lp[tri(k, l + 64 <= k ? l + 64 : 0)] : 0.0;
          double X = zrow[k];
          for (int j = k; j < q - 1; ++j) {
            const double z0 = l <= j + 1 ? Lp[tri(j + 1, l <= j + 1 ? l : 0)] : 0.0;
            const double z1 = l + 64 <= j + 1 ? Lp[tri(j + 1, l + 64 <= j + 1 ? l + 64 : 0)] : 0.0;
            const double zk = zrow[j + 1];
            const double h = __builtin_sqrt(__builtin_fma(X, X, zk * zk));
            const double ih = 1.0 / h;
            const double cs = zk * ih, sn = -X * ih;
            const double n0 = __builtin_fma(cs, x0, sn * z0), n1 = __builtin_fma(cs, x1, sn * z1);
            x0 = __builtin_fma(-sn, x0, cs * z0);
            x1 = __builtin_fma(-sn, x1, cs * z1);
            X = h;
            wave_lds_sync();
            // new row i' = i (i < k) or i - 1 (i > k), column j: rows <= j only
            const int i0 = l < k ? l : l - 1, i1 = l + 64 < k ? l + 64 : l + 63;
            if (l != k && i0 <= j && l <= j + 1) Lp[tri(j, i0)] = n0;
            if (l + 64 != k && i1 <= j && l + 64 <= j + 1) Lp[tri(j, i1)] = n1;
          }
        } else if (wv == 1 || wv == 2) {
          // Q1's rows, one column per thread
          const int c = tid - 64;
          if (k < q - 1) {
            double X = zrow[k];
            double cur = QR.row(k)[c];
            for (int j = k; j < q - 1; ++j) {
              const double zk = zrow[j + 1];
              const double nx = QR.row(j + 1)[c];
              const double h = __builtin_sqrt(__builtin_fma(X, X, zk * zk));
              const double ih = 1.0 / h;
              const double cs = zk * ih, sn = -X * ih;
              QR.row(j)[c] = __builtin_fma(cs, cur, sn * nx);
              cur = __builtin_fma(-sn, cur, cs * nx);
              X = h;
            }
          }
        } else if (wv == 3) {
          // positions k+1 .. q-1 move down by one (reads before writes: one
          // wave's DS instructions run in order)
          const double l0 = lamb[l + 1], l1 = lamb[l + 64 < NB - 1 ? l + 65 : NB - 1];
          const int i0 = iamb[l + 1], i1 = iamb[l + 64 < NB - 1 ? l + 65 : NB - 1];
          wave_lds_sync();
          if (l >= k && l < q - 1) {
            lamb[l] = l0;
            iamb[l] = i0;
          } else if (l == q - 1) {
            lamb[l] = 0.0;
            iamb[l] = -1;
          }
          if (l + 64 >= k && l + 64 < q - 1) {
            lamb[l + 64] = l1;
            iamb[l + 64] = i1;
          } else if (l + 64 == q - 1) {
            lamb[l + 64] = 0.0;
            iamb[l + 64] = -1;
          }
        }
        --q;
#pragma unroll
        for (int t = 0; t < RT; ++t)  // p stays selected: its slack after the partial step
          if (row[t] == p && lk == 0) lds[B_CSP + wv] = s[t];
      }
      clk.tick(17);
      if (selecting) publish_key();
      clk.tick(18);
      __syncthreads();
      clk.tick(6);
    }

    // ------------------------------------------------------------ outputs
    // full multiplier vector by row (vb), the active-set words,
    // g = y + D_W^T lam = y + D^T lam_full: each wave sums its 32 rows of D
    // weighted by their multipliers (16-lane row sums), the eight partial
    // vectors are added per column
    for (int e = tid; e < MB; e += NT) vb[e] = 0.0;
    __syncthreads();
    if (tid < q && iamb[tid] >= 0) vb[iamb[tid]] = lamb[tid];
    __syncthreads();
    {
      double lw[RT];
#pragma unroll
      for (int t = 0; t < RT; ++t) lw[t] = vb[row[t]];
      double *part = lds + OFF_ROWS + wv * PV;  // the Q1 rows are dead now
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          double a = lw[0] * E[0][k][r];
#pragma unroll
          for (int t = 1; t < RT; ++t) a = __builtin_fma(lw[t], E[t][k][r], a);
          a = row_sum(a);
          if (li == 0) part[34 * lk + 4 * k + r] = a;  // permuted column order, padded
        }
    }
    __syncthreads();
    if (tid < NB) {
      double gsum = yb[pad(tid)];
#pragma unroll
      for (int w = 0; w < NWV; ++w) gsum += lds[OFF_ROWS + w * PV + pad(tid)];
      yb[pad(tid)] = gsum;
    }
    {
      uint32_t word = 0;
#pragma unroll
      for (int t = 0; t < RT; ++t) word |= (uint32_t)(__ballot(act[t] && lk == 0) & 0xFFFFull) << (16 * t);
      if (l == 0) flags[2 + wv] = (int)word;  // rows 32 wv .. 32 wv + 31
    }
    __syncthreads();
    for (int e = tid; e < m; e += NT) lamg[g * m + e] = vb[e];
    const int words = (m + 31) >> 5;
    if (tid < words) actg[g * words + tid] = (uint32_t)flags[2 + tid];
    // x = -L^{-T} g: L again (the triangle held Z)
    bool finite = true;
    clk.tick(7);
    if (spd) {
      // loads issued in passes of 6 before their stores: three round trips,
      // not one per element pass (more registers here spill elsewhere)
      const int ne = tri(nb, 0);
      for (int e0 = tid; e0 < ne; e0 += 6 * NT) {
        double lv[6];
#pragma unroll
        for (int u = 0; u < 6; ++u) {
          const int e = e0 + NT * u;
          lv[u] = Lgl[e < ne ? e : 0];
        }
#pragma unroll
        for (int u = 0; u < 6; ++u) {
          const int e = e0 + NT * u;
          if (e < ne) Lp[e] = lv[u];
        }
      }
      __syncthreads();
      clk.tick(8);
      if (wv == 0) {
        double x0 = -yb[pad(perm(l))], x1 = -yb[pad(perm(l + 64))];
        solve_upper(Lp, nb, l, x0, x1);
        if (l < n) xg[g * n + l] = x0;
        if (l + 64 < n) xg[g * n + l + 64] = x1;
        const bool bad = (l < n && !(__builtin_fabs(x0) < kInf)) || (l + 64 < n && !(__builtin_fabs(x1) < kInf));
        finite = __ballot(bad) == 0;
      }
    } else if (wv == 0) {
      if (l < n) xg[g * n + l] = 0.0;
      if (l + 64 < n) xg[g * n + l + 64] = 0.0;
    }
    if (tid == 0) {
      statg[g] = (status == QPB_OK && !finite) ? QPB_NUMERICAL : status;
      if (itg) itg[g] = it;
    }
    __syncthreads();
    clk.tick(9);
  }
  if (threadIdx.x == 0) clk.flush(dbg);
}

}  // namespace gram
}  // namespace qpb

// scratch: per workgroup (NB - QL) D_W rows beyond the LDS ones + the queue head
template <bool BOX>
static hipError_t launch_gi_gram(const qpb_desc *d, const double *H, const double *f, const double *A,
                                 const double *b, double *x, double *lam, uint32_t *active, int32_t *status,
                                 int32_t *iters, unsigned long long *sections, hipStream_t stream) {
  const int max_iter = d->max_iter > 0 ? d->max_iter : 4 * (d->n + d->m) + 8;
  const double tol = d->feas_tol > 0 ? d->feas_tol : 1e-10;
  int dev = 0, cus = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return e;
  const long long grid = d->batch < cus ? d->batch : cus;
  const size_t rows_bytes = (size_t)grid * qpb::gram::SCRATCH * sizeof(double);
  // cached per stream (qpb_workspace.hip); the launch is queued under its lock
  return qpb_with_workspace(stream, rows_bytes + 256, [&](void *buf) {
    int *queue = reinterpret_cast<int *>(static_cast<char *>(buf) + rows_bytes);
    hipError_t err = hipMemsetAsync(queue, 0, sizeof(int), stream);
    if (err != hipSuccess) return err;
    if constexpr (!BOX)  // the stamped diagnostic build exists for the dense form only
      if (sections) {
        hipLaunchKernelGGL((qpb::gram::gi_gram_kernel<true, BOX>), dim3((unsigned)grid), dim3(qpb::gram::NT), 0, stream, H,
                         f, A, b, x, lam, active, status, iters, d->n, d->m, (long long)d->batch, max_iter, tol,
                         queue, static_cast<double *>(buf), sections);
        return hipGetLastError();
      }
    hipLaunchKernelGGL((qpb::gram::gi_gram_kernel<false, BOX>), dim3((unsigned)grid), dim3(qpb::gram::NT), 0, stream, H,
                         f, A, b, x, lam, active, status, iters, d->n, d->m, (long long)d->batch, max_iter, tol,
                         queue, static_cast<double *>(buf), nullptr);
    return hipGetLastError();
  });
}

extern "C" hipError_t qpb_launch_gi_gram(const qpb_desc *d, const double *H, const double *f, const double *A,
                                         const double *b, double *x, double *lam, uint32_t *active,
                                         int32_t *status, int32_t *iters, unsigned long long *sections,
                                         hipStream_t stream) {
  return launch_gi_gram<false>(d, H, f, A, b, x, lam, active, status, iters, sections, stream);
}
// qpb_solve_box for 32 < n <= 128: lb, ub in A's and b's places (d->m == 2 d->n)
extern "C" hipError_t qpb_launch_gi_gram_box(const qpb_desc *d, const double *H, const double *f, const double *lb,
                                             const double *ub, double *x, double *lam, uint32_t *active,
                                             int32_t *status, int32_t *iters, hipStream_t stream) {
  return launch_gi_gram<true>(d, H, f, lb, ub, x, lam, active, status, iters, nullptr, stream);
}
