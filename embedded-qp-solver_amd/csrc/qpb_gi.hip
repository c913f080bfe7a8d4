// qpb_gi.hip -- batched dense active-set QP kernel for gfx950 (n <= 16).
//
//   min 1/2 x^T H x + f^T x   s.t.   A x <= b        (fp64, one QP per 16 lanes)
//
// Replaces, batched, the reference's hot path: the dense kernels of
// matrix/matrix_ops/matrix_ops.c (matrix_mult GEMV :235-271, LU/inverse
// :487-630, vector ops :158-411, norm :632-656) driving the solver iterations
// of qp_solvers/qp_solvers.c.  The constrained iteration north_star asks for
// (absent from the reference) is the dual active-set method of
// Goldfarb & Idnani (Math. Prog. 27, 1983), which needs no feasible start:
//
//   setup   H = L L^T, D = A L^{-T}, y = L^{-1} f in ONE right-looking sweep:
//           step k broadcasts pivot row k of the Schur complement (DPP
//           row_newbcast from lane k); by symmetry it is also column k, so
//           the same broadcast drives the Schur update of row l (lane l), the
//           substitution of both D rows of lane l and the lane-parallel y.
//           Slack of the unconstrained minimiser x0 = -H^{-1} f
//           (test/qp_ref.py:35's answer): s = b - A x0 = b + D y.
//   iterate D = A L^{-T} Q is kept in the rotated basis Q: the rows of the
//           active constraints are zero on the free basis columns q..15.
//           Pick the violated row p with the largest violation per unit
//           length of its free part, -s_p / |D[p, q:]| (dual steepest edge;
//           the squared free norms are kept up to date, fp32 keys); its row
//           d = D[p,:] splits into d1 (columns < q) and d2 (columns >= q).
//           Dual step r = R^{-1} d1 (lane-parallel back substitution over the
//           prefetched R column), partial step t1 (ratio test over the active
//           multipliers), full step t2 = -s_p / |d2|^2, slacks s -= t D d2.
//           full step  -> ADD p: one Householder reflection on columns q..15
//                         of D (every lane updates its own rows; its product
//                         D v = D d2 + alpha D[:, q] reuses the slack step's
//                         D d2 and reads column q by a branch tree on q), new
//                         column of R;
//           partial    -> DROP k: delete column k of R, Givens rotations
//                         restore triangularity (also applied to D).
//   finish  x = -H^{-1} (f + A^T lam) from the final multipliers (KKT
//           stationarity): the active rows of A are re-read, two lane-
//           parallel triangular solves with L kept in LDS.
//
// Data layout per QP (lane l = 0..15 of the QP's 16-lane DPP row):
//   registers  rows l + 16 r (r < MR) of D, their slacks, 1/||a_row||,
//              |D row|^2, |free part|^2, active flags; multiplier / row of
//              active position l, R[l][l] and its reciprocal; in a DROP the
//              parameters of Givens rotation l
//   LDS        L (packed rows), R (16 x 16 column-major, zero diagonal; its
//              column 0 carries the exchange row).  The whole slot is the staging buffer of the
//              coalesced input transposes before the factorisation, and the
//              dead R holds the lambda scatter and the x capture after the
//              loop.
// Every product with a vector held one entry per lane (d2, the Householder
// vector) is a v_fmac_f64_dpp reading the entry from lane j by row_newbcast:
// no LDS round trip, no copy of the vector in every lane.
// No branch or select compares the lane id with a compile-time constant:
// such masks are hoisted by the compiler and end up spilled (SGPR pressure).
#include "qpb_common.h"
#include "qpb.h"

namespace qpb {

constexpr int NL = 16;  // lanes per QP
constexpr int QPB = 4;  // QPs per workgroup (one wavefront)
constexpr int RS = 18;  // row stride (doubles) of the input transposes: conflict-free b128

// packed lower triangle of L: row i at i(i+1)/2.  Reads may run past a row's
// end into the next rows (always inside the QP's slot): the solves never use
// those values.
__host__ __device__ constexpr int lrow(int i) { return i * (i + 1) / 2; }
constexpr int L_SIZE = lrow(NL);  // 136

// LDS slot of one QP: 394 doubles = 3,152 B, 12,608 B per wave -> 12 waves
// per CU (3 per SIMD, matching the VGPR budget).  A CU holds 12 one-wave
// workgroups of up to 12,800 B of LDS each and 11 from 13,056 B
// (tools/probe/occupancy_probe.hip, measured on the MI355X): the round-4 slot
// (426 doubles, 13,632 B per wave) ran 11 waves per CU, one SIMD in four
// with two (the wave timeline, tools/wave_timeline.py).
constexpr int OFF_L = 0;                  // L (136)
constexpr int OFF_T = L_SIZE;             // R, column-major 16 x 16: R[i][j] at j*16 + i;
                                          // column 0 (no entry above the diagonal) doubles as
                                          // the exchange row outside a DROP
constexpr int OFF_XCH = OFF_T + NL * NL;  // 392: s_p, |d|^2 of the exchange
constexpr int SLOT = OFF_XCH + 2;         // 394
constexpr int kWaveLdsMax = 12800;        // bytes per one-wave workgroup for 12 per CU
constexpr double kDepTol = 1e-24;         // |d2|^2 <= kDepTol |d|^2  <=>  z = 0
static_assert(SLOT % 2 == 0 && OFF_T % 2 == 0 && OFF_XCH % 2 == 0, "b128 alignment");
static_assert(4 * SLOT * 8 <= kWaveLdsMax, "12 waves (3 per SIMD) per CU by LDS");
static_assert(NL * RS <= SLOT, "input transposes are staged over the whole slot");

// sum_{j<N} x(j) y(j) with 2 independent accumulators
template <int N, class FX, class FY>
__device__ __forceinline__ double dot2(FX &&x, FY &&y, double init = 0.0) {
  double a0 = init, a1 = 0.0;
  unroll<N>([&](auto J) {
    constexpr int j = J;
    if constexpr (j % 2 == 0) a0 = __builtin_fma(x(j), y(j), a0);
    if constexpr (j % 2 == 1) a1 = __builtin_fma(x(j), y(j), a1);
  });
  return a0 + a1;
}

// 16 doubles from LDS (16-byte aligned) as 8 b128 reads
__device__ __forceinline__ void lds_row16(const double *src, double (&dst)[NL]) {
#pragma unroll
  for (int j = 0; j < NL; j += 2) {
    const double2 v = *reinterpret_cast<const double2 *>(&src[j]);
    dst[j] = v.x;
    dst[j + 1] = v.y;
  }
}

// out[r] = sum_j vec[lane j] * x[r][j] over the row's 16 lanes, DPP-fused;
// the MR rows interleaved, two chains each (2 MR independent accumulators);
// the caller has issued dpp_ready(vec)
template <int MR>
__device__ __forceinline__ void bdot_rows(double vec, const double (&x)[MR][NL], double (&out)[MR]) {
  double a[MR][2];
#pragma unroll
  for (int r = 0; r < MR; ++r) a[r][0] = a[r][1] = 0.0;
  unroll<NL>([&](auto J) {
    constexpr int j = J;
#pragma unroll
    for (int r = 0; r < MR; ++r) fmac_bc<j>(a[r][j & 1], vec, x[r][j]);
  });
#pragma unroll
  for (int r = 0; r < MR; ++r) out[r] = a[r][0] + a[r][1];
}

// MR: rows of D per lane (m <= 16 MR).  N16: n == 16 (coalesced loads).
// FULL: n == 16 and m == 16 MR (no padding rows: no masking anywhere).
// One group = the 4 QPs of a wavefront; `grp` its index.
template <int MR, bool N16, bool FULL, bool STAMP>
__device__ __forceinline__ void gi_group(
    double *lds, const double *__restrict__ Hg, const double *__restrict__ fg, const double *__restrict__ Ag,
    const double *__restrict__ bg, double *__restrict__ xg, double *__restrict__ lamg,
    uint32_t *__restrict__ actg, int32_t *__restrict__ statg, int32_t *__restrict__ itg, int n, int m,
    long long batch, int max_iter, double feas_tol, int flags, unsigned long long *__restrict__ dbg,
    long long grp) {
  static_assert(!FULL || N16, "FULL implies n == 16");
  SectionClock<STAMP> clk;
  const int l = threadIdx.x & (NL - 1);
  const int slot = threadIdx.x >> 4;
  const int sh = (threadIdx.x & 63) & ~(NL - 1);  // this row's bit offset in a wave ballot
  // Rows past the end of the batch (last group only) do not leave: they replay
  // the batch's last QP -- same trip count, so they never extend the wave's
  // loop -- and store nothing.  Every lane of the wave stays live, so the
  // cross-row reads (wave_max4's readlanes) only ever see real QP state.
  const long long graw = grp * QPB + slot;
  const bool live = graw < batch;
  const long long g = live ? graw : batch - 1;
  if constexpr (FULL) {
    n = NL;
    m = NL * MR;
  }

  // LDS slots in the order 0, 2, 1, 3: ds_read_b64 serves 32 lanes (two QPs)
  // per cycle; slots 0/1 and 2/3 are 2 SLOT = 788 doubles apart, 40 banks mod
  // 64, so contiguous 16-lane reads of the two QPs share 8 of the 64 banks
  // (one slot apart they would share 20)
  double *base = lds + (((slot & 1) << 1) | (slot >> 1)) * SLOT;
  double *Lp = base + OFF_L;
  double *Tv = base + OFF_T;  // R, column-major (zero diagonal)
  // the exchange row in R's column 0: the back substitution never reads that
  // column, a DROP rebuilds it before use, an ADD at q = 0 rewrites it
  double *xch = Tv;
  double *xsd = base + OFF_XCH;  // s_p, |D[p,:]|^2

  // ------------------------------------------------------------------ load
  // (flags & QPB_FLAG_DIAG_L2: every QP reads the inputs of QP g mod 512;
  // QPB_FLAG_DIAG_MALL: of QP g mod 16384 (107 MB, Infinity-Cache resident
  // after the first launch) -- diagnostics that take HBM out of the kernel time)
  const long long gi = (flags & QPB_FLAG_DIAG_L2) ? (g & 511) : (flags & QPB_FLAG_DIAG_MALL) ? (g & 16383) : g;
  const double *Hq = Hg + gi * (long long)n * n;
  // m == 0: A/b may be NULL -- point the (masked) row loads at H instead
  const double *Aq = m > 0 ? Ag + gi * (long long)m * n : Hq;
  const double *bq = m > 0 ? bg + gi * (long long)m : Hq;
  double Lr[NL];  // row l of H, becomes row l of L
  double E[MR][NL];
  double s[MR], bl[MR], thr[MR];
  float ddr[MR];  // |D[r,:]|^2 (the dependency test's scale; clamped to FLT_MAX)
  float fn2[MR];  // |D[r, q:]|^2, the free part of the row (scale of the selection key)
  bool act[MR];
  bool infeasible_row = false;
  // b and f with the matrices (same round trip)
  double bv[MR];
#pragma unroll
  for (int r = 0; r < MR; ++r) bv[r] = bq[(FULL || l + NL * r < m) ? l + NL * r : 0];
  const double fv = fg[gi * n + (l < n ? l : n - 1)];
  const double fl = (N16 || l < n) ? fv : 0.0;
  [[maybe_unused]] const int hr = l >> 3, hc = 2 * (l & 7);
  // stage 16 rows of a 16-column matrix (as loaded) in this QP's slot (L and
  // R are written after the factorisation)
  auto stage = [&](const double2 (&v)[8]) {
    wave_lds_sync();
#pragma unroll
    for (int t = 0; t < 8; ++t) *reinterpret_cast<double2 *>(&base[(2 * t + hr) * RS + hc]) = v[t];
    wave_lds_sync();
  };
  // row r's constant data from its entries: the violation threshold of the
  // slack, s / |a| < -tol (1 + |b| / |a|), i.e. s < -tol (|a| + |b|) (-inf: a
  // zero row, never selected), and the zero row's own test 0 <= b
  auto row_norms = [&](int r, const double (&row)[NL]) {
    const double nrm2 = dot2<NL>([&](int j) { return row[j]; }, [&](int j) { return row[j]; });
    const bool ok = FULL || l + NL * r < m;
    bl[r] = ok ? bv[r] : 0.0;
    thr[r] = nrm2 > 0.0 ? -feas_tol * (nrm2 * rsq1(nrm2) + __builtin_fabs(bl[r])) : -kInf;
    infeasible_row = infeasible_row || (ok && nrm2 == 0.0 && bl[r] < -feas_tol * (1.0 + __builtin_fabs(bl[r])));
    act[r] = false;
  };
  if constexpr (N16) {
    // Coalesced 16-byte loads: one instruction reads 2 whole rows (256 B) of
    // each of the wave's 4 QPs -- lane l gets row 2t + (l>>3), columns
    // 2(l&7), 2(l&7)+1.  Rows reach their owner lane through a transpose in
    // this QP's LDS slot (free until the factorisation ends).
    double2 hv[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) hv[t] = *reinterpret_cast<const double2 *>(&Hq[(2 * t + hr) * NL + hc]);
    auto load_a = [&](int r, double2 (&v)[8]) {
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int row = NL * r + 2 * t + hr;
        if constexpr (FULL)
          v[t] = *reinterpret_cast<const double2 *>(&Aq[row * NL + hc]);
        else
          v[t] = row < m ? *reinterpret_cast<const double2 *>(&Aq[row * NL + hc]) : make_double2(0.0, 0.0);
      }
    };
    // all input rows in flight at once (one HBM round trip); instruction
    // selection sinks loads to their first use, so an empty asm consumes
    // them right here
    double2 av[MR][8];
#pragma unroll
    for (int r = 0; r < MR; ++r) load_a(r, av[r]);
#pragma unroll
    for (int r = 0; r < MR; ++r) asm volatile("" ::"v"(bv[r]));
    asm volatile("" ::"v"(fv));
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      asm volatile("" ::"v"(hv[t].x), "v"(hv[t].y));
#pragma unroll
      for (int r = 0; r < MR; ++r) asm volatile("" ::"v"(av[r][t].x), "v"(av[r][t].y));
    }
    stage(hv);
    lds_row16(&base[l * RS], Lr);
#pragma unroll
    for (int r = 0; r < MR; ++r) {
      stage(av[r]);
      lds_row16(&base[l * RS], E[r]);
      row_norms(r, E[r]);
    }
    wave_lds_sync();
  } else {  // padded n < 16: clamped per-lane row loads, identity outside n
    const int lc = l < n ? l : n - 1;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const double h = Hq[lc * n + (j < n ? j : n - 1)];
      Lr[j] = (l < n && j < n) ? h : (l == j ? 1.0 : 0.0);
    }
#pragma unroll
    for (int r = 0; r < MR; ++r) {
      const int row = l + NL * r;
      const bool ok = row < m;
      const int rc = ok ? row : 0;
#pragma unroll
      for (int j = 0; j < NL; ++j) {
        const double a = Aq[rc * n + (j < n ? j : n - 1)];
        E[r][j] = (ok && j < n) ? a : 0.0;
      }
      row_norms(r, E[r]);
    }
  }
  clk.tick(0);
#ifdef QPB_WAVE_TRACE
  if (!STAMP && dbg) {  // diagnostic build: the inputs have arrived
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    if (threadIdx.x == 0) dbg[8ull * grp + 5] = t;
  }
#endif

  bool spd = true;
  double ya = fl;
  {
    // ---- H = L L^T, D = A L^{-T}, y = L^{-1} f: one right-looking sweep.
    // Step k: pr = row k of the current Schur complement (lane k's Lr, DPP
    // broadcast) = column k by symmetry, so L[j][k] = pr[j] / sqrt(akk) and
    //   row l:  Lr[j] -= c pr[j] (j > k),  c = Lr[k] / akk;   Lr[k] = L[l][k]
    //   D rows: E[k] /= sqrt(akk), E[j] -= E[k] pr[j] / akk (j > k)
    //   y:      lane-parallel, f_l -= c f_k (f_k read from lane k by the FMA)
    // Lanes l < k keep updating dead entries of their row (the upper triangle,
    // never read).  The pivot row is read straight from lane k by the FMAs
    // (v_fmac_f64_dpp); the sched_barrier and the rsq chain keep every write of
    // Lr[j] and of f (previous step) well over two instructions before these
    // reads.  Lane k's own Lr[j] is updated last, after the D rows have read it.
    // s = b + D y accumulates in the same sweep, negated: D[r][k] y_k =
    // (e ik)(f_k ik) = -ne2 f_k, one DPP-fused FMA per row with f_k from lane k
    // (y itself is never formed).
    double ns[MR];  // -s during the sweep
#pragma unroll
    for (int r = 0; r < MR; ++r) ns[r] = -bl[r];
    unroll<NL>([&](auto K) {
      constexpr int k = K;
      __builtin_amdgcn_sched_barrier(0);
      const double akk = bc<k>(Lr[k]);
      spd = spd && (akk > 0.0);
      const double ik = rsq1(akk);
      const double ik2 = ik * ik;
      const double nc = -(Lr[k] * ik2);
      double ne2[MR];
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        const double e = E[r][k];
        ne2[r] = -(e * ik2);
        E[r][k] = e * ik;
      }
#pragma unroll
      for (int r = 0; r < MR; ++r) fmac_bc<k>(ns[r], ya, ne2[r]);
      unroll<NL - 1 - k>([&](auto J) {
        constexpr int j = k + 1 + J;
#pragma unroll
        for (int r = 0; r < MR; ++r) fmac_bc<k>(E[r][j], Lr[j], ne2[r]);
        fmac_bc<k>(Lr[j], Lr[j], nc);
      });
      fmac_bc<k>(ya, ya, nc);  // lane k's own f_k becomes 0 (dead)
      Lr[k] *= ik;
    });
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < MR; ++r) s[r] = -ns[r];
    // L -> LDS, packed rows (lane l writes row l), kept for the final solves.
    // Lane l also writes its dead entries j > l, over the start of later rows:
    // stores go in descending j, and a row's own entry at such an address has
    // a smaller j, so it lands last (a wave's DS instructions execute in order).
    unroll<NL>([&](auto J) {
      constexpr int j = NL - 1 - J;
      Lp[lrow(l) + j] = Lr[j];
      wave_lds_sync();
    });
  }
  // |D[r,:]|^2 = |a_r L^{-T}|^2: the loop's reflections are orthogonal, so it
  // never changes (the dependency test's scale).  Clamped to FLT_MAX instead
  // of overflowing to inf (rows with |D_r| > 1.8e19, e.g. |a| = 1e20 over a
  // unit H): the test |d2|^2 > 1e-24 |D_p|^2 then still rejects a dependent
  // row (|d2|^2 ~ eps^2 |D_p|^2) up to |D_p| ~ 1e23, where it used to reject
  // every row and end the QP INFEASIBLE.
#pragma unroll
  for (int r = 0; r < MR; ++r) {
    ddr[r] = __builtin_fminf((float)dot2<NL>([&](int j) { return E[r][j]; }, [&](int j) { return E[r][j]; }),
                             3.402823466e38f);
    fn2[r] = ddr[r];
  }
  clk.tick(1);

  // ------------------------------------------------------ active-set loop
  // R (upper triangular, active positions; column j = position j, column-major
  // so the lane-parallel accesses are contiguous) lives in LDS with a ZERO
  // diagonal; lane l keeps 1 / R[l][l] in a register, so the back
  // substitution needs no masking.
#pragma unroll
  for (int j = 0; j < NL; j += 2) *reinterpret_cast<double2 *>(&Tv[l * NL + j]) = make_double2(0.0, 0.0);
  int q = 0;           // active-set size
  double um = 0.0;     // multiplier of active position l
  int iam = -1;        // constraint index at active position l
  double invRd = 0.0;  // 1 / R[l][l]
  int status;
  bool done;
  {
    // any lane seeing an infeasible zero row marks the whole QP
    const double bad = row_min(infeasible_row ? -1.0 : 0.0);
    const bool inf0 = bad < 0.0;
    status = !spd ? QPB_NOT_SPD : (inf0 ? QPB_INFEASIBLE : QPB_MAX_ITER);
    done = !spd || inf0;
  }
  bool selecting = true;
  int p = 0;
  double up = 0.0;  // multiplier of the constraint being added
  int it = 0;
  wave_lds_sync();
  clk.tick(3);

  while (!done && it < max_iter) {
    ++it;
    if (selecting) {
      // The violation test is fp64 on the slack normalised by |a_row| (the
      // feasibility tolerance); among the violated rows the argmax runs on
      // 32-bit keys: the fp32 violation per unit length of the row's free
      // part, -s / |D[r, q:]| (dual steepest edge: 4.66 instead of 5.05
      // iterations per QP on the bench family, 6.18 instead of 6.97 on the
      // dense one, tools/gi_select_sim.py), row index in the low 5 bits, so
      // one DPP-fused v_max_u32 per step reduces the row (0 = none violated)
      uint32_t key = 0u;
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        const bool viol = !act[r] && s[r] < thr[r];
        // fn2 in [0, FLT_MAX] (clamped where it shrinks); the 2^-100 floor keeps
        // a violated row's key above 31 -- never 0, the "none violated" key --
        // when the ratio underflows (row 0 included)
        const float kf = __builtin_fmaf((float)(-s[r]), __builtin_amdgcn_rsqf(fn2[r]), 0x1p-100f);
        const uint32_t kr = (__float_as_uint(kf) & ~31u) | (uint32_t)(l + NL * r);
        key = viol && kr > key ? kr : key;
      }
      key = row_max_u32(key);
      if (key == 0u) {
        status = QPB_OK;
        done = true;
        break;
      }
      p = (int)(key & 31u);
      up = 0.0;
      selecting = false;
    }
    clk.tick(4);
    // wave-uniform bound on the active set size (q <= NL always; the clamp
    // keeps every R column loop inside the QP's slot regardless)
    const int qmax = __builtin_elementwise_min(wave_max4(q), NL);

    // ---- row p of D, s_p and |D[p,:]|^2 through the exchange row; lane l
    // keeps its entry D[p][l] (d = -D[p,:] in G-I's sign convention; the
    // signs are folded into the formulas below)
    const int owner = p & (NL - 1), prow = p >> 4;
    if (l == owner) {
#pragma unroll
      for (int r = 0; r < MR; ++r)
        if (r == prow) {
#pragma unroll
          for (int j = 0; j < NL; j += 2) *reinterpret_cast<double2 *>(&xch[j]) = make_double2(E[r][j], E[r][j + 1]);
          *reinterpret_cast<double2 *>(xsd) = make_double2(s[r], (double)ddr[r]);
        }
    }
    wave_lds_sync();
    const double Dpl = xch[l];
    const double2 spdd = *reinterpret_cast<const double2 *>(xsd);
    const double Dpq = xch[q & (NL - 1)];  // q == 16: an ADD is impossible (d2 = 0)
    const double sp = spdd.x, dd = spdd.y;  // s_p, |D[p,:]|^2
    wave_lds_sync();
    const double d2 = (l >= q) ? Dpl : 0.0;  // D[p, q:]
    dpp_ready(d2);
    // slack direction D d2 (d2 read from lane j by the FMAs)
    double u[MR];
    bdot_rows<MR>(d2, E, u);
    const double nd2 = row_sum(d2 * d2);  // |d2|^2
    clk.tick(5);

    // ---- r = R^{-1} d1: lane-parallel back substitution over the active positions
    double rm = 0.0;
    if (qmax > 0) {
      // on the negated accumulator: nacc_l += R[l][j] * r_j, r_j = nacc_j * (-1/R_jj)
      // read from lane j by the FMA itself (the product was written just
      // before: fmac_bc_nop issues the DPP read hazard's wait states)
      const double ninv = -invRd;
      double nacc = (l < q) ? Dpl : 0.0;  // = -d1_l
      unroll<NL>([&](auto JJ) {
        constexpr int j = NL - 1 - JJ;
        // (column 0 holds no entry above the diagonal: skipped)
        if (j > 0 && j < qmax) fmac_bc_nop<j>(nacc, nacc * ninv, Tv[j * NL + l]);
      });
      rm = nacc * ninv;  // r_l (0 for l >= q)
    }
    clk.tick(6);

    // ---- step lengths
    double t1 = kBig;
    int k = 0;
    if (qmax > 0) {
      // the exact minimum ratio, then the lowest position attaining it
      const double ratio = um * rcp1(rm);
      const bool cand = l < q && rm > 0.0;
      t1 = row_min_raw(cand ? ratio : kBig);
      k = (int)row_min_u32(cand && ratio == t1 ? (uint32_t)l : 31u) & (NL - 1);
    }
    const double ir = rsq1(nd2);  // 1/|d2| (only used when nd2 > 0)
    const double t2 = (nd2 > kDepTol * dd) ? -sp * (ir * ir) : kBig;
    const double t = t1 < t2 ? t1 : t2;
    if (!(t < kBig)) {
      status = QPB_INFEASIBLE;
      done = true;
      break;
    }
    if (t2 < kBig) {  // primal step: slacks s -= t A z,  A z = -D[:, q:] d2
#pragma unroll
      for (int r = 0; r < MR; ++r) s[r] = __builtin_fma(t, u[r], s[r]);
    }
    um = __builtin_fma(-t, rm, um);
    up += t;
    clk.tick(7);

    if (t2 <= t1) {
      // ---------------- ADD p: Householder on columns q.. of D.  With
      // dq = -D[p,q]: alpha = -sign(dq) |d2|, v = d2 + alpha e_q (the negated
      // G-I vector: same reflection), beta = 1 / (|d2|^2 + alpha D[p,q]) =
      // 1 / (|d2| (|d2| + |D[p,q]|)): one reciprocal.
      const double nrm = nd2 * ir;
      const bool neg = Dpq <= 0.0;
      const double alpha = neg ? -nrm : nrm;
      const double beta = ir * rcp1(nrm + __builtin_fabs(Dpq));
      const double ia = neg ? -ir : ir;  // 1 / alpha
      const double v = d2 + (l == q ? alpha : 0.0);
      // E v = E d2 + alpha E[:, q] = u + alpha E[:, q]: no second product;
      // column q by a branch tree on q (its distinct values in the wave)
      double nw[MR];
      switch (q & (NL - 1)) {
#define QPB_COLQ_CASE(J)                                        \
  case J:                                                        \
    asm volatile("");                                            \
    for (int r = 0; r < MR; ++r) nw[r] = E[r][J];                \
    break;
        QPB_COLQ_CASE(0) QPB_COLQ_CASE(1) QPB_COLQ_CASE(2) QPB_COLQ_CASE(3)
        QPB_COLQ_CASE(4) QPB_COLQ_CASE(5) QPB_COLQ_CASE(6) QPB_COLQ_CASE(7)
        QPB_COLQ_CASE(8) QPB_COLQ_CASE(9) QPB_COLQ_CASE(10) QPB_COLQ_CASE(11)
        QPB_COLQ_CASE(12) QPB_COLQ_CASE(13) QPB_COLQ_CASE(14) QPB_COLQ_CASE(15)
#undef QPB_COLQ_CASE
      }
#pragma unroll
      for (int r = 0; r < MR; ++r) nw[r] = -beta * __builtin_fma(alpha, nw[r], u[r]);
      dpp_ready(v);
#pragma unroll
      for (int r = 0; r < MR; ++r) unroll<NL>([&](auto J) {
          constexpr int j = J;
          fmac_bc<j>(E[r][j], v, nw[r]);
        });
      // the reflection maps e_q to -d2 / alpha: column q of the new D is
      // -u / alpha, and it leaves the free part of every row
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        const float c = (float)(u[r] * ia);
        fn2[r] = __builtin_fmaxf(__builtin_fmaf(-c, c, fn2[r]), 0.0f);
      }
      // new column q of R: d1 strictly above the diagonal, alpha on it
      Tv[q * NL + l] = (l < q) ? -Dpl : 0.0;
      if (l == q) {
        invRd = ia;
        iam = p;
        um = up;
      }
#pragma unroll
      for (int r = 0; r < MR; ++r) act[r] = act[r] || (l == owner && r == prow);
      ++q;
      selecting = true;
      clk.tick(8);
    } else {
      // ---------------- DROP active position k
      const int c = __shfl(iam, k, NL);
#pragma unroll
      for (int r = 0; r < MR; ++r) act[r] = act[r] && !(l == (c & (NL - 1)) && r == (c >> 4));
      const double un = __shfl(um, (l + 1) & (NL - 1), NL);
      const int in = __shfl(iam, (l + 1) & (NL - 1), NL);
      if (l >= k && l < q - 1) {
        um = un;
        iam = in;
      } else if (l == q - 1) {
        um = 0.0;
        iam = -1;
      }
      // full R (diagonal put back), delete column k: lane l (column l) reads
      // column l + 1 whole, then writes it (in-order DS: every read precedes
      // every write)
      wave_lds_sync();
      if (l < q) Tv[l * NL + l] = rcp1(invRd);  // R[l][l] (alpha when it was added)
      wave_lds_sync();
      {
        double col[NL];
        lds_row16(&Tv[((l + 1) & (NL - 1)) * NL], col);
        wave_lds_sync();
        if (l >= k && l < q - 1) {
#pragma unroll
          for (int j = 0; j < NL; j += 2) *reinterpret_cast<double2 *>(&Tv[l * NL + j]) = make_double2(col[j], col[j + 1]);
        } else if (l == q - 1) {
#pragma unroll
          for (int j = 0; j < NL; j += 2) *reinterpret_cast<double2 *>(&Tv[l * NL + j]) = make_double2(0.0, 0.0);
        }
      }
      // Givens rotations restore the upper-triangular R; lane j keeps the
      // parameters of rotation j, which the unrolled D update reads by DPP
      double gc = 0.0, gs = 0.0;
      for (int j = k; j < q - 1; ++j) {
        wave_lds_sync();
        const double a = Tv[j * NL + j], bb = Tv[j * NL + j + 1];
        const double irr = rsq1(__builtin_fma(a, a, bb * bb));
        const double cj = a * irr, sj = bb * irr;
        const double rj = Tv[l * NL + j], rj1 = Tv[l * NL + j + 1];
        wave_lds_sync();
        if (l >= j && l < q - 1) {
          Tv[l * NL + j] = __builtin_fma(cj, rj, sj * rj1);
          Tv[l * NL + j + 1] = (l == j) ? 0.0 : __builtin_fma(-sj, rj, cj * rj1);
        }
        if (l == j) {
          gc = cj;
          gs = sj;
        }
      }
      wave_lds_sync();
      Tv[l * NL + q - 1] = 0.0;
      unroll<NL - 1>([&](auto JJ) {
        constexpr int j = JJ;
        if (j + 1 < qmax && j >= k && j < q - 1) {
          const double cj = bc<j>(gc), sj = bc<j>(gs);
#pragma unroll
          for (int r = 0; r < MR; ++r) {
            const double e0 = E[r][j], e1 = E[r][j + 1];
            E[r][j] = __builtin_fma(cj, e0, sj * e1);
            E[r][j + 1] = __builtin_fma(-sj, e0, cj * e1);
          }
        }
      });
      --q;
      // column q (after the rotations) joins the free part: recompute
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        float a0 = 0.0f, a1 = 0.0f;
        unroll<NL>([&](auto J) {
          constexpr int j = J;
          const float e = (float)E[r][j];
          if constexpr (j % 2 == 0) a0 = __builtin_fmaf(e, j >= q ? e : 0.0f, a0);
          if constexpr (j % 2 == 1) a1 = __builtin_fmaf(e, j >= q ? e : 0.0f, a1);
        });
        fn2[r] = a0 + a1;
      }
      // back to the zero-diagonal form
      wave_lds_sync();
      const double dg = (l < q) ? Tv[l * NL + l] : 0.0;
      wave_lds_sync();
      if (l < q) Tv[l * NL + l] = 0.0;
      invRd = (l < q) ? rcp1(dg) : 0.0;
      clk.tick(9);
    }
    wave_lds_sync();
  }
  clk.tick(10);

  // ------------------------------------------------------------- outputs
  // (the active rows of A re-read, one coalesced 128-B row per active position)
  const int qm = __builtin_elementwise_min(wave_max4(q), NL);
  // The QP index and its A block again, recomputed from an opaque copy of the
  // slot instead of held across the loop (held, the allocator spilled them)
  int slot_o = slot;
  asm volatile("" : "+v"(slot_o));
  const long long go = live ? grp * QPB + slot_o : batch - 1;
  const long long gio = (flags & QPB_FLAG_DIAG_L2) ? (go & 511) : (flags & QPB_FLAG_DIAG_MALL) ? (go & 16383) : go;
  const double *Aqo = m > 0 ? Ag + gio * (long long)m * n : Hg + gio * (long long)n * n;
  // The A-row loads go out first, in at most two groups of eight (one
  // wave-uniform test per group: a test per load made each load a branch
  // with its own wait); the work that does not need them -- the multipliers by
  // row and their stores, the active-set word, L's row -- runs while they are
  // in flight.  Positions past qm read a valid row and are not summed.
  const int ias = iam > 0 ? iam : 0;
  asm volatile("s_nop 1" ::"v"(ias));  // its DPP reads below may sit behind a branch only
  const int lc = l < n ? l : n - 1;
  double arow[NL];
  unroll<2>([&](auto H) {
    constexpr int k0 = 8 * H;
    if (k0 < qm) {
      __builtin_amdgcn_sched_barrier(0);
      unroll<8>([&](auto K) {
        constexpr int kk = k0 + K;
        arow[kk] = Aqo[bci<kk>(ias) * n + lc];
      });
    }
  });
  double *lamb = Tv;  // lambda scatter (32) over the dead R; the solves below capture in Tv[32:48]
  double *xcap = Tv + 2 * NL;
#pragma unroll
  for (int r = 0; r < 2; ++r) lamb[l + NL * r] = 0.0;
  wave_lds_sync();
  if (l < q && iam >= 0) lamb[iam] = um;
  wave_lds_sync();
  double lamr[MR];
#pragma unroll
  for (int r = 0; r < MR; ++r) lamr[r] = lamb[l + NL * r];
  const double invd = rcp1(Lp[lrow(l) + l]);
  double Lrow[NL];  // row l of L (entries past l are dead)
#pragma unroll
  for (int j = 0; j < NL; ++j) Lrow[j] = Lp[lrow(l) + j];
  wave_lds_sync();
#pragma unroll
  for (int r = 0; r < MR; ++r) {
    const int row = l + NL * r;
    if (live && (FULL || row < m)) lamg[go * m + row] = lamr[r];
  }
  uint32_t w0 = 0;
#pragma unroll
  for (int r = 0; r < MR; ++r) {
    const unsigned long long bal = __ballot(act[r]);
    w0 |= (uint32_t)((bal >> sh) & 0xFFFFull) << (16 * r);
  }
  if (live && l == 0 && m > 0) actg[go] = w0;
  // x = -H^{-1} (f + A^T lam): g = f + sum_k u_k a_{iam_k}, then L y = g,
  // L^T x = -y, lane-parallel: step k broadcasts the finished component from
  // lane k; finished lanes keep updating (dead values) and the components are
  // captured by same-address LDS stores.
  double gl = fl;
  unroll<2>([&](auto H) {
    constexpr int k0 = 8 * H;
    if (k0 < qm) {
      unroll<8>([&](auto K) {
        constexpr int kk = k0 + K;
        if (kk < qm) gl = __builtin_fma(bc<kk>(um), (N16 || l < n) ? arow[kk] : 0.0, gl);
      });
    }
  });
  {
    double acc = gl;
    unroll<NL>([&](auto K) {
      constexpr int kk = K;
      const double yk = bc<kk>(acc * invd);
      acc = __builtin_fma(-Lrow[kk], yk, acc);
      xcap[kk] = yk;
    });
  }
  wave_lds_sync();
  {
    double acc = xcap[l];
    wave_lds_sync();
    unroll<NL>([&](auto K) {
      constexpr int kk = NL - 1 - K;
      const double xk = bc<kk>(acc * invd);
      acc = __builtin_fma(-Lp[lrow(kk) + l], xk, acc);
      xcap[kk] = xk;
    });
  }
  wave_lds_sync();
  const double xl = -xcap[l];
  {
    // a non-finite x on any lane -> NUMERICAL for the QP
    const double bad = row_min((__builtin_fabs(xl) < kInf) ? 0.0 : -1.0);
    if (status == QPB_OK && bad < 0.0) status = QPB_NUMERICAL;
  }
  if (live && (N16 || l < n)) xg[go * n + l] = xl;
  if (live && l == 0) {
    statg[go] = status;
    if (itg) itg[go] = it;
  }
  clk.tick(11);
  clk.flush(dbg);
}

template <int MR, bool N16, bool FULL, bool STAMP = false, int OCC = 2>
__global__ __launch_bounds__(64, OCC) void gi_dense_kernel(
    const double *__restrict__ Hg, const double *__restrict__ fg, const double *__restrict__ Ag,
    const double *__restrict__ bg, double *__restrict__ xg, double *__restrict__ lamg,
    uint32_t *__restrict__ actg, int32_t *__restrict__ statg, int32_t *__restrict__ itg, int n, int m,
    long long batch, int max_iter, double feas_tol, int flags = 0,
    unsigned long long *__restrict__ dbg = nullptr) {
  __shared__ double lds[QPB * SLOT];
#ifdef QPB_WAVE_TRACE
  // diagnostic build only (tools/wave_timeline.py): each wave's start and end
  // on the 100 MHz real-time and the shader clocks, and where it ran
  unsigned long long rt0, mt0, rt1, mt1;
  unsigned hw, xcc;
  asm volatile("s_memrealtime %0\n\ts_memtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(rt0), "=s"(mt0)::"memory");
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
#endif
  gi_group<MR, N16, FULL, STAMP>(lds, Hg, fg, Ag, bg, xg, lamg, actg, statg, itg, n, m, batch, max_iter, feas_tol,
#ifdef QPB_WAVE_TRACE
                                 flags, dbg, blockIdx.x);
#else
                                 flags, STAMP ? dbg : nullptr, blockIdx.x);
#endif
#ifdef QPB_WAVE_TRACE
#if QPB_WAVE_TRACE == 2
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the end after the output stores have drained
#endif
  asm volatile("s_memrealtime %0\n\ts_memtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(rt1), "=s"(mt1)::"memory");
  if (!STAMP && dbg && threadIdx.x == 0) {
    unsigned long long *r = dbg + 8ull * blockIdx.x;
    r[0] = rt0;
    r[1] = rt1;
    r[2] = mt0;
    r[3] = mt1;
    r[4] = hw | ((unsigned long long)xcc << 32);
  }
#endif
}

}  // namespace qpb

// launcher used by qpb_api.hip
extern "C" hipError_t qpb_launch_gi(const qpb_desc *d, const double *H, const double *f, const double *A,
                                    const double *b, double *x, double *lam, uint32_t *active,
                                    int32_t *status, int32_t *iters, hipStream_t stream) {
  const long long blocks = (d->batch + qpb::QPB - 1) / qpb::QPB;
  const int max_iter = d->max_iter > 0 ? d->max_iter : 4 * (d->n + d->m) + 8;
  const double tol = d->feas_tol > 0 ? d->feas_tol : 1e-10;
#define QPB_GI_LAUNCH(MR, N16, FULL)                                                                               \
  hipLaunchKernelGGL((qpb::gi_dense_kernel<MR, N16, FULL, false, 3>), dim3((unsigned)blocks), dim3(64), 0, stream, \
                     H, f, A, b, x, lam, active, status, iters, d->n, d->m, (long long)d->batch, max_iter, tol,    \
                     d->flags)
  const bool n16 = d->n == 16;
  if (d->m <= 16) {
    if (n16 && d->m == 16) QPB_GI_LAUNCH(1, true, true);
    else if (n16) QPB_GI_LAUNCH(1, true, false);
    else QPB_GI_LAUNCH(1, false, false);
  } else {
    if (n16 && d->m == 32) QPB_GI_LAUNCH(2, true, true);  // 3 waves per SIMD (VGPRs and LDS)
    else if (n16) QPB_GI_LAUNCH(2, true, false);
    else QPB_GI_LAUNCH(2, false, false);
  }
#undef QPB_GI_LAUNCH
  return hipGetLastError();
}

// diagnostic: per-section wave ticks of the n=16, 16<m<=32 kernel (sections[256][20])
extern "C" hipError_t qpb_launch_gi_sections(const qpb_desc *d, const double *H, const double *f, const double *A,
                                             const double *b, double *x, double *lam, uint32_t *active,
                                             int32_t *status, int32_t *iters, unsigned long long *sections,
                                             hipStream_t stream) {
  const long long blocks = (d->batch + qpb::QPB - 1) / qpb::QPB;
  const int max_iter = d->max_iter > 0 ? d->max_iter : 4 * (d->n + d->m) + 8;
  const double tol = d->feas_tol > 0 ? d->feas_tol : 1e-10;
  if (d->n != 16 || d->m <= 16) return hipErrorInvalidValue;
#ifdef QPB_WAVE_TRACE
  // the diagnostic build launches the shipped kernel and writes 8 words per
  // wave: the caller's buffer holds 8 * ceil(batch / 4) (tools/wave_timeline.py)
  if (d->m == 32) {
    hipLaunchKernelGGL((qpb::gi_dense_kernel<2, true, true, false, 3>), dim3((unsigned)blocks), dim3(64), 0, stream,
                       H, f, A, b, x, lam, active, status, iters, d->n, d->m, (long long)d->batch, max_iter, tol,
                       d->flags, sections);
    return hipGetLastError();
  }
#endif
  hipLaunchKernelGGL((qpb::gi_dense_kernel<2, true, false, true>), dim3((unsigned)blocks), dim3(64), 0, stream, H, f,
                     A, b, x, lam, active, status, iters, d->n, d->m, (long long)d->batch, max_iter, tol, d->flags,
                     sections);
  return hipGetLastError();
}
