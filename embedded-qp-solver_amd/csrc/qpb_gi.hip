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
//   setup   H = L L^T (Cholesky, row l of H in lane l, left-looking, row k of
//           L broadcast by DPP row_newbcast); D = A L^{-T}, y = L^{-1} f by
//           forward substitution (row k of L read from LDS);
//           slack of the unconstrained minimiser x0 = -H^{-1} f
//           (test/qp_ref.py:35's answer): s = b - A x0 = b + D y.
//   iterate pick the most violated row p (normalised slack, exact row min);
//           d = -D[p,:] (= J^T n+ in G-I's notation, J = L^{-T} Q, n+ = -a_p),
//           dual step r = R^{-1} d1 (lane-parallel back substitution),
//           partial step t1 (ratio test over the active multipliers),
//           full step t2 = -s_p / |d2|^2, slacks s -= t D[:, q:] d2;
//           full step  -> ADD p: one Householder reflection on columns q..15
//                         of D (every lane updates its own rows), new column
//                         of R;
//           partial    -> DROP k: delete column k of R, Givens rotations
//                         restore triangularity (also applied to D).
//   finish  x = -H^{-1} (f + A^T lam) from the final multipliers (KKT
//           stationarity): the q active rows of A are re-read, two triangular
//           solves with L kept in LDS.
//
// Data layout per QP (lane l = 0..15 of the QP's 16-lane DPP row):
//   registers  rows l + 16 r (r < MR) of D, their slacks, 1/||a_row||,
//              |D row|^2, active flags; multiplier / row of active position l
//   LDS        L (packed lower triangle, reciprocal diagonal), R (16 x 18
//              padded rows, zero diagonal + separate diagonal), exchange row,
//              Givens parameters, lambda scatter buffer.  The R area doubles
//              as the staging buffer of the coalesced input transposes.
#include "qpb_common.h"
#include "qpb.h"

namespace qpb {

constexpr int NL = 16;  // lanes per QP
constexpr int QPB = 4;  // QPs per workgroup (one wavefront)
constexpr int RS = 18;  // R row stride (doubles): conflict-free b64 / b128 row access

// packed lower triangle of L with even-length rows (16-byte aligned b128
// reads): row i starts at sum_{j<i} roundup(j+1, 2) = 2u(u+1) (i = 2u) or
// 2(u+1)^2 (i = 2u+1)
__host__ __device__ constexpr int lrow(int i) {
  const int u = i >> 1;
  return (i & 1) ? 2 * (u + 1) * (u + 1) : 2 * u * (u + 1);
}
constexpr int L_SIZE = lrow(NL);  // 144

constexpr int OFF_L = 0;
constexpr int OFF_R = OFF_L + L_SIZE;     // 144: R, 16 x RS
constexpr int OFF_XCH = OFF_R + 16 * RS;  // 432: d (16), s_p, |d|^2
constexpr int OFF_CS = OFF_XCH + 18;      // Givens cosines (16)
constexpr int OFF_SN = OFF_CS + 16;       // Givens sines (16)
constexpr int OFF_RDG = OFF_SN + 16;      // diagonal of R (16)
constexpr int OFF_LAM = OFF_RDG + 16;     // lambda scatter (32)
constexpr int SLOT = OFF_LAM + 32;        // 530 doubles per QP
constexpr double kDepTol = 1e-24;         // |d2|^2 <= kDepTol |d|^2  <=>  z = 0

// Diagnostic build only (STAMP = true, qpb_solve_sections): s_memrealtime stamps (100 MHz)
// accumulate each wave's cycles per kernel section; the real kernel has none.
constexpr int kSections = 12;
template <bool ON>
struct SectionClock {
  __device__ __forceinline__ void tick(int) {}
  __device__ __forceinline__ void flush(unsigned long long *) {}
};
template <>
struct SectionClock<true> {
  unsigned long long last, acc[kSections];
  __device__ __forceinline__ unsigned long long now() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
  }
  __device__ __forceinline__ SectionClock() {
    for (int i = 0; i < kSections; ++i) acc[i] = 0;
    last = now();
  }
  __device__ __forceinline__ void tick(int i) {
    const unsigned long long t = now();
    acc[i] += t - last;
    last = t;
  }
  __device__ __forceinline__ void flush(unsigned long long *dbg) {
    if ((threadIdx.x & 63) == 0)
      for (int i = 0; i < kSections; ++i) atomicAdd(&dbg[i], acc[i]);
  }
};

// sum_{j<N} x(j) y(j) with 4 independent accumulators: short dependency
// chains (the kernel is latency-bound at 2-3 waves per SIMD)
template <int N, class FX, class FY>
__device__ __forceinline__ double dot4(FX &&x, FY &&y, double init = 0.0) {
  double a0 = init, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  unroll<N>([&](auto J) {
    constexpr int j = J;
    if constexpr (j % 4 == 0) a0 = __builtin_fma(x(j), y(j), a0);
    if constexpr (j % 4 == 1) a1 = __builtin_fma(x(j), y(j), a1);
    if constexpr (j % 4 == 2) a2 = __builtin_fma(x(j), y(j), a2);
    if constexpr (j % 4 == 3) a3 = __builtin_fma(x(j), y(j), a3);
  });
  return (a0 + a1) + (a2 + a3);
}

template <int MR, bool N16, bool STAMP = false>
__global__ __launch_bounds__(64, 2) void gi_dense_kernel(
    const double *__restrict__ Hg, const double *__restrict__ fg, const double *__restrict__ Ag,
    const double *__restrict__ bg, double *__restrict__ xg, double *__restrict__ lamg,
    uint32_t *__restrict__ actg, int32_t *__restrict__ statg, int32_t *__restrict__ itg, int n, int m,
    long long batch, int max_iter, double feas_tol, int flags = 0,
    unsigned long long *__restrict__ dbg = nullptr) {
  __shared__ double lds[QPB * SLOT];
  SectionClock<STAMP> clk;
  const int l = threadIdx.x & (NL - 1);
  const int slot = threadIdx.x >> 4;
  const long long g = (long long)blockIdx.x * QPB + slot;
  if (g >= batch) return;  // whole 16-lane rows leave together

  double *Lp = lds + slot * SLOT + OFF_L;
  double *R = lds + slot * SLOT + OFF_R;
  double *xch = lds + slot * SLOT + OFF_XCH;
  double *gcs = lds + slot * SLOT + OFF_CS;
  double *gsn = lds + slot * SLOT + OFF_SN;
  double *Rdg = lds + slot * SLOT + OFF_RDG;
  double *lamb = lds + slot * SLOT + OFF_LAM;

  // ------------------------------------------------------------------ load
  // (flags & QPB_FLAG_DIAG_L2: every QP reads the inputs of QP g mod 64 --
  // a diagnostic that takes HBM latency out of the kernel time)
  const long long gi = (flags & 1) ? (g & 63) : g;
  const double *Hq = Hg + gi * (long long)n * n;
  // m == 0: A/b may be NULL -- point the (masked) row loads at H instead
  const double *Aq = m > 0 ? Ag + gi * (long long)m * n : Hq;
  const double *bq = m > 0 ? bg + gi * (long long)m : Hq;
  double Lr[NL];  // row l of H, becomes row l of L
  double E[MR][NL];
  double s[MR], invn[MR], bl[MR], dn[MR];
  bool act[MR];
  bool infeasible_row = false;
  if (N16) {
    // Coalesced 16-byte loads: one instruction reads 2 whole rows (256 B) of
    // each of the wave's 4 QPs -- lane l gets row 2t + (l>>3), columns
    // 2(l&7), 2(l&7)+1.  Rows reach their owner lane through a transpose in
    // this QP's R region of LDS (free until the active-set loop).
    const int hr = l >> 3, hc = 2 * (l & 7);
    double2 hv[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) hv[t] = *reinterpret_cast<const double2 *>(&Hq[(2 * t + hr) * NL + hc]);
    double2 av[MR][8];
#pragma unroll
    for (int r = 0; r < MR; ++r)
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int row = NL * r + 2 * t + hr;
        av[r][t] = row < m ? *reinterpret_cast<const double2 *>(&Aq[row * NL + hc]) : make_double2(0.0, 0.0);
      }
#pragma unroll
    for (int t = 0; t < 8; ++t) *reinterpret_cast<double2 *>(&R[(2 * t + hr) * RS + hc]) = hv[t];
    wave_lds_sync();
#pragma unroll
    for (int j = 0; j < NL; j += 2) {
      const double2 v = *reinterpret_cast<const double2 *>(&R[l * RS + j]);
      Lr[j] = v.x;
      Lr[j + 1] = v.y;
    }
#pragma unroll
    for (int r = 0; r < MR; ++r) {
      wave_lds_sync();
#pragma unroll
      for (int t = 0; t < 8; ++t) *reinterpret_cast<double2 *>(&R[(2 * t + hr) * RS + hc]) = av[r][t];
      wave_lds_sync();
#pragma unroll
      for (int j = 0; j < NL; j += 2) {
        const double2 v = *reinterpret_cast<const double2 *>(&R[l * RS + j]);
        E[r][j] = v.x;
        E[r][j + 1] = v.y;
      }
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
    }
  }
#pragma unroll
  for (int r = 0; r < MR; ++r) {
    const int row = l + NL * r;
    const bool ok = row < m;
    const double nrm2 = dot4<NL>([&](int j) { return E[r][j]; }, [&](int j) { return E[r][j]; });
    const double bv = bq[ok ? row : 0];
    bl[r] = ok ? bv : 0.0;
    invn[r] = nrm2 > 0.0 ? rsq(nrm2) : 0.0;
    // a zero row is the constant constraint 0 <= b
    infeasible_row = infeasible_row || (ok && nrm2 == 0.0 && bl[r] < -feas_tol * (1.0 + __builtin_fabs(bl[r])));
    act[r] = false;
  }
  const double fv = fg[gi * n + (l < n ? l : n - 1)];
  const double fl = (l < n) ? fv : 0.0;
  double yf[NL];
  unroll<NL>([&](auto J) { yf[J] = bc<J>(fl); });  // f replicated on every lane
  clk.tick(0);

  // ---- Cholesky H = L L^T (left-looking: step k broadcasts row k of L from
  // lane k by DPP row_newbcast and finishes column k on every lane)
  bool spd = true;
  unroll<NL>([&](auto K) {
    constexpr int k = K;
    __builtin_amdgcn_sched_barrier(0);
    const double a = Lr[k] - dot4<k>([&](int j) { return Lr[j]; }, [&](int j) { return bc<k>(Lr[j]); });
    const double akk = bc<k>(a);
    spd = spd && (akk > 0.0);
    const double ik = rsq(akk);
    // row l keeps L[l][0..l]; the diagonal is stored as its reciprocal
    Lr[k] = (l > k) ? a * ik : ((l == k) ? ik : 0.0);
  });
  // L -> LDS, packed rows (lane l writes row l), kept for the final solves
  unroll<NL / 2>([&](auto J) {
    constexpr int j = 2 * J;
    if (j <= l) *reinterpret_cast<double2 *>(&Lp[lrow(l) + j]) = make_double2(Lr[j], Lr[j + 1]);
  });
  wave_lds_sync();
  clk.tick(1);

  // ---- forward substitutions, row k of L read from LDS (same address on the
  // QP's 16 lanes: broadcast reads): D = A L^{-T} (rows l, l+16), y = L^{-1} f
  unroll<NL>([&](auto K) {
    constexpr int k = K;
    __builtin_amdgcn_sched_barrier(0);
    double Lk[k + 2];
    unroll<(k + 2) / 2>([&](auto J) {
      const double2 v = *reinterpret_cast<const double2 *>(&Lp[lrow(k) + 2 * J]);
      Lk[2 * J] = v.x;
      Lk[2 * J + 1] = v.y;
    });
    const double ik = Lk[k];
#pragma unroll
    for (int r = 0; r < MR; ++r)
      E[r][k] = (E[r][k] - dot4<k>([&](int j) { return Lk[j]; }, [&](int j) { return E[r][j]; })) * ik;
    yf[k] = (yf[k] - dot4<k>([&](int j) { return Lk[j]; }, [&](int j) { return yf[j]; })) * ik;
  });
#pragma unroll
  for (int r = 0; r < MR; ++r) {
    s[r] = dot4<NL>([&](int j) { return E[r][j]; }, [&](int j) { return yf[j]; }, bl[r]);
    dn[r] = dot4<NL>([&](int j) { return E[r][j]; }, [&](int j) { return E[r][j]; });
  }
  clk.tick(2);

  // ------------------------------------------------------ active-set loop
  // R (upper triangular, active columns) lives in LDS with a ZERO diagonal;
  // the diagonal is kept in Rdg[] (and 1/R[l][l] in a register) so the back
  // substitution needs no masking.
#pragma unroll
  for (int j = 0; j < RS; j += 2) *reinterpret_cast<double2 *>(&R[l * RS + j]) = make_double2(0.0, 0.0);
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
      // most violated row by normalised slack; the key carries the row index
      double key = kBig;
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        const double v = s[r] * invn[r];
        const bool viol = !act[r] && invn[r] > 0.0 && v < -feas_tol * (1.0 + __builtin_fabs(bl[r]) * invn[r]);
        key = viol ? __builtin_fmin(key, pack_key(v, l + NL * r)) : key;
      }
      key = row_min(key);
      if (!(key < 0.0)) {  // no violated row (violations are negative keys)
        status = QPB_OK;
        done = true;
        break;
      }
      p = key_index(key);
      up = 0.0;
      selecting = false;
    }
    clk.tick(4);
    const int qmax = wave_max4(q);  // wave-uniform bound on the active set size

    // ---- d = -D[p,:] and s_p to every lane through the exchange row
    const int owner = p & (NL - 1), prow = p >> 4;
    if (l == owner) {
#pragma unroll
      for (int r = 0; r < MR; ++r)
        if (r == prow) {
#pragma unroll
          for (int j = 0; j < NL; j += 2) *reinterpret_cast<double2 *>(&xch[j]) = make_double2(E[r][j], E[r][j + 1]);
          xch[NL] = s[r];
          xch[NL + 1] = dn[r];
        }
    }
    wave_lds_sync();
    double d2[NL];  // -D[p, q:] (zero in the active columns)
#pragma unroll
    for (int j = 0; j < NL; j += 2) {
      const double2 v = *reinterpret_cast<const double2 *>(&xch[j]);
      d2[j] = (j >= q) ? -v.x : 0.0;
      d2[j + 1] = (j + 1 >= q) ? -v.y : 0.0;
    }
    const double sp = xch[NL];
    const double dd = xch[NL + 1];  // |D[p,:]|^2 (invariant under the column rotations)
    const double dl = -xch[l];
    const double dq = (q < NL) ? -xch[q] : 0.0;
    const double nd2 = dot4<NL>([&](int j) { return d2[j]; }, [&](int j) { return d2[j]; });
    clk.tick(5);

    // ---- r = R^{-1} d1: lane-parallel back substitution over the active positions
    double rm = 0.0;
    if (qmax > 0) {
      double acc = (l < q) ? dl : 0.0;
      unroll<NL>([&](auto JJ) {
        constexpr int j = NL - 1 - JJ;
        if (j < qmax) acc = __builtin_fma(-R[l * RS + j], bc<j>(acc * invRd), acc);
      });
      rm = acc * invRd;  // r_l (0 for l >= q)
    }
    clk.tick(6);

    // ---- step lengths
    double t1 = kBig;
    int k = 0;
    if (qmax > 0) {
      const double tk = row_min((l < q && rm > 0.0) ? pack_key(um * rcp(rm), l) : kBig);
      t1 = tk;
      k = key_index(tk);
    }
    const double t2 = (nd2 > kDepTol * dd) ? -sp * rcp(nd2) : kBig;
    const double t = t1 < t2 ? t1 : t2;
    if (!(t < kBig)) {
      status = QPB_INFEASIBLE;
      done = true;
      break;
    }
    if (t2 < kBig) {  // primal step: slacks s -= t A z,  A z = D[:, q:] d2
#pragma unroll
      for (int r = 0; r < MR; ++r)
        s[r] = __builtin_fma(-t, dot4<NL>([&](int j) { return E[r][j]; }, [&](int j) { return d2[j]; }), s[r]);
    }
    um = __builtin_fma(-t, rm, um);
    up += t;
    clk.tick(7);

    if (t2 <= t1) {
      // ---------------- ADD p: Householder on columns q.. of D
      const double nrm = __builtin_sqrt(nd2);
      const double alpha = dq >= 0.0 ? -nrm : nrm;
      const double beta = rcp(nd2 - alpha * dq);
#pragma unroll
      for (int j = 0; j < NL; ++j) d2[j] -= (j == q) ? alpha : 0.0;  // d2 -> Householder vector
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        const double w = beta * dot4<NL>([&](int j) { return E[r][j]; }, [&](int j) { return d2[j]; });
#pragma unroll
        for (int j = 0; j < NL; ++j) E[r][j] = __builtin_fma(-w, d2[j], E[r][j]);
      }
      // new column q of R: d1 strictly above the diagonal, alpha on it
      R[l * RS + q] = (l < q) ? dl : 0.0;
      if (l == q) {
        Rdg[q] = alpha;
        invRd = rcp(alpha);
        iam = p;
        um = up;
      }
      if (l == owner) {
#pragma unroll
        for (int r = 0; r < MR; ++r)
          if (r == prow) act[r] = true;
      }
      ++q;
      selecting = true;
      clk.tick(8);
    } else {
      // ---------------- DROP active position k
      const int c = __shfl(iam, k, NL);
      if (l == (c & (NL - 1))) {
#pragma unroll
        for (int r = 0; r < MR; ++r)
          if (r == (c >> 4)) act[r] = false;
      }
      const double un = __shfl(um, (l + 1) & (NL - 1), NL);
      const int in = __shfl(iam, (l + 1) & (NL - 1), NL);
      if (l >= k && l < q - 1) {
        um = un;
        iam = in;
      } else if (l == q - 1) {
        um = 0.0;
        iam = -1;
      }
      // full R (diagonal put back), delete column k (lane l owns column l)
      wave_lds_sync();
      if (l < q) R[l * RS + l] = Rdg[l];
      wave_lds_sync();
      double colv[NL];
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        if (i < qmax) {
          const double nxt = R[i * RS + l + 1];
          const double cur = R[i * RS + l];
          colv[i] = (l >= k && l < q - 1) ? nxt : ((l == q - 1) ? 0.0 : cur);
        }
      }
      wave_lds_sync();
#pragma unroll
      for (int i = 0; i < NL; ++i)
        if (i < qmax) R[i * RS + l] = colv[i];
      // Givens rotations restore the upper-triangular R
      for (int j = k; j < q - 1; ++j) {
        wave_lds_sync();
        const double a = R[j * RS + j], bb = R[(j + 1) * RS + j];
        const double ir = rsq(__builtin_fma(a, a, bb * bb));
        const double cj = a * ir, sj = bb * ir;
        const double rj = R[j * RS + l], rj1 = R[(j + 1) * RS + l];
        wave_lds_sync();
        if (l >= j && l < q - 1) {
          R[j * RS + l] = __builtin_fma(cj, rj, sj * rj1);
          R[(j + 1) * RS + l] = (l == j) ? 0.0 : __builtin_fma(-sj, rj, cj * rj1);
        }
        if (l == 0) {
          gcs[j] = cj;
          gsn[j] = sj;
        }
      }
      wave_lds_sync();
      R[(q - 1) * RS + l] = 0.0;
      unroll<NL - 1>([&](auto JJ) {
        constexpr int j = JJ;
        if (j + 1 < qmax && j >= k && j < q - 1) {
          const double cj = gcs[j], sj = gsn[j];
#pragma unroll
          for (int r = 0; r < MR; ++r) {
            const double e0 = E[r][j], e1 = E[r][j + 1];
            E[r][j] = __builtin_fma(cj, e0, sj * e1);
            E[r][j + 1] = __builtin_fma(-sj, e0, cj * e1);
          }
        }
      });
      --q;
      // back to the zero-diagonal form
      wave_lds_sync();
      const double dg = (l < q) ? R[l * RS + l] : 0.0;
      wave_lds_sync();
      if (l < q) {
        Rdg[l] = dg;
        R[l * RS + l] = 0.0;
      }
      invRd = (l < q) ? rcp(dg) : 0.0;
      clk.tick(9);
    }
    wave_lds_sync();
  }
  clk.tick(10);

  // ------------------------------------------------------------- outputs
  // x = -H^{-1} (f + A^T lam): g = f + sum_k u_k a_{iact_k} (the active rows of
  // A re-read, one coalesced 128-B row per active position), then L y = g,
  // L^T x = -y with L from LDS (column sweeps, one broadcast per step).
  const int qm = wave_max4(q);
  double gl = fl;
  {
    // all loads first (branch-free: inactive positions read row 0 and carry
    // a zero multiplier), then the sum
    const int ias = iam > 0 ? iam : 0;
    const int lc = l < n ? l : n - 1;
    double arow[NL];
    unroll<NL>([&](auto K) {
      constexpr int kk = K;
      if (kk < qm) arow[kk] = Aq[bci<kk>(ias) * n + lc];
    });
    unroll<NL>([&](auto K) {
      constexpr int kk = K;
      if (kk < qm) gl = __builtin_fma(bc<kk>(um), (l < n) ? arow[kk] : 0.0, gl);
    });
  }
  // forward: y_k = g_k / L_kk on lane k, then lanes l > k: g_l -= L[l][k] y_k
  unroll<NL>([&](auto K) {
    constexpr int kk = K;
    const double yk = bc<kk>(gl * Lp[lrow(kk) + kk]);
    gl = (l == kk) ? yk : ((l > kk) ? __builtin_fma(-Lp[lrow(l) + kk], yk, gl) : gl);
  });
  // backward: x_k = y_k / L_kk on lane k, then lanes l < k: y_l -= L[k][l] x_k
  unroll<NL>([&](auto K) {
    constexpr int kk = NL - 1 - K;
    const double xk = bc<kk>(gl * Lp[lrow(kk) + kk]);
    gl = (l == kk) ? xk : ((l < kk) ? __builtin_fma(-Lp[lrow(kk) + l], xk, gl) : gl);
  });
  const double xl = -gl;
  {
    // a non-finite x on any lane -> NUMERICAL for the QP
    const double bad = row_min((__builtin_fabs(xl) < kInf) ? 0.0 : -1.0);
    if (status == QPB_OK && bad < 0.0) status = QPB_NUMERICAL;
  }
#pragma unroll
  for (int r = 0; r < 2; ++r) lamb[l + NL * r] = 0.0;
  wave_lds_sync();
  if (l < q && iam >= 0) lamb[iam] = um;
  wave_lds_sync();
#pragma unroll
  for (int r = 0; r < MR; ++r) {
    const int row = l + NL * r;
    if (row < m) lamg[g * m + row] = lamb[row];
  }
  if (l < n) xg[g * n + l] = xl;
  const int sh = (threadIdx.x & 63) & ~(NL - 1);
  uint32_t w0 = 0;
#pragma unroll
  for (int r = 0; r < MR; ++r) {
    const unsigned long long bal = __ballot(act[r]);
    w0 |= (uint32_t)((bal >> sh) & 0xFFFFull) << (16 * r);
  }
  if (l == 0) {
    if (m > 0) actg[g] = w0;
    statg[g] = status;
    if (itg) itg[g] = it;
  }
  clk.tick(11);
  clk.flush(dbg);
}

}  // namespace qpb

// launcher used by qpb_api.hip
extern "C" hipError_t qpb_launch_gi(const qpb_desc *d, const double *H, const double *f, const double *A,
                                    const double *b, double *x, double *lam, uint32_t *active,
                                    int32_t *status, int32_t *iters, hipStream_t stream) {
  const long long blocks = (d->batch + qpb::QPB - 1) / qpb::QPB;
  const int max_iter = d->max_iter > 0 ? d->max_iter : 4 * (d->n + d->m) + 8;
  const double tol = d->feas_tol > 0 ? d->feas_tol : 1e-10;
#define QPB_GI_LAUNCH(MR, N16)                                                                                     \
  hipLaunchKernelGGL((qpb::gi_dense_kernel<MR, N16>), dim3((unsigned)blocks), dim3(64), 0, stream, H, f, A, b, x, \
                     lam, active, status, iters, d->n, d->m, (long long)d->batch, max_iter, tol, d->flags)
  const bool n16 = d->n == 16;
  if (d->m <= 16) {
    if (n16) QPB_GI_LAUNCH(1, true); else QPB_GI_LAUNCH(1, false);
  } else {
    if (n16) QPB_GI_LAUNCH(2, true); else QPB_GI_LAUNCH(2, false);
  }
#undef QPB_GI_LAUNCH
  return hipGetLastError();
}

// diagnostic: per-section wave cycles of the n=16, 16<m<=32 kernel (sections[12])
extern "C" hipError_t qpb_launch_gi_sections(const qpb_desc *d, const double *H, const double *f, const double *A,
                                             const double *b, double *x, double *lam, uint32_t *active,
                                             int32_t *status, int32_t *iters, unsigned long long *sections,
                                             hipStream_t stream) {
  const long long blocks = (d->batch + qpb::QPB - 1) / qpb::QPB;
  const int max_iter = d->max_iter > 0 ? d->max_iter : 4 * (d->n + d->m) + 8;
  const double tol = d->feas_tol > 0 ? d->feas_tol : 1e-10;
  if (d->n != 16 || d->m <= 16) return hipErrorInvalidValue;
  hipLaunchKernelGGL((qpb::gi_dense_kernel<2, true, true>), dim3((unsigned)blocks), dim3(64), 0, stream, H, f, A, b,
                     x, lam, active, status, iters, d->n, d->m, (long long)d->batch, max_iter, tol, d->flags, sections);
  return hipGetLastError();
}
