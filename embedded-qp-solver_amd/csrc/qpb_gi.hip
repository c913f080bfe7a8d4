// qpb_gi.hip -- batched dense active-set QP kernel for gfx950 (n <= 16).
//
//   min 1/2 x^T H x + f^T x   s.t.   A x <= b        (fp64, one QP per 16 lanes)
//
// Replaces, batched, the reference's hot path: the dense kernels of
// matrix/matrix_ops/matrix_ops.c (matrix_mult GEMV :235-271, LU/inverse
// :487-630, vector ops :158-411, norm :632-656) driving the solver iterations
// of qp_solvers/qp_solvers.c; the constrained iteration north_star asks for
// (absent from the reference) is the dual active-set method of
// Goldfarb & Idnani (Math. Prog. 27, 1983), which needs no feasible start:
//
//   setup   H = L L^T (Cholesky, row l of H in lane l's registers, right-
//           looking, column k of L broadcast by DPP row_newbcast);
//           J = L^{-T}, D = A J, y = L^{-1} f by forward substitution;
//           x = -J y (unconstrained minimiser = test/qp_ref.py:35's answer),
//           slack s = b - A x = b + D y.
//   iterate pick the most violated row p (normalised slack, exact row argmin);
//           d = -D[p,:] (= J^T n+ in G-I's notation, n+ = -a_p), primal step
//           z = J2 d2 (columns >= q), dual step r = R^{-1} d1 (lane-parallel
//           back substitution), partial step t1 (ratio test over the active
//           multipliers), full step t2 = -s_p / |d2|^2;
//           full step  -> ADD p: one Householder reflection on columns q..15
//                         of [D; J] (every lane updates its own rows), new
//                         column of R;
//           partial    -> DROP k: delete column k of R, Givens rotations
//                         restore triangularity (also applied to [D; J]).
//
// Data layout per QP (lane l = 0..15 of the QP's row):
//   registers  E[r][0..15] = row l + 16 r of D (r < MR),  E[MR] = row l of J,
//              slack s[r], 1/||a_row||, active flag, x_l, multiplier/row of
//              active position l
//   LDS        R (16 x 18 doubles, padded rows: conflict-free b128 row reads),
//              exchange row for d, Givens parameters, lambda scatter buffer
// No global memory besides the inputs (read once) and the outputs.
#include "qpb_common.h"
#include "qpb.h"

namespace qpb {

constexpr int NL = 16;     // lanes per QP
constexpr int QPB = 16;    // QPs per 256-thread workgroup
constexpr int RS = 18;     // R row stride (doubles)
constexpr int OFF_XCH = 16 * RS;          // 288: d (16) + s_p
constexpr int OFF_CS = OFF_XCH + 18;      // 306: Givens cosines (16)
constexpr int OFF_SN = OFF_CS + 16;       // 322: Givens sines (16)
constexpr int OFF_LAM = OFF_SN + 16;      // 338: lambda scatter (64)
constexpr int SLOT = OFF_LAM + 64;        // 402 doubles per QP
constexpr double kDepTol = 1e-24;         // |d2|^2 <= kDepTol |d|^2  <=>  z = 0

template <int MR, bool N16>
__global__ __launch_bounds__(256, 2) void gi_dense_kernel(
    const double *__restrict__ Hg, const double *__restrict__ fg, const double *__restrict__ Ag,
    const double *__restrict__ bg, double *__restrict__ xg, double *__restrict__ lamg,
    uint32_t *__restrict__ actg, int32_t *__restrict__ statg, int32_t *__restrict__ itg, int n, int m,
    long long batch, int max_iter, double feas_tol) {
  __shared__ double lds[QPB * SLOT];
  const int l = threadIdx.x & (NL - 1);
  const int slot = threadIdx.x >> 4;
  const long long g = (long long)blockIdx.x * QPB + slot;
  if (g >= batch) return;  // whole 16-lane rows leave together

  double *R = lds + slot * SLOT;
  double *xch = R + OFF_XCH;
  double *gcs = R + OFF_CS;
  double *gsn = R + OFF_SN;
  double *lamb = R + OFF_LAM;

  // ------------------------------------------------------------------ load
  const double *Hq = Hg + g * (long long)n * n;
  const double *Aq = Ag + g * (long long)m * n;
  double Lr[NL];  // row l of H, becomes row l of L
  double E[MR + 1][NL];
  double s[MR], invn[MR], bl[MR];
  bool act[MR];
  bool infeasible_row = false;
  if (N16) {  // n == 16: unconditional, 16-byte loads of whole rows
#pragma unroll
    for (int j = 0; j < NL; j += 2) {
      const double2 h = *reinterpret_cast<const double2 *>(&Hq[l * NL + j]);
      Lr[j] = h.x;
      Lr[j + 1] = h.y;
    }
  } else {  // padded: clamped addresses (no per-element branches), identity outside n
    const int lc = l < n ? l : n - 1;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const double h = Hq[lc * n + (j < n ? j : n - 1)];
      Lr[j] = (l < n && j < n) ? h : (l == j ? 1.0 : 0.0);
    }
  }
#pragma unroll
  for (int r = 0; r < MR; ++r) {
    const int row = l + NL * r;
    const bool ok = row < m;
    const int rc = ok ? row : 0;
    if (N16) {
#pragma unroll
      for (int j = 0; j < NL; j += 2) {
        const double2 a = m > 0 ? *reinterpret_cast<const double2 *>(&Aq[rc * NL + j]) : make_double2(0.0, 0.0);
        E[r][j] = ok ? a.x : 0.0;
        E[r][j + 1] = ok ? a.y : 0.0;
      }
    } else {
#pragma unroll
      for (int j = 0; j < NL; ++j) {
        const double a = m > 0 ? Aq[rc * n + (j < n ? j : n - 1)] : 0.0;
        E[r][j] = (ok && j < n) ? a : 0.0;
      }
    }
    double nrm2 = 0.0;
#pragma unroll
    for (int j = 0; j < NL; ++j) nrm2 = __builtin_fma(E[r][j], E[r][j], nrm2);
    const double bv = m > 0 ? bg[g * m + rc] : 0.0;
    bl[r] = ok ? bv : 0.0;
    invn[r] = nrm2 > 0.0 ? 1.0 / __builtin_sqrt(nrm2) : 0.0;
    // a zero row is the constant constraint 0 <= b
    infeasible_row = infeasible_row || (ok && nrm2 == 0.0 && bl[r] < -feas_tol * (1.0 + __builtin_fabs(bl[r])));
    act[r] = false;
  }
#pragma unroll
  for (int j = 0; j < NL; ++j) E[MR][j] = (j == l) ? 1.0 : 0.0;  // e_l -> row l of J
  const double fv = fg[g * n + (l < n ? l : n - 1)];
  const double fl = (l < n) ? fv : 0.0;
  double yf[NL];
  unroll<NL>([&](auto J) { yf[J] = bc<J>(fl); });  // f replicated on every lane

  // ---- Cholesky H = L L^T (left-looking: step k broadcasts row k of L from
  // lane k by DPP row_newbcast and finishes column k on every lane)
  bool spd = true;
  unroll<NL>([&](auto K) {
    constexpr int k = K;
    __builtin_amdgcn_sched_barrier(0);
    double a = Lr[k];
    unroll<k>([&](auto J) { a = __builtin_fma(-Lr[J], bc<k>(Lr[J]), a); });
    const double akk = bc<k>(a);
    spd = spd && (akk > 0.0);
    const double ik = 1.0 / __builtin_sqrt(akk);
    // row l keeps L[l][0..l]; the diagonal is stored as its reciprocal
    Lr[k] = (l > k) ? a * ik : ((l == k) ? ik : 0.0);
  });
  // L -> LDS (row l at R + l*RS; the R area is free until the active-set loop)
#pragma unroll
  for (int j = 0; j < NL; j += 2) *reinterpret_cast<double2 *>(&R[l * RS + j]) = make_double2(Lr[j], Lr[j + 1]);
  wave_lds_sync();

  // ---- forward substitutions with row k of L read from LDS (same address on
  // the 16 lanes of a QP: broadcast reads): D = A L^{-T} (rows l, l+16),
  // J = L^{-T} (row l), y = L^{-1} f
  unroll<NL>([&](auto K) {
    constexpr int k = K;
    __builtin_amdgcn_sched_barrier(0);
    double Lk[k + 1];
    unroll<k + 1>([&](auto J) { Lk[J] = R[k * RS + J]; });
    const double ik = Lk[k];
#pragma unroll
    for (int r = 0; r <= MR; ++r) {
      double e = E[r][k];
      unroll<k>([&](auto J) { e = __builtin_fma(-Lk[J], E[r][J], e); });
      E[r][k] = e * ik;
    }
    double y = yf[k];
    unroll<k>([&](auto J) { y = __builtin_fma(-Lk[J], yf[J], y); });
    yf[k] = y * ik;
  });
  wave_lds_sync();

  double xl = 0.0;
#pragma unroll
  for (int j = 0; j < NL; ++j) xl = __builtin_fma(-E[MR][j], yf[j], xl);
#pragma unroll
  for (int r = 0; r < MR; ++r) {
    double a = bl[r];
#pragma unroll
    for (int j = 0; j < NL; ++j) a = __builtin_fma(E[r][j], yf[j], a);
    s[r] = a;
  }

  // ------------------------------------------------------ active-set loop
#pragma unroll
  for (int j = 0; j < RS; j += 2) *reinterpret_cast<double2 *>(&R[l * RS + j]) = make_double2(0.0, 0.0);
  int q = 0;              // active-set size
  double um = 0.0;        // multiplier of active position l
  int iam = -1;           // constraint index at active position l
  double invRd = 0.0;     // 1 / R[l][l]
  int status;
  bool done;
  {
    // any lane seeing an infeasible zero row marks the whole QP
    double flag = infeasible_row ? 1.0 : 0.0;
    int dummy = 0;
    double negflag = -flag;
    row_argmin(negflag, dummy);
    const bool inf0 = negflag < 0.0;
    status = !spd ? QPB_NOT_SPD : (inf0 ? QPB_INFEASIBLE : QPB_MAX_ITER);
    done = !spd || inf0;
  }
  bool selecting = true;
  int p = 0;
  double up = 0.0;  // multiplier of the constraint being added
  int it = 0;
  wave_lds_sync();

  while (!done && it < max_iter) {
    ++it;
    if (selecting) {
      double bv = kInf;
      int bi = 1 << 30;
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        const double v = s[r] * invn[r];
        const bool viol = !act[r] && invn[r] > 0.0 &&
                          v < -feas_tol * (1.0 + __builtin_fabs(bl[r]) * invn[r]);
        const double key = viol ? v : kInf;
        const int idx = l + NL * r;
        const bool take = key < bv;
        bv = take ? key : bv;
        bi = take ? idx : bi;
      }
      row_argmin(bv, bi);
      if (!(bv < kInf)) {
        status = QPB_OK;
        done = true;
        break;
      }
      p = bi;
      up = 0.0;
      selecting = false;
    }

    // ---- d = -D[p,:] and s_p to every lane through the exchange row
    const int owner = p & (NL - 1), prow = p >> 4;
    if (l == owner) {
#pragma unroll
      for (int r = 0; r < MR; ++r)
        if (r == prow) {
#pragma unroll
          for (int j = 0; j < NL; j += 2) *reinterpret_cast<double2 *>(&xch[j]) = make_double2(E[r][j], E[r][j + 1]);
          xch[NL] = s[r];
        }
    }
    wave_lds_sync();
    double d[NL];
#pragma unroll
    for (int j = 0; j < NL; j += 2) {
      const double2 v = *reinterpret_cast<const double2 *>(&xch[j]);
      d[j] = -v.x;
      d[j + 1] = -v.y;
    }
    const double sp = xch[NL];
    const double dl = -xch[l];
    const double dq = (q < NL) ? -xch[q] : 0.0;
    double d2[NL];
    double nd2 = 0.0, dd = 0.0;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      d2[j] = (j >= q) ? d[j] : 0.0;
      nd2 = __builtin_fma(d2[j], d2[j], nd2);
      dd = __builtin_fma(d[j], d[j], dd);
    }

    // ---- r = R^{-1} d1 (lane-parallel back substitution over the active positions)
    double Rrow[NL];
#pragma unroll
    for (int j = 0; j < NL; j += 2) {
      const double2 v = *reinterpret_cast<const double2 *>(&R[l * RS + j]);
      Rrow[j] = v.x;
      Rrow[j + 1] = v.y;
    }
    double acc = (l < q) ? dl : 0.0;
    unroll<NL>([&](auto JJ) {
      constexpr int j = NL - 1 - JJ;
      double rj = bc<j>(acc * invRd);
      rj = (j < q) ? rj : 0.0;
      acc = (l < j) ? __builtin_fma(-Rrow[j], rj, acc) : acc;
    });
    const double rm = acc * invRd;  // r_l (0 for l >= q)

    // ---- step lengths
    double t1 = (l < q && rm > 0.0) ? um / rm : kInf;
    int k = l;
    row_argmin(t1, k);
    const double t2 = (nd2 > kDepTol * dd) ? -sp / nd2 : kInf;
    const double t = t1 < t2 ? t1 : t2;
    if (!(t < kInf)) {
      status = QPB_INFEASIBLE;
      done = true;
      break;
    }
    if (t2 < kInf) {  // primal step x += t z, s -= t A z  (A z = D[:, q:] d2)
      double z = 0.0;
#pragma unroll
      for (int j = 0; j < NL; ++j) z = __builtin_fma(E[MR][j], d2[j], z);
      xl = __builtin_fma(t, z, xl);
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        double az = 0.0;
#pragma unroll
        for (int j = 0; j < NL; ++j) az = __builtin_fma(E[r][j], d2[j], az);
        s[r] = __builtin_fma(-t, az, s[r]);
      }
    }
    um = __builtin_fma(-t, rm, um);
    up += t;

    if (t2 <= t1) {
      // ---------------- ADD p: Householder on columns q.. of [D; J]
      const double nrm = __builtin_sqrt(nd2);
      const double alpha = dq >= 0.0 ? -nrm : nrm;
      const double beta = 1.0 / (nd2 - alpha * dq);
      double v[NL];
#pragma unroll
      for (int j = 0; j < NL; ++j) v[j] = (j == q) ? d2[j] - alpha : d2[j];
#pragma unroll
      for (int r = 0; r <= MR; ++r) {
        double w = 0.0;
#pragma unroll
        for (int j = 0; j < NL; ++j) w = __builtin_fma(E[r][j], v[j], w);
        w *= beta;
#pragma unroll
        for (int j = 0; j < NL; ++j) E[r][j] = __builtin_fma(-w, v[j], E[r][j]);
      }
      // new column q of R: d1 above the diagonal, alpha on it
      R[l * RS + q] = (l < q) ? dl : ((l == q) ? alpha : 0.0);
      if (l == q) {
        invRd = 1.0 / alpha;
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
      // delete column k of R (lane l owns column l)
      wave_lds_sync();
      double colv[NL];
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        const double nxt = R[i * RS + l + 1];
        const double cur = R[i * RS + l];
        colv[i] = (l >= k && l < q - 1) ? nxt : ((l == q - 1) ? 0.0 : cur);
      }
      wave_lds_sync();
#pragma unroll
      for (int i = 0; i < NL; ++i) R[i * RS + l] = colv[i];
      // Givens rotations restore the upper-triangular R
      for (int j = k; j < q - 1; ++j) {
        wave_lds_sync();
        const double a = R[j * RS + j], bb = R[(j + 1) * RS + j];
        const double rho = __builtin_sqrt(__builtin_fma(a, a, bb * bb));
        const double cj = a / rho, sj = bb / rho;
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
        if (j >= k && j < q - 1) {
          const double cj = gcs[j], sj = gsn[j];
#pragma unroll
          for (int r = 0; r <= MR; ++r) {
            const double e0 = E[r][j], e1 = E[r][j + 1];
            E[r][j] = __builtin_fma(cj, e0, sj * e1);
            E[r][j + 1] = __builtin_fma(-sj, e0, cj * e1);
          }
        }
      });
      wave_lds_sync();
      --q;
      invRd = (l < q) ? 1.0 / R[l * RS + l] : 0.0;
    }
    wave_lds_sync();
  }

  // ------------------------------------------------------------- outputs
  if (status == QPB_OK && !(__builtin_fabs(xl) < kInf)) status = QPB_NUMERICAL;
  // a NaN on any lane -> NUMERICAL for the QP
  {
    double bad = (__builtin_fabs(xl) < kInf) ? 0.0 : -1.0;
    int dummy = 0;
    row_argmin(bad, dummy);
    if (status == QPB_OK && bad < 0.0) status = QPB_NUMERICAL;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) lamb[l + NL * r] = 0.0;
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
  uint32_t w0 = 0, w1 = 0;
#pragma unroll
  for (int r = 0; r < MR; ++r) {
    const unsigned long long bal = __ballot(act[r]);
    const uint32_t bits = (uint32_t)((bal >> sh) & 0xFFFFull);
    if (r == 0) w0 |= bits;
    if (r == 1) w0 |= bits << 16;
    if (r == 2) w1 |= bits;
    if (r == 3) w1 |= bits << 16;
  }
  const int words = (m + 31) >> 5;
  if (l == 0) {
    if (words > 0) actg[g * words] = w0;
    if (words > 1) actg[g * words + 1] = w1;
    statg[g] = status;
    if (itg) itg[g] = it;
  }
}

}  // namespace qpb

// launcher used by qpb_api.hip
extern "C" hipError_t qpb_launch_gi(const qpb_desc *d, const double *H, const double *f, const double *A,
                                    const double *b, double *x, double *lam, uint32_t *active,
                                    int32_t *status, int32_t *iters, hipStream_t stream) {
  const long long blocks = (d->batch + qpb::QPB - 1) / qpb::QPB;
  const int max_iter = d->max_iter > 0 ? d->max_iter : 4 * (d->n + d->m) + 8;
  const double tol = d->feas_tol > 0 ? d->feas_tol : 1e-10;
#define QPB_GI_LAUNCH(MR, N16)                                                                              \
  hipLaunchKernelGGL((qpb::gi_dense_kernel<MR, N16>), dim3((unsigned)blocks), dim3(256), 0, stream, H, f, A, b, x, \
                     lam, active, status, iters, d->n, d->m, (long long)d->batch, max_iter, tol)
  const bool n16 = d->n == 16;
  if (d->m <= 16) {
    if (n16) QPB_GI_LAUNCH(1, true); else QPB_GI_LAUNCH(1, false);
  } else {
    if (n16) QPB_GI_LAUNCH(2, true); else QPB_GI_LAUNCH(2, false);
  }
#undef QPB_GI_LAUNCH
  return hipGetLastError();
}
