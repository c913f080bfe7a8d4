// qpb_gi_box.hip -- batched box-constrained QP kernel for gfx950 (n <= 16).
//
//   min 1/2 x^T H x + f^T x   s.t.   lb <= x <= ub        (fp64, one QP per 16 lanes)
//
// The constraint class of the reference's only constrained solver, admm()
// (qp_solvers/qp_solvers.c:146-319, box bounds config.h:29-30), solved exactly:
// the dual active-set method of qpb_gi.hip (Goldfarb & Idnani) on the implicit
// A = [I; -I], b = [ub; -lb] -- SURVEY.md §8b's BOX constraint kind and §8d's
// box fast path (2,824 algorithmic bytes per QP at n = 16 instead of 6,920).
// With A implicit the kernel is qpb_gi.hip with three simplifications:
//   D = A L^{-T} = [L^{-T}; -L^{-T}]: lane l keeps ONE row, row l of L^{-T}
//     (the setup sweep starts it from e_l); the lower bound's row is its
//     negative, so the slack step's product and the Householder reflection
//     touch 16 values per lane instead of 32, and every row has norm 1.
//   the exchange row: the owner lane writes its only row (no row select);
//     readers fold in the sign of the selected bound (the reflection is
//     sign-free: v v^T with v = sgn v').
//   x = -H^{-1} (f + lambda_u - lambda_l): no rows of A to read back.
// Constraint numbering inside the kernel: row l (upper bound of x_l) and row
// 16 + l (lower bound); outputs use qpb_solve's m = 2n numbering (upper bounds
// 0..n-1, lower bounds n..2n-1), i.e. A = [I; -I] row order.  Infinite bounds
// (or a NULL lb / ub) are absent constraints: their slack is +inf.
#include "qpb_common.h"
#include "qpb.h"

namespace qpb {
namespace box {

constexpr int NL = 16;  // lanes per QP
constexpr int QPB = 4;  // QPs per wavefront
constexpr int RS = 18;  // row stride of the H transpose (conflict-free b128 rows)
__host__ __device__ constexpr int lrow(int i) { return i * (i + 1) / 2; }
constexpr int L_SIZE = lrow(NL);  // 136
// per QP: L packed (136) | R column-major 16 x 16 with zero diagonal | exchange 32
constexpr int OFF_L = 0;
constexpr int OFF_R = L_SIZE;
constexpr int OFF_XCH = OFF_R + NL * NL;
constexpr int SLOT = OFF_XCH + 2;  // 394 doubles: s_p (the exchange row is R's column 0, as qpb_gi.hip)
constexpr double kDepTol = 1e-24;
static_assert(NL * RS <= SLOT, "the H transpose is staged over the whole slot");
// 12 one-wave workgroups per CU need <= 12,800 B of LDS each (qpb_gi.hip,
// tools/probe/occupancy_probe.hip); the round-4 slot (424 doubles = 13,568 B)
// ran 11
static_assert(4 * SLOT * 8 <= 12800, "12 waves per CU by LDS");

template <int N, class FX, class FY>
__device__ __forceinline__ double dot2(FX &&x, FY &&y) {
  double a0 = 0.0, a1 = 0.0;
  unroll<N>([&](auto J) {
    constexpr int j = J;
    if constexpr (j % 2 == 0) a0 = __builtin_fma(x(j), y(j), a0);
    else a1 = __builtin_fma(x(j), y(j), a1);
  });
  return a0 + a1;
}

__device__ __forceinline__ void lds_row16(const double *src, double (&dst)[NL]) {
#pragma unroll
  for (int j = 0; j < NL; j += 2) {
    const double2 v = *reinterpret_cast<const double2 *>(&src[j]);
    dst[j] = v.x;
    dst[j + 1] = v.y;
  }
}

// N16: n == 16 (coalesced H loads through an LDS transpose); otherwise the
// rows are padded with the identity and the padded variables get no bounds
template <bool N16>
__global__ __launch_bounds__(64, 3) void gi_box_kernel(const double *__restrict__ Hg, const double *__restrict__ fg,
                                                       const double *__restrict__ lbg, const double *__restrict__ ubg,
                                                       double *__restrict__ xg, double *__restrict__ lamg,
                                                       uint32_t *__restrict__ actg, int32_t *__restrict__ statg,
                                                       int32_t *__restrict__ itg, int n, long long batch,
                                                       int max_iter, double feas_tol) {
  __shared__ double lds[QPB * SLOT];
  const int l = threadIdx.x & (NL - 1);
  const int slot = threadIdx.x >> 4;
  // rows past the end of the batch replay its last QP and store nothing (as
  // in qpb_gi.hip: every lane stays live for the cross-row readlanes)
  const long long graw = (long long)blockIdx.x * QPB + slot;
  const bool live = graw < batch;
  const long long g = live ? graw : batch - 1;
  if constexpr (N16) n = NL;
  double *base = lds + (((slot & 1) << 1) | (slot >> 1)) * SLOT;  // slots 0, 2, 1, 3 (bank spread)
  double *Lp = base + OFF_L;
  double *R = base + OFF_R;
  double *xch = R;  // the exchange row in R's column 0 (never read by the back substitution)
  double *xsp = base + OFF_XCH;

  // ------------------------------------------------------------------ load
  const bool var = N16 || l < n;  // lane l carries variable l
  const int lc = var ? l : n - 1;
  const double *Hq = Hg + g * (long long)n * n;
  const double fv = fg[g * n + lc];
  const double ubv = ubg ? ubg[g * n + lc] : kInf;
  const double lbv = lbg ? lbg[g * n + lc] : -kInf;
  double Lr[NL];  // row l of H, becomes row l of L
  double E[NL];   // row l of D = L^{-T}, from e_l
  if constexpr (N16) {
    // one instruction reads two whole rows of each of the wave's 4 QPs; the
    // rows reach their owner lanes through a transpose in this QP's LDS slot
    // (L and R are written after the factorisation)
    const int hr = l >> 3, hc = 2 * (l & 7);
    double2 hv[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) hv[t] = *reinterpret_cast<const double2 *>(&Hq[(2 * t + hr) * NL + hc]);
    asm volatile("" ::"v"(fv), "v"(ubv), "v"(lbv));
#pragma unroll
    for (int t = 0; t < 8; ++t) asm volatile("" ::"v"(hv[t].x), "v"(hv[t].y));
    wave_lds_sync();
#pragma unroll
    for (int t = 0; t < 8; ++t) *reinterpret_cast<double2 *>(&base[(2 * t + hr) * RS + hc]) = hv[t];
    wave_lds_sync();
    lds_row16(&base[l * RS], Lr);
    wave_lds_sync();
  } else {
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const double h = Hq[lc * n + (j < n ? j : n - 1)];
      Lr[j] = (l < n && j < n) ? h : (l == j ? 1.0 : 0.0);
    }
  }
#pragma unroll
  for (int j = 0; j < NL; ++j) E[j] = l == j ? 1.0 : 0.0;
  // b of the two rows: ub (x_l <= ub_l) and -lb (-x_l <= -lb_l)
  const double bu = var ? ubv : kInf, bl = var ? -lbv : kInf;
  // violation thresholds of the (unit-norm) rows; -inf for an absent bound
  const double thu = -feas_tol * (1.0 + __builtin_fabs(bu)), thl = -feas_tol * (1.0 + __builtin_fabs(bl));
  const double fl = var ? fv : 0.0;

  // ---- H = L L^T, D = L^{-T} (row l from e_l), y = L^{-1} f in one
  // right-looking sweep (qpb_gi.hip, one D row per lane); e = D y accumulates
  // alongside (y_k is final at step k)
  bool spd = true;
  double ya = fl, ey = 0.0;
  unroll<NL>([&](auto K) {
    constexpr int k = K;
    __builtin_amdgcn_sched_barrier(0);
    const double akk = bc<k>(Lr[k]);
    spd = spd && (akk > 0.0);
    const double ik = rsq1(akk);
    const double ik2 = ik * ik;
    const double nc = -(Lr[k] * ik2);
    const double e = E[k];
    const double ne2 = -(e * ik2);
    E[k] = e * ik;
    unroll<NL - 1 - k>([&](auto J) {
      constexpr int j = k + 1 + J;
      fmac_bc<k>(E[j], Lr[j], ne2);
      fmac_bc<k>(Lr[j], Lr[j], nc);
    });
    Lr[k] *= ik;
    const double c = -nc;
    const double fk = bc<k>(ya);
    ya = __builtin_fma(-c, fk, ya);
    ey = __builtin_fma(E[k], fk * ik, ey);
  });
  __builtin_amdgcn_sched_barrier(0);
  // L -> LDS, packed rows, for the final solves (descending j: a lane's dead
  // entries past its diagonal land first and are overwritten by their owners)
  unroll<NL>([&](auto J) {
    constexpr int j = NL - 1 - J;
    Lp[lrow(l) + j] = Lr[j];
    wave_lds_sync();
  });
  // slacks of the unconstrained minimiser x0 = -L^{-T} y: b + D y per row
  double su = bu + ey, sl = bl - ey;
  // |D[l, q:]|^2, the free part of both of the lane's rows (scale of the
  // selection key, as qpb_gi.hip)
  float fn2 = (float)dot2<NL>([&](int j) { return E[j]; }, [&](int j) { return E[j]; });

  // ------------------------------------------------------ active-set loop
  // zeroed in pairs at lane-rotated positions (the same position in every
  // lane's column would be an 8-way bank conflict per store)
#pragma unroll
  for (int j = 0; j < NL; j += 2)
    *reinterpret_cast<double2 *>(&R[l * NL + ((j + 2 * l) & (NL - 1))]) = make_double2(0.0, 0.0);
  int q = 0;
  double um = 0.0;  // multiplier of active position l
  int iam = -1;     // constraint (0..15 upper, 16..31 lower) at active position l
  double rdg = 0.0, invRd = 0.0;
  bool actu = false, actl = false;
  int status = spd ? QPB_MAX_ITER : QPB_NOT_SPD;
  bool done = !spd;
  bool selecting = true;
  int p = 0;
  double up = 0.0;
  int it = 0;
  wave_lds_sync();
  while (!done && it < max_iter) {
    ++it;
    if (selecting) {
      // violated bounds (rows of unit norm) ranked by dual steepest edge,
      // -s / |D[l, q:]| as in qpb_gi.hip (the same choices as the dense path
      // on A = [I; -I]): fp32 keys with the row in the low 5 bits, DPP-fused max
      // (fn2 >= 0, clamped where it shrinks; the 2^-100 floor keeps a violated
      // bound's key nonzero -- 0 is "none violated" -- when the ratio underflows)
      const float rf = __builtin_amdgcn_rsqf(fn2);
      const uint32_t ku = (__float_as_uint(__builtin_fmaf((float)(-su), rf, 0x1p-100f)) & ~31u) | (uint32_t)l;
      const uint32_t kl = (__float_as_uint(__builtin_fmaf((float)(-sl), rf, 0x1p-100f)) & ~31u) | (uint32_t)(l + NL);
      uint32_t key = (!actu && su < thu) ? ku : 0u;
      key = (!actl && sl < thl && kl > key) ? kl : key;
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
    const int qmax = __builtin_elementwise_min(wave_max4(q), NL);
    const int owner = p & (NL - 1);
    const double sgn = p < NL ? 1.0 : -1.0;  // D[p,:] = sgn * (row `owner` of L^{-T})
    if (l == owner) {
#pragma unroll
      for (int j = 0; j < NL; j += 2) *reinterpret_cast<double2 *>(&xch[j]) = make_double2(E[j], E[j + 1]);
      *xsp = p < NL ? su : sl;
    }
    wave_lds_sync();
    const double wl = xch[l];
    const double wq = xch[q & (NL - 1)];  // q == 16: only used by an ADD, impossible then
    const double sp = *xsp;
    // the selected row with its active columns zeroed, entry j at lane j
    // (d2 = sgn * w2): the products below take it by DPP broadcast
    const double w2 = l >= q ? wl : 0.0;
    dpp_ready(w2);
    const double Dpl = sgn * wl, Dpq = sgn * wq;
    const double dl = -Dpl;
    const double nd2 = row_sum(l >= q ? wl * wl : 0.0);  // |d2|^2
    const double dd = row_sum(wl * wl);                  // |D[p,:]|^2

    // ---- r = R^{-1} d1 (lane-parallel back substitution, DPP-fused FMAs)
    double rm = 0.0;
    if (qmax > 0) {
      const double ninv = -invRd;
      double nacc = (l < q) ? Dpl : 0.0;
      unroll<NL>([&](auto JJ) {
        constexpr int j = NL - 1 - JJ;
        if (j > 0 && j < qmax) fmac_bc_nop<j>(nacc, nacc * ninv, R[j * NL + l]);  // column 0: no entry above the diagonal
      });
      rm = nacc * ninv;
    }
    // ---- step lengths: exact ratio minimum, then the lowest position reaching it
    double t1 = kBig;
    int k = 0;
    if (qmax > 0) {
      const double ratio = um * rcp1(rm);
      const bool cand = l < q && rm > 0.0;
      t1 = row_min(cand ? ratio : kBig);
      k = (int)row_min_u32(cand && ratio == t1 ? (uint32_t)l : 31u) & (NL - 1);
    }
    const double ir = rsq1(nd2);
    const double t2 = (nd2 > kDepTol * dd) ? -sp * (ir * ir) : kBig;
    const double t = t1 < t2 ? t1 : t2;
    if (!(t < kBig)) {
      status = QPB_INFEASIBLE;
      done = true;
      break;
    }
    double u = 0.0;  // D[l,:] . d2
    if (t2 < kBig) {  // slacks s -= t D[:, q:] d2: the upper row's product, negated for the lower
      double a0 = 0.0, a1 = 0.0;
      unroll<NL>([&](auto J) {
        constexpr int j = J;
        fmac_bc<j>(j % 2 ? a1 : a0, w2, E[j]);
      });
      u = sgn * (a0 + a1);
      su = __builtin_fma(t, u, su);
      sl = __builtin_fma(-t, u, sl);
    }
    pin(su);
    pin(sl);
    um = __builtin_fma(-t, rm, um);
    up += t;

    if (t2 <= t1) {
      // ---------------- ADD p: Householder on columns q.. of D.  v = d2 +
      // alpha e_q = sgn (w2 + sgn alpha e_q), and the reflection I - beta v v^T
      // only sees v v^T, so the unsigned v' = w2 + sgn alpha e_q is formed in LDS
      const double nrm = nd2 * ir;
      const double alpha = Dpq <= 0.0 ? -nrm : nrm;
      const double beta = ir * rcp1(nrm + __builtin_fabs(Dpq));
      const double ia = Dpq <= 0.0 ? -ir : ir;  // 1 / alpha
      // the reflection maps e_q to -d2 / alpha: column q of the new D is
      // -u / alpha, and it leaves the free part of the row
      const float cq = (float)(u * ia);
      fn2 = __builtin_fmaxf(__builtin_fmaf(-cq, cq, fn2), 0.0f);
      const double v = w2 + (l == q ? sgn * alpha : 0.0);
      dpp_ready(v);
      double a0 = 0.0, a1 = 0.0;
      unroll<NL>([&](auto J) {
        constexpr int j = J;
        fmac_bc<j>(j % 2 ? a1 : a0, v, E[j]);
      });
      const double nw = -beta * (a0 + a1);
      unroll<NL>([&](auto J) {
        constexpr int j = J;
        fmac_bc<j>(E[j], v, nw);
      });
      R[q * NL + l] = (l < q) ? dl : 0.0;
      if (l == q) {
        rdg = alpha;
        invRd = ia;
        iam = p;
        um = up;
      }
      if (l == owner) {
        actu = actu || p < NL;
        actl = actl || p >= NL;
      }
      ++q;
      selecting = true;
    } else {
      // ---------------- DROP active position k (as qpb_gi.hip)
      const int c = __shfl(iam, k, NL);
      if (l == (c & (NL - 1))) {
        actu = actu && c >= NL;
        actl = actl && c < NL;
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
      if (l < q) R[l * NL + l] = rdg;
      // lane l copies column l+1 whole (one pass: in-order DS, every read
      // precedes every write), pairs at lane-rotated positions (conflict-free)
      {
        double2 col[NL / 2];
#pragma unroll
        for (int t = 0; t < NL / 2; ++t)
          col[t] = *reinterpret_cast<const double2 *>(&R[((l + 1) & (NL - 1)) * NL + ((2 * t + 2 * l) & (NL - 1))]);
        wave_lds_sync();
        if (l >= k && l < q - 1) {
#pragma unroll
          for (int t = 0; t < NL / 2; ++t) *reinterpret_cast<double2 *>(&R[l * NL + ((2 * t + 2 * l) & (NL - 1))]) = col[t];
        } else if (l == q - 1) {
#pragma unroll
          for (int t = 0; t < NL / 2; ++t)
            *reinterpret_cast<double2 *>(&R[l * NL + ((2 * t + 2 * l) & (NL - 1))]) = make_double2(0.0, 0.0);
        }
      }
      // Givens rotations restore the upper-triangular R (lane j keeps rotation
      // j's parameters for the D update, which reads them by DPP) ...
      double gc = 0.0, gs = 0.0;
      for (int j = k; j < q - 1; ++j) {
        wave_lds_sync();
        const double a = R[j * NL + j], bb = R[j * NL + j + 1];
        const double irr = rsq1(__builtin_fma(a, a, bb * bb));
        const double cj = a * irr, sj = bb * irr;
        const double rj = R[l * NL + j], rj1 = R[l * NL + j + 1];
        wave_lds_sync();
        if (l >= j && l < q - 1) {
          R[l * NL + j] = __builtin_fma(cj, rj, sj * rj1);
          R[l * NL + j + 1] = (l == j) ? 0.0 : __builtin_fma(-sj, rj, cj * rj1);
        }
        if (l == j) {
          gc = cj;
          gs = sj;
        }
      }
      wave_lds_sync();
      R[l * NL + q - 1] = 0.0;
      // ... and the same rotations on D's columns
      unroll<NL - 1>([&](auto JJ) {
        constexpr int j = JJ;
        if (j + 1 < qmax && j >= k && j < q - 1) {
          const double cj = bc<j>(gc), sj = bc<j>(gs);
          const double e0 = E[j], e1 = E[j + 1];
          E[j] = __builtin_fma(cj, e0, sj * e1);
          E[j + 1] = __builtin_fma(-sj, e0, cj * e1);
        }
      });
      --q;
      // column q (after the rotations) joins the free part: recompute
      {
        float a0 = 0.0f, a1 = 0.0f;
        unroll<NL>([&](auto J) {
          constexpr int j = J;
          const float e = (float)E[j];
          if constexpr (j % 2 == 0) a0 = __builtin_fmaf(e, j >= q ? e : 0.0f, a0);
          if constexpr (j % 2 == 1) a1 = __builtin_fmaf(e, j >= q ? e : 0.0f, a1);
        });
        fn2 = a0 + a1;
      }
      wave_lds_sync();
      const double dg = (l < q) ? R[l * NL + l] : 0.0;
      wave_lds_sync();
      if (l < q) R[l * NL + l] = 0.0;
      rdg = dg;
      invRd = (l < q) ? rcp1(dg) : 0.0;
    }
    wave_lds_sync();
  }

  // ------------------------------------------------------------- outputs
  // multipliers by constraint (row l: upper bound of x_l, row 16 + l: lower)
  double *lamb = R;  // 32 over the dead R; the solves capture in R[32:48]
  double *xcap = R + 2 * NL;
  wave_lds_sync();
  lamb[l] = 0.0;
  lamb[l + NL] = 0.0;
  wave_lds_sync();
  if (l < q && iam >= 0) lamb[iam] = um;
  wave_lds_sync();
  const double lu = lamb[l], ll = lamb[l + NL];
  wave_lds_sync();
  // x = -H^{-1} (f + A^T lam), A^T lam = lam_u - lam_l: L y = g, L^T x = -y,
  // lane-parallel (finished components captured by same-address LDS stores)
  const double invd = rcp1(Lp[lrow(l) + l]);
  double Lrow[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) Lrow[j] = Lp[lrow(l) + j];
  wave_lds_sync();
  {
    double acc = fl + lu - ll;
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
    const double bad = row_min((__builtin_fabs(xl) < kInf) ? 0.0 : -1.0);
    if (status == QPB_OK && bad < 0.0) status = QPB_NUMERICAL;
  }
  if (live && var) {
    xg[g * n + l] = xl;
    lamg[g * 2 * n + l] = lu;
    lamg[g * 2 * n + n + l] = ll;
  }
  const int sh = (threadIdx.x & 63) & ~(NL - 1);
  const uint32_t wu = (uint32_t)((__ballot(actu) >> sh) & 0xFFFFull);
  const uint32_t wlo = (uint32_t)((__ballot(actl) >> sh) & 0xFFFFull);
  if (live && l == 0) {
    actg[g] = wu | (wlo << n);  // m = 2n <= 32: one word, A = [I; -I] row order
    statg[g] = status;
    if (itg) itg[g] = it;
  }
}

}  // namespace box
}  // namespace qpb

extern "C" hipError_t qpb_launch_gi_box(const qpb_desc *d, const double *H, const double *f, const double *lb,
                                        const double *ub, double *x, double *lam, uint32_t *active, int32_t *status,
                                        int32_t *iters, hipStream_t stream) {
  const long long blocks = (d->batch + qpb::box::QPB - 1) / qpb::box::QPB;
  const int max_iter = d->max_iter > 0 ? d->max_iter : 4 * (3 * d->n) + 8;
  const double tol = d->feas_tol > 0 ? d->feas_tol : 1e-10;
  if (d->n == 16)
    hipLaunchKernelGGL(qpb::box::gi_box_kernel<true>, dim3((unsigned)blocks), dim3(64), 0, stream, H, f, lb, ub, x,
                       lam, active, status, iters, d->n, (long long)d->batch, max_iter, tol);
  else
    hipLaunchKernelGGL(qpb::box::gi_box_kernel<false>, dim3((unsigned)blocks), dim3(64), 0, stream, H, f, lb, ub, x,
                       lam, active, status, iters, d->n, (long long)d->batch, max_iter, tol);
  return hipGetLastError();
}
