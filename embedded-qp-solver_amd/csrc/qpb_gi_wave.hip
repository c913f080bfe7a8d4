// qpb_gi_wave.hip -- active-set QP kernel for 16 < n <= 32, m <= 64 (gfx950).
//
// Same method as qpb_gi.hip (dual active set of Goldfarb & Idnani on
// D = A L^{-T}, see there), mapped one QP per 64-lane wavefront: lane l owns
// row l of D, every per-QP scalar is wave-uniform, so control flow never
// diverges and no QP waits for another.  Single values from one lane are
// broadcast by v_readlane (SGPR results).  Selection: dual steepest edge
// (-s / |D[l, q:]|) as in qpb_gi.hip, 14.94 -> 13.83 iterations per QP on
// the configs[4] batch.
//
// Setup, one right-looking sweep as in qpb_gi.hip, except that the pivot row
// is gathered by symmetry: row k of the Schur complement is its column k, and
// element k of a lane's row is a compile-time register index -- every lane
// stores it (one b64 store per step, no lane-selected writes).  Row r of H / L is split over the
// two wave halves (lane r: columns 0-15, lane r + 32: columns 16-31), so the
// upper half carries half the Schur update instead of idling, and the row
// costs 32 VGPRs instead of 64 (the sweep's spills went from 104 to 25 dwords;
// 6.30 -> 5.88 ms at B = 262,144 with bitwise the same output,
// profiles/r02/s4/ab_n32_half_sweep.json).
//
// Vectors every lane needs whole (the sweep's pivot column, row p of D, the
// Householder vector, y) are held as a DPP operand pair -- entry j at lane
// j & 15 of every 16-lane row -- and enter the FMAs by their own row_newbcast
// (v_fmac_f64_dpp): the LDS only carries two b64 reads per lane per vector,
// not 16 broadcast b128 reads per product (round 3: 5.86 -> 4.64 ms at
// B = 262,144, profiles/r03/n32/ab_wave_v4.json).  The loop's back
// substitution runs in the same layout (4.63 -> 4.57 ms), and R's column
// stride is padded to 34 doubles: DROP's row-wise reads and writes were 16-
// to 32-way bank conflicts, 1 400 of them per QP (PMC), now 35 (4.54 ->
// 4.44 ms, profiles/r03/n32/ab_wave_rstride.json).
//
// LDS per QP (one wave): L packed rows (n(n+1)/2), R column-major NP x NP with
// zero diagonal, the pivot / exchange vector, the y / x capture.
//
// BOX (round 5, qpb_solve_box for 16 < n <= 32): lb <= x <= ub with
// A = [I; -I], b = [ub; -lb] kept implicit -- the constraint class of the
// reference's admm() (qp_solvers.c:255-319, box config.h:29-30) at the
// reference's larger N_DIM.  Row l of D starts from +-e (no A is read: 9.7 KB
// per QP at n = 32 instead of 26.1 KB), the same sweep turns it into
// +-row of L^{-T}, the loop is unchanged, and x = -H^{-1}(f + lam_u - lam_l)
// needs no A rows.  Absent bounds (NULL or +-inf) have slack +inf.
#include <type_traits>

#include "qpb_common.h"
#include "qpb.h"



namespace qpb {
namespace wv {

constexpr int NP = 32;                              // padded n
constexpr int NH = NP / 2;                          // H / L row half held per lane
constexpr int L_SIZE = NP * (NP + 1) / 2;           // 528
constexpr int OFF_L = 0;
constexpr int RS = NP + 1;                          // R column stride (odd): row-wise and column-
                                                    // wise b64 accesses both conflict-free
constexpr int OFF_R = L_SIZE;                       // 528: R[i][j] at j*RS + i; column 0 (no entry
                                                    // above the diagonal) doubles as the exchange row
constexpr int OFF_X = OFF_R + NP * RS;              // 1584: s_p, |d|^2 of the exchange
constexpr int SLOT = OFF_X + 2;                     // 1586 doubles = 12,688 B
// a CU holds 12 one-wave workgroups of <= 12,800 B of LDS (11 from 13,056 B:
// tools/probe/occupancy_probe.hip); the round-4 slot (RS = 34, a separate
// exchange row: 13,248 B) ran 11
static_assert(SLOT * 8 <= 12800, "12 waves (3 per SIMD) per CU by LDS");
static_assert(OFF_R % 2 == 0 && OFF_X % 2 == 0, "b128 alignment of the exchange row and s_p");
constexpr double kDepTol = 1e-24;

__host__ __device__ constexpr int lrow(int i) { return i * (i + 1) / 2; }

__device__ __forceinline__ double readlane_d(double v, int lane) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const int lo = __builtin_amdgcn_readlane((int)(unsigned)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(unsigned)(b >> 32), lane);
  return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
// exact min over the 64 lanes (wave-uniform result)
__device__ __forceinline__ double wave_min(double v) {
  v = row_min(v);
  const double a = readlane_d(v, 0), b = readlane_d(v, 16), c = readlane_d(v, 32), d = readlane_d(v, 48);
  return __builtin_fmin(__builtin_fmin(a, b), __builtin_fmin(c, d));
}
__device__ __forceinline__ bool wave_any(bool p) { return __ballot(p) != 0; }

template <int N, class FX, class FY>
__device__ __forceinline__ double dot2(FX &&x, FY &&y, double init = 0.0) {
  double a0 = init, a1 = 0.0;
  unroll<N>([&](auto J) {
    constexpr int j = J;
    if constexpr (j % 2 == 0) a0 = __builtin_fma(x(j), y(j), a0);
    else a1 = __builtin_fma(x(j), y(j), a1);
  });
  return a0 + a1;
}

// D[l,:] . v for a vector held as v[j] = vA at lane j (j < 16) and vB at
// lane j - 16 (j >= 16) of every 16-lane row: the FMA takes v[j] by its own
// DPP broadcast (row_newbcast), four accumulators.  The caller has issued
// dpp_ready on a VALU-written vA / vB.
__device__ __forceinline__ double bdot(const double (&E)[NP], double vA, double vB) {
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  unroll<NH>([&](auto J) {
    constexpr int j = J;
    fmac_bc<j>(a[j & 1], vA, E[j]);
    fmac_bc<j>(a[2 + (j & 1)], vB, E[NH + j]);
  });
  return (a[0] + a[1]) + (a[2] + a[3]);
}
__device__ __forceinline__ void dpp_ready2(double a, double b) { asm volatile("s_nop 1" ::"v"(a), "v"(b)); }

// one QP per wavefront; MR = 1 (m <= 64); OCC waves per SIMD
// REDO: solve only the QPs the mixed-precision kernel marked (status
// kRedoStatus, qpb_gi_mixed.hip); every other wave exits at once
constexpr int32_t kRedoStatus = 100;
template <int OCC, bool STAMP = false, bool REDO = false, bool BOX = false>
__global__ __launch_bounds__(64, OCC) void gi_wave_kernel(
    const double *__restrict__ Hg, const double *__restrict__ fg, const double *__restrict__ Ag,
    const double *__restrict__ bg, double *__restrict__ xg, double *__restrict__ lamg, uint32_t *__restrict__ actg,
    int32_t *__restrict__ statg, int32_t *__restrict__ itg, int n, int m, long long batch, int max_iter,
    double feas_tol, unsigned long long *__restrict__ dbg = nullptr) {
  __shared__ double lds[SLOT];
  SectionClock<STAMP> clk;
  const int l = threadIdx.x;
  const long long g = blockIdx.x;
  if (g >= batch) return;
  if constexpr (REDO) {
    if (statg[g] != kRedoStatus) return;
  }
  double *Lp = lds + OFF_L;
  double *R = lds + OFF_R;
  double *xch = R;             // the exchange row: R's column 0, never read by the back substitution
  double *xsd = lds + OFF_X;   // s_p, |D[p,:]|^2

  const double *Hq = Hg + g * (long long)n * n;
  // BOX: Ag = lb, bg = ub (n per QP, either may be NULL), m = 2n
  const double *Aq = BOX ? Hq : m > 0 ? Ag + g * (long long)m * n : Hq;
  const double *bq = BOX ? Hq : m > 0 ? bg + g * (long long)m : Hq;
  const bool rowok = l < m;

  // ------------------------------------------------------------------ load
  // H and A are read flat and coalesced (lane l takes element i*64 + l: a
  // row-per-lane read would touch 64 cache lines per instruction and, with
  // eight QPs in flight per CU, thrash the vector L1), staged in LDS as rows
  // of stride NP + 2 doubles (16-byte aligned rows, conflict-free b128 row
  // reads) and read back one row per lane: A rows 0-31, A rows 32-63, then H
  // (each part at most 32 rows = 16 loads of 64 lanes); H row r = l & 31 is
  // read back as half a row per lane (lane r: columns 0-15, lane r + 32:
  // columns 16-31, the sweep's split layout).
  double Lr[NH], E[NP];
  double bv;
  if constexpr (BOX) {
    // row l < n: x_l <= ub_l; row n + i: -x_i <= -lb_i.  An absent bound
    // (NULL array) is ub = +inf / lb = -inf, so both rows get b = +inf (as
    // gi_box), never a -inf slack
    const int bi = l < n ? l : (l < 2 * n ? l - n : 0);
    const double *bnd = l < n ? bg : Ag;
    const double v = bnd ? bnd[g * n + bi] : (l < n ? kInf : -kInf);
    bv = l < n ? v : -v;
    if (!(bv == bv)) bv = kInf;  // NaN bound: absent
  } else {
    bv = bq[rowok ? l : 0];
  }
  const double fv = fg[g * n + (l < n ? l : 0)];
  {
    constexpr int RST = NP + 2;  // staged row stride
    const int nn = n * n, h0 = (m < NP ? m : NP) * n, h1 = m * n - h0;  // A rows 0-31 | 32-63
    double hv[16], av[2][16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int e = i * 64 + l;
      // clamped, not masked: lane-vs-runtime compares would be hoisted into
      // SGPR masks; elements past the end land in rows nobody reads
      hv[i] = Hq[min(e, nn - 1)];
      if constexpr (!BOX) {
        av[0][i] = Aq[max(min(e, h0 - 1), 0)];
        av[1][i] = Aq[max(h0 + min(e, h1 - 1), 0)];
      }
    }
    // flat element e = i*64 + l -> (row, col) of an n-column matrix, stepped
    // per i by 64 = q0*n + r0 (n > 16, so one wrap per step at most)
    const int q0 = 64 / n, r0 = 64 - q0 * n;
    const int rl = l / n, cl = l - rl * n;
    auto stage = [&](const double (&v)[16]) {
      int r = rl, c = cl;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        lds[min(r, NP) * RST + c] = v[i];  // rows >= the part's own: unread
        c += r0;
        r += q0;
        if (c >= n) {
          c -= n;
          ++r;
        }
      }
    };
    auto fetch_row = [&](double (&dst)[NP], int row, bool keep) {
      if (keep) {
#pragma unroll
        for (int j = 0; j < NP; j += 2) {
          const double2 v = *reinterpret_cast<const double2 *>(&lds[row * RST + j]);
          dst[j] = v.x;
          dst[j + 1] = v.y;
        }
      }
    };
#pragma unroll
    for (int j = 0; j < NP; ++j) E[j] = 0.0;
#pragma unroll
    for (int j = 0; j < NH; ++j) Lr[j] = 0.0;
    // columns >= n of the staging rows stay zero for all three parts
#pragma unroll
    for (int i = 0; i < (NP * RST + 127) / 128; ++i)
      if (i * 128 + 2 * l < (NP + 1) * RST)
        *reinterpret_cast<double2 *>(&lds[i * 128 + 2 * l]) = make_double2(0.0, 0.0);
    wave_lds_sync();
    if constexpr (BOX) {
      // row l: +e_l (l < n), -e_{l-n} (n <= l < 2n)
#pragma unroll
      for (int j = 0; j < NP; ++j) E[j] = (l == j && l < n) ? 1.0 : (l - n == j && l < 2 * n) ? -1.0 : 0.0;
    } else {
      // A first: the 64 loaded registers of A are released before L's 64 are
      // filled (peak E + L + H's 32 staged values, not E + L + A)
      stage(av[0]);
      wave_lds_sync();
      fetch_row(E, l & (NP - 1), l < NP && rowok);
      wave_lds_sync();
      if (m > NP) {
        stage(av[1]);
        wave_lds_sync();
        fetch_row(E, l & (NP - 1), l >= NP && rowok);
        wave_lds_sync();
      }
    }
    stage(hv);
    wave_lds_sync();
    if ((l & (NP - 1)) < n) {
      const double *src = &lds[(l & (NP - 1)) * RST + (l >> 5) * NH];
#pragma unroll
      for (int j = 0; j < NH; j += 2) {
        const double2 v = *reinterpret_cast<const double2 *>(&src[j]);
        Lr[j] = v.x;
        Lr[j + 1] = v.y;
      }
    }
    wave_lds_sync();
  }

  clk.tick(0);  // load
  const double nrm2 = dot2<NP>([&](int j) { return E[j]; }, [&](int j) { return E[j]; });
  const double bl = rowok ? bv : 0.0;
  // violated: s / |D row| < -tol (1 + |b| / |D row|), i.e. s < -tol (|D row| + |b|)
  const double thr = (rowok && nrm2 > 0.0) ? -feas_tol * (nrm2 * rsq(nrm2) + __builtin_fabs(bl)) : -kInf;
  const bool infeasible0 =
      wave_any(rowok && nrm2 == 0.0 && bl < -feas_tol * (1.0 + __builtin_fabs(bl)));
  const double fl = l < n ? fv : 0.0;

  // ---- H = L L^T, D = A L^{-T}, y = L^{-1} f (right-looking, pivot row by symmetry)
  if (l < NP) R[l] = 0.0;  // y capture (components >= n stay zero)
  bool spd = true;
  double ya = fl;
  // Split rows: lane (h, r) = (l >> 5, l & 31) holds S[r][16h .. 16h + 15] of
  // the Schur complement.  Step k: every lane stores its entry kk = k % 16 at
  // pv[32h + r], so column k (= pivot row k by symmetry) is pv[32 kh + .],
  // kh = k / 16.  Lane l reads two entries of it, PA = S[l & 15][k] and
  // PB = S[16 + (l & 15)][k] (the same pair in every 16-lane row), and the
  // updates take S[j][k] from lane j & 15 of the row by the FMA's own DPP
  // broadcast: the pivot row is neither held nor streamed from LDS.  The half
  // owning column k scales it into L[r][k]; entries left of it are final L
  // (zero coefficient ch on the lower half), entries right of it take the
  // Schur update.
  const bool hi = l >= NP;
  const int r = l & (NP - 1), li = l & (NH - 1);
  double *pv = R + 2 * NP;  // R is free until the loop (R[0..31]: y capture)
  unroll<NP>([&](auto K) {
    constexpr int k = K, kh = k / NH, kk = k % NH;
    if (k >= n) return;  // wave-uniform: padded columns stay zero
    __builtin_amdgcn_sched_barrier(0);
    wave_lds_sync();
    pv[l] = Lr[kk];
    wave_lds_sync();
    const double PA = pv[NP * kh + li], PB = pv[NP * kh + NH + li];
    const double akk = pv[NP * kh + k];
    const double srk = (r & NH) ? PB : PA;  // S[r][k]
    spd = spd && (akk > 0.0);
    const double ik = rsq(akk);
    const double ik2 = ik * ik;
    const double c = srk * ik2;
    const double ch = hi ? c : 0.0;
    const double e = E[k];
    const double me2 = -(e * ik2);
    E[k] = e * ik;
    pin(E[k]);  // scaled here: sunk to the sweep's exit, the 1/sqrt pivots stay live (spills)
    // D row: columns j > k
    unroll<NP - 1 - k>([&](auto JJ) {
      constexpr int j = k + 1 + JJ;
      if constexpr (j < NH) fmac_bc<j>(E[j], PA, me2);
      else fmac_bc<j - NH>(E[j], PB, me2);
    });
    const double mc = -c, mch = -ch;
    if constexpr (kh == 0) {
      // entry jj of the lane's half is column 16h + jj: S[16h + jj][k] is
      // lane jj's PA (lower half) or PB (upper half)
      const double Ph = hi ? PB : PA;
      dpp_ready(Ph);
      unroll<NH>([&](auto JJ) {
        constexpr int jj = JJ;
        if constexpr (jj < kk) {
          fmac_bc<jj>(Lr[jj], Ph, mch);
        } else if constexpr (jj == kk) {
          double u = Lr[jj];
          fmac_bc<jj>(u, Ph, mc);
          Lr[jj] = hi ? u : Lr[jj] * ik;
        } else {
          fmac_bc<jj>(Lr[jj], Ph, mc);
        }
      });
    } else {
      Lr[kk] = hi ? Lr[kk] * ik : Lr[kk];
      // the upper half's entries j - 16 (the lower half's are final: ch = 0)
      unroll<NP - 1 - k>([&](auto JJ) {
        constexpr int j = k + 1 + JJ;
        fmac_bc<j - NH>(Lr[j - NH], PB, mch);
      });
    }
    const double fk = readlane_d(ya, k);
    ya = __builtin_fma(-c, fk, ya);
    R[k] = fk * ik;  // y_k, same-address store from every lane
  });
  clk.tick(1);  // sweep
  // L -> LDS, packed rows: the upper half first, then the lower half, each in
  // descending column order.  A dead entry (column j > r) lands in a later row
  // at a smaller column, whose owner writes it afterwards (in-order DS).
  unroll<NH>([&](auto J) {
    constexpr int jj = NH - 1 - J;
    if (hi) Lp[lrow(r) + NH + jj <= L_SIZE - 1 ? lrow(r) + NH + jj : L_SIZE - 1] = Lr[jj];
    wave_lds_sync();
  });
  unroll<NH>([&](auto J) {
    constexpr int jj = NH - 1 - J;
    if (!hi) Lp[lrow(r) + jj] = Lr[jj];
    wave_lds_sync();
  });
  // y replicated: s = b + D y, |D row|^2
  wave_lds_sync();
  double s = bl + bdot(E, R[li], R[NH + li]);
  const double dn = dot2<NP>([&](int j) { return E[j]; }, [&](int j) { return E[j]; });
  float fn2 = (float)dn;  // |D[l, q:]|^2, the free part of the row (scale of the selection key)

  // ------------------------------------------------------ active-set loop
  wave_lds_sync();
  for (int j = 0; j < NP; ++j) R[j * RS + (l & (NP - 1))] = 0.0;
  int q = 0;
  double um = 0.0, rdg = 0.0;
  double ninvA = 0.0, ninvB = 0.0;  // -1 / R_jj of positions j = l & 15 and 16 + (l & 15)
  int iam = -1;
  bool act = false;
  int status = !spd ? QPB_NOT_SPD : (infeasible0 ? QPB_INFEASIBLE : QPB_MAX_ITER);
  bool done = !spd || infeasible0;
  bool selecting = true;
  int p = 0;
  double up = 0.0;
  int it = 0;
  wave_lds_sync();
  clk.tick(2);  // L store, s, |D row|^2
  while (!done && it < max_iter) {
    ++it;
    if (selecting) {
      // dual steepest edge as in qpb_gi.hip: the most violated row by
      // -s / |D[l, q:]| (fp32), the row in the low 6 bits (0 = none violated)
      const bool viol = !act && s < thr;
      // (fn2 >= 0, clamped where it shrinks; the 2^-100 floor keeps a violated
      // row's key nonzero when the ratio underflows or fn2 overflows)
      const float kf = __builtin_fmaf((float)(-s), __builtin_amdgcn_rsqf(fn2), 0x1p-100f);
      uint32_t kk = viol ? ((__float_as_uint(kf) & ~63u) | (uint32_t)l) : 0u;
      kk = row_max_u32(kk);
      const uint32_t k0 = __builtin_amdgcn_readlane(kk, 0), k1 = __builtin_amdgcn_readlane(kk, 16);
      const uint32_t k2 = __builtin_amdgcn_readlane(kk, 32), k3 = __builtin_amdgcn_readlane(kk, 48);
      const uint32_t key = __builtin_elementwise_max(__builtin_elementwise_max(k0, k1), __builtin_elementwise_max(k2, k3));
      if (key == 0u) {
        status = QPB_OK;
        break;
      }
      p = (int)(key & 63u);
      up = 0.0;
      selecting = false;
    }
    clk.tick(3);  // select
    // row p of D, s_p, |D_p|^2 through LDS; the active columns zeroed there
    wave_lds_sync();
    if (l == p) {
#pragma unroll
      for (int j = 0; j < NP; j += 2) *reinterpret_cast<double2 *>(&xch[j]) = make_double2(E[j], E[j + 1]);
      *reinterpret_cast<double2 *>(xsd) = make_double2(s, dn);
    }
    wave_lds_sync();
    // row p as the DPP operand pair (entry j at lane j & 15 of every row),
    // d2 = its columns >= q
    const double XA = xch[li], XB = xch[NH + li];
    const double Dpq = xch[q < NP ? q : 0];
    const double2 spdd = *reinterpret_cast<const double2 *>(xsd);
    const double sp = spdd.x, dd = spdd.y;
    const double Dpl = (l & NH) ? XB : XA;  // D[p][l], lanes 0-31
    const double d2A = li >= q ? XA : 0.0, d2B = li + NH >= q ? XB : 0.0;
    dpp_ready2(d2A, d2B);
    const double nd2 = row_sum(__builtin_fma(d2A, d2A, d2B * d2B));  // |d2|^2
    const double dl = (l < NP) ? -Dpl : 0.0;

    clk.tick(4);  // exchange
    // r = R^{-1} d1 over the active positions, in the DPP layout: lane i of
    // every row carries positions i (nA) and 16 + i (nB), on the negated
    // accumulator n = -acc (n_l += R[l][j] r_j, r_j = n_j * (-1 / R_jj)); r_j
    // enters the FMAs by their own DPP broadcast from lane j & 15.  Steps run
    // in groups of four columns whose R entries are read up front; a step
    // j >= q adds zeros (n_j = 0, column j of R is zero).
    double rm = 0.0;
    if (q > 0) {
      double nA = li < q ? XA : 0.0, nB = li + NH < q ? XB : 0.0;  // -d1 = D[p][0:q]
      unroll<NP / 4>([&](auto G) {
        constexpr int j0 = NP - 4 - 4 * G;
        if (j0 < q) {
          double ra[4], rb[4];
          unroll<4>([&](auto I) {
            constexpr int j = j0 + 3 - I;
            if constexpr (j > 0) ra[I] = R[j * RS + li];
            if constexpr (j >= NH) rb[I] = R[j * RS + NH + li];
          });
          unroll<4>([&](auto I) {
            constexpr int j = j0 + 3 - I;
            if constexpr (j >= NH) {
              const double tj = nB * ninvB;
              fmac_bc_nop<j - NH>(nA, tj, ra[I]);
              fmac_bc<j - NH>(nB, tj, rb[I]);
            } else if constexpr (j > 0) {  // column 0: no entry above the diagonal
              const double tj = nA * ninvA;
              fmac_bc_nop<j>(nA, tj, ra[I]);
            }
          });
        }
      });
      const double rA = nA * ninvA, rB = nB * ninvB;
      rm = (l < q) ? ((l & NH) ? rB : rA) : 0.0;
    }
    clk.tick(5);  // back solve
    const double t2 = (nd2 > kDepTol * dd) ? -sp * rcp(nd2) : kBig;
    double t1 = kBig;
    int k = 0;
    if (q > 0) {
      const double ratio = um * rcp(rm);
      const bool cand = l < q && rm > 0.0;
      // the reduction only when a candidate ratio is below t2 (a partial step);
      // otherwise the QP adds p and t1 stays kBig (as qpb_gi.hip)
      if (__ballot(cand && ratio < t2)) {
        // the packed key only picks k; the step is lane k's exact ratio
        const double tk = wave_min(cand ? pack_key64(ratio, l) : kBig);
        k = __builtin_amdgcn_readfirstlane(key_index64(tk));
        const double tx = readlane_d(ratio, k);
        t1 = tk < kBig ? tx : kBig;
      }
    }
    const double t = t1 < t2 ? t1 : t2;
    if (!(t < kBig)) {
      status = QPB_INFEASIBLE;
      break;
    }
    // d2 is streamed from the exchange row (broadcast reads), not held
    double ud = 0.0;  // D[l,:] . d2
    if (t2 < kBig) {
      ud = bdot(E, d2A, d2B);
      s = __builtin_fma(t, ud, s);
    }
    pin(s);
    um = __builtin_fma(-t, rm, um);
    up += t;

    clk.tick(6);  // step
    if (t2 <= t1) {
      // ADD p (Householder on columns q.., v = d2 + alpha e_q as in qpb_gi.hip)
      const double nrm = nd2 * rsq(nd2);
      const double alpha = Dpq <= 0.0 ? -nrm : nrm;
      const double beta = rcp(__builtin_fma(alpha, Dpq, nd2));
      const double ia = rcp(alpha);
      // the reflection maps e_q to -d2 / alpha: the new column q is -ud / alpha
      // and leaves the free part, whose norm the reflection otherwise keeps
      const float cq = (float)(ud * ia);
      fn2 = __builtin_fmaxf(__builtin_fmaf(-cq, cq, fn2), 0.0f);
      // v = d2 + alpha e_q in the DPP operand pair; E -= beta (E . v) v^T
      const double vA = d2A + (li == q ? alpha : 0.0), vB = d2B + (li + NH == q ? alpha : 0.0);
      // E v = E d2 + alpha E[:, q] = ud + alpha E[q] (q wave-uniform: a
      // scalar branch tree picks the register)
      double eq = 0.0;
      switch (q & (NP - 1)) {
#define QPB_COLQ_CASE(J) \
  case J:                \
    eq = E[J];           \
    break;
        QPB_COLQ_CASE(0) QPB_COLQ_CASE(1) QPB_COLQ_CASE(2) QPB_COLQ_CASE(3)
        QPB_COLQ_CASE(4) QPB_COLQ_CASE(5) QPB_COLQ_CASE(6) QPB_COLQ_CASE(7)
        QPB_COLQ_CASE(8) QPB_COLQ_CASE(9) QPB_COLQ_CASE(10) QPB_COLQ_CASE(11)
        QPB_COLQ_CASE(12) QPB_COLQ_CASE(13) QPB_COLQ_CASE(14) QPB_COLQ_CASE(15)
        QPB_COLQ_CASE(16) QPB_COLQ_CASE(17) QPB_COLQ_CASE(18) QPB_COLQ_CASE(19)
        QPB_COLQ_CASE(20) QPB_COLQ_CASE(21) QPB_COLQ_CASE(22) QPB_COLQ_CASE(23)
        QPB_COLQ_CASE(24) QPB_COLQ_CASE(25) QPB_COLQ_CASE(26) QPB_COLQ_CASE(27)
        QPB_COLQ_CASE(28) QPB_COLQ_CASE(29) QPB_COLQ_CASE(30) QPB_COLQ_CASE(31)
#undef QPB_COLQ_CASE
      }
      const double mw = -beta * __builtin_fma(alpha, eq, ud);
      dpp_ready2(vA, vB);
      unroll<NH>([&](auto J) {
        constexpr int j = J;
        fmac_bc<j>(E[j], vA, mw);
        fmac_bc<j>(E[NH + j], vB, mw);
      });
      if (l < NP) R[q * RS + l] = (l < q) ? dl : 0.0;
      if (l == q) {
        rdg = alpha;
        iam = p;
        um = up;
      }
      if (li == q) ninvA = -ia;
      if (li + NH == q) ninvB = -ia;
      if (l == p) act = true;
      ++q;
      selecting = true;
      clk.tick(7);  // add
    } else {
      // DROP active position k
      const int c = __builtin_amdgcn_readlane(iam, k);
      if (l == c) act = false;
      const double un = __shfl(um, (l + 1) & 63);
      const int in = __shfl(iam, (l + 1) & 63);
      if (l >= k && l < q - 1) {
        um = un;
        iam = in;
      } else if (l == q - 1) {
        um = 0.0;
        iam = -1;
      }
      const int lc = l & (NP - 1);
      wave_lds_sync();
      if (l < q) R[l * RS + l] = rdg;
      // columns k+1 .. q-1 move left by one, column q-1 clears: lane l copies
      // column l+1 whole (rows >= q are zero), a quarter column per pass (DS
      // instructions run in order, so each read precedes every lane's write;
      // b64: the odd stride leaves odd columns 8-byte aligned)
      const bool shift = l >= k && l < q - 1, clear = l == q - 1;
      unroll<4>([&](auto Hh) {
        constexpr int i0 = (NP / 4) * Hh;
        double col[NP / 4];
        wave_lds_sync();
        unroll<NP / 4>([&](auto I) { col[I] = R[((lc + 1) & (NP - 1)) * RS + i0 + I]; });
        wave_lds_sync();
        if (shift || clear) {
          unroll<NP / 4>([&](auto I) { R[lc * RS + i0 + I] = clear ? 0.0 : col[I]; });
        }
      });
      for (int j = k; j < q - 1; ++j) {
        wave_lds_sync();
        const double a = R[j * RS + j], bb = R[j * RS + j + 1];
        const double ir = rsq(__builtin_fma(a, a, bb * bb));
        const double cj = a * ir, sj = bb * ir;
        const double rj = R[lc * RS + j], rj1 = R[lc * RS + j + 1];
        wave_lds_sync();
        if (l >= j && l < q - 1) {
          R[l * RS + j] = __builtin_fma(cj, rj, sj * rj1);
          R[l * RS + j + 1] = (l == j) ? 0.0 : __builtin_fma(-sj, rj, cj * rj1);
        }
        // the same rotation on columns j, j+1 of D (j wave-uniform)
        unroll<NP - 1>([&](auto JJ) {
          constexpr int jj = JJ;
          if (jj == j) {
            const double e0 = E[jj], e1 = E[jj + 1];
            E[jj] = __builtin_fma(cj, e0, sj * e1);
            E[jj + 1] = __builtin_fma(-sj, e0, cj * e1);
            // keeps the 31 branches distinct: merged, they would address E
            // through a pointer phi and put it on the stack (scratch)
            asm volatile("; rot %0" ::"n"(jj));
          }
        });
      }
      // column q-1 rejoins the free part
      unroll<NP>([&](auto JJ) {
        constexpr int jj = JJ;
        if (jj == q - 1) {
          fn2 = __builtin_fmaf((float)E[jj], (float)E[jj], fn2);
          asm volatile("; fn %0" ::"n"(jj));
        }
      });
      wave_lds_sync();
      if (l < NP) R[l * RS + q - 1] = 0.0;
      --q;
      wave_lds_sync();
      const double dg = (l < q) ? R[l * RS + l] : 0.0;
      const double dgA = R[li * RS + li], dgB = R[(NH + li) * RS + NH + li];
      wave_lds_sync();
      if (l < q) R[l * RS + l] = 0.0;
      rdg = dg;
      ninvA = li < q ? -rcp(dgA) : 0.0;
      ninvB = li + NH < q ? -rcp(dgB) : 0.0;
      clk.tick(8);  // drop
    }
  }
  clk.tick(9);  // loop exit

  // ------------------------------------------------------------- outputs
  // x = -H^{-1} (f + A^T lam): g = f + sum_k u_k a_{iact_k}, then L y = g,
  // L^T x = -y lane-parallel (L read from LDS, broadcasts by v_readlane)
  double gl = fl;
  const int ll = l & (NP - 1);
  double *lamb = R;  // lambda by row (64 entries over the dead R)
  if constexpr (BOX) {
    // a_k = +e_k (k < n) or -e_{k-n}: g_l = f_l + lam[l] - lam[n + l], the
    // multipliers scattered by row first (no A rows to gather)
    wave_lds_sync();
    lamb[l] = 0.0;
    wave_lds_sync();
    if (l < q && iam >= 0) lamb[iam] = um;
    wave_lds_sync();
    if (l < n) gl = fl + (lamb[l] - lamb[n + l]);
  } else {
    // every active row's element first (one memory round trip instead of q
    // dependent ones), 16 at a time (one trip for q <= 16, the usual case;
    // 8 at a time was 0.3-0.6 % slower), then the sum in position order
    const int lc = l < n ? l : 0;
    const int ias = iam > 0 ? iam : 0;
    unroll<NP / 16>([&](auto Hh) {
      constexpr int k0 = 16 * Hh;
      if (k0 < q) {
        double arow[16];
        __builtin_amdgcn_sched_barrier(0);
        unroll<16>([&](auto K) {
          constexpr int kk = k0 + K;
          arow[K] = kk < q ? Aq[__builtin_amdgcn_readlane(ias, kk) * n + lc] : 0.0;
        });
        unroll<16>([&](auto K) {
          constexpr int kk = k0 + K;
          if (kk < q) gl = __builtin_fma(readlane_d(um, kk), (l < n) ? arow[K] : 0.0, gl);
        });
      }
    });
  }
  wave_lds_sync();
  const double invd = ll < n ? rcp(Lp[lrow(ll) + ll]) : 0.0;
  // Both solves lane-parallel: step k broadcasts the finished component from
  // lane k (v_readlane), every lane then updates its own; a lane's entries
  // past its own component are read unmasked (they sit inside L's packed
  // storage) and only update dead values, and each component is captured by
  // a same-address LDS store as it is broadcast (64..95 of the dead R).
  // Masking those entries instead (kk < ll / kk > ll per step) kept 64 lane
  // masks live in SGPRs and spilled them (round 6: 112 SGPR spills).
  double *xcap = R + 2 * NP;
  double xl;
  {
    double Lrow[NP];  // row ll of L (entries past the diagonal: dead)
    unroll<NP>([&](auto K) {
      constexpr int kk = K;
      Lrow[kk] = Lp[lrow(ll) + kk];
    });
    double acc = gl;
    unroll<NP>([&](auto K) {
      constexpr int kk = K;
      if (kk < n) {
        const double yk = readlane_d(acc * invd, kk);
        acc = __builtin_fma(-Lrow[kk], yk, acc);
        xcap[kk] = yk;
      }
    });
  }
  wave_lds_sync();
  {
    double acc = ll < n ? xcap[ll] : 0.0;
    double Lcol[NP];  // column ll of L (entries above the diagonal: dead)
    unroll<NP>([&](auto K) {
      constexpr int kk = K;
      Lcol[kk] = Lp[lrow(kk) + ll];
    });
    wave_lds_sync();
    unroll<NP>([&](auto K) {
      constexpr int kk = NP - 1 - K;
      if (kk < n) {
        const double xk = readlane_d(acc * invd, kk);
        acc = __builtin_fma(-Lcol[kk], xk, acc);
        xcap[kk] = xk;
      }
    });
    wave_lds_sync();
    xl = -xcap[ll];
  }
  if (status == QPB_OK && wave_any(l < n && !(__builtin_fabs(xl) < kInf))) status = QPB_NUMERICAL;
  clk.tick(10);  // x = -H^{-1} (f + A^T lam)
  // lambda scatter through LDS (64 entries over the dead R; BOX: done above)
  if constexpr (!BOX) {
    wave_lds_sync();
    lamb[l] = 0.0;
    wave_lds_sync();
    if (l < q && iam >= 0) lamb[iam] = um;
  }
  wave_lds_sync();
  if (rowok) lamg[g * m + l] = lamb[l];
  if (l < n) xg[g * n + l] = xl;
  const unsigned long long bal = __ballot(act);
  if (l == 0) {
    if (m > 0) {
      const int words = (m + 31) / 32;
      actg[g * words] = (uint32_t)bal;
      if (words > 1) actg[g * words + 1] = (uint32_t)(bal >> 32);
    }
    statg[g] = status;
    if (itg) itg[g] = it;
  }
  clk.tick(11);  // stores
  clk.flush(dbg);
}

}  // namespace wv
}  // namespace qpb

extern "C" hipError_t qpb_launch_gi_wave(const qpb_desc *d, const double *H, const double *f, const double *A,
                                         const double *b, double *x, double *lam, uint32_t *active, int32_t *status,
                                         int32_t *iters, hipStream_t stream) {
  const int max_iter = d->max_iter > 0 ? d->max_iter : 4 * (d->n + d->m) + 8;
  const double tol = d->feas_tol > 0 ? d->feas_tol : 1e-10;
  // three waves per SIMD: the 168-VGPR cap spills ~50 dwords, nearly all in
  // the setup sweep; measured 6.30 ms against 6.47 ms for two waves with the
  // same code at B = 262,144 (profiles/r02/ab_n32.json; round 1 measured
  // the opposite on its kernel)
  hipLaunchKernelGGL(qpb::wv::gi_wave_kernel<3>, dim3((unsigned)d->batch), dim3(64), 0, stream, H, f, A, b, x, lam,
                     active, status, iters, d->n, d->m, (long long)d->batch, max_iter, tol);
  return hipGetLastError();
}

extern "C" hipError_t qpb_launch_gi_wave_sections(const qpb_desc *d, const double *H, const double *f,
                                                  const double *A, const double *b, double *x, double *lam,
                                                  uint32_t *active, int32_t *status, int32_t *iters,
                                                  unsigned long long *sections, hipStream_t stream) {
  const int max_iter = d->max_iter > 0 ? d->max_iter : 4 * (d->n + d->m) + 8;
  const double tol = d->feas_tol > 0 ? d->feas_tol : 1e-10;
  hipLaunchKernelGGL((qpb::wv::gi_wave_kernel<2, true>), dim3((unsigned)d->batch), dim3(64), 0, stream, H, f, A, b,
                     x, lam, active, status, iters, d->n, d->m, (long long)d->batch, max_iter, tol, sections);
  return hipGetLastError();
}

extern "C" hipError_t qpb_launch_gi_wave_redo(const qpb_desc *d, const double *H, const double *f, const double *A,
                                              const double *b, double *x, double *lam, uint32_t *active,
                                              int32_t *status, int32_t *iters, hipStream_t stream) {
  const int max_iter = d->max_iter > 0 ? d->max_iter : 4 * (d->n + d->m) + 8;
  const double tol = d->feas_tol > 0 ? d->feas_tol : 1e-10;
  hipLaunchKernelGGL((qpb::wv::gi_wave_kernel<2, false, true>), dim3((unsigned)d->batch), dim3(64), 0, stream, H, f,
                     A, b, x, lam, active, status, iters, d->n, d->m, (long long)d->batch, max_iter, tol);
  return hipGetLastError();
}

// qpb_solve_box for 16 < n <= 32 (m = 2n): A = [I; -I], b = [ub; -lb] implicit
extern "C" hipError_t qpb_launch_gi_wave_box(const qpb_desc *d, const double *H, const double *f, const double *lb,
                                             const double *ub, double *x, double *lam, uint32_t *active,
                                             int32_t *status, int32_t *iters, hipStream_t stream) {
  const int max_iter = d->max_iter > 0 ? d->max_iter : 4 * (d->n + d->m) + 8;
  const double tol = d->feas_tol > 0 ? d->feas_tol : 1e-10;
  hipLaunchKernelGGL((qpb::wv::gi_wave_kernel<3, false, false, true>), dim3((unsigned)d->batch), dim3(64), 0, stream,
                     H, f, lb, ub, x, lam, active, status, iters, d->n, d->m, (long long)d->batch, max_iter, tol);
  return hipGetLastError();
}
