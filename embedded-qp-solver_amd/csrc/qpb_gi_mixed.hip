// qpb_gi_mixed.hip -- mixed-precision active-set kernel for 16 < n <= 32,
// m <= 64 (BASELINE configs[4]: fp32 factorisation + fp64 iterative
// refinement), gfx950.
//
// The active set is found in fp32: the dual Goldfarb-Idnani method of
// qpb_gi_wave.hip (D = A L^{-T}, Householder ADDs, Givens DROPs; one QP per
// 64-lane wavefront, lane l owns row l of D and, while factorising, row l of
// H) with every factor, slack and multiplier in fp32 -- half the registers
// and LDS of the fp64 kernel and fp32 FMAs (3.1 against 5.2 cycles per wave
// instruction on gfx950, tools/probe/valu_probe.hip).  Then, in fp64, for
// that active set W:
//
//   KKT system   [H    A_W^T] [x]   [-f ]
//                [A_W  0    ] [l] = [b_W]
//   residuals    r1 = -f - H x - A_W^T l,   r2 = b_W - A_W x     (fp64, the
//                original fp64 H and A rows re-read from L2 / Infinity Cache)
//   correction   v  = H^{-1} r1,  c = A_W v - r2,
//                dl = M^{-1} c    (M = A_W H^{-1} A_W^T = R^T R, the fp32 R of
//                                  the active-set loop),
//                dx = v - H^{-1} A_W^T dl,   with H^{-1} = L^{-T} L^{-1} from
//                                  the fp32 L (fp64 arithmetic on fp32 entries)
// repeated kRefine times (each step gains ~cond(H) * 2^-24; cond <~ 1e4 for
// the conditioned family of configs[4]).  The result is then VERIFIED in
// fp64: every row's slack against feas_tol, every multiplier >= 0, the last
// correction below 1e-11 relative.  A QP that fails (or whose fp32 pass ended
// NOT_SPD / INFEASIBLE / MAX_ITER) is marked and re-solved by the fp64 kernel
// (qpb_gi_wave.hip, REDO mode) in a second launch on the same stream, so
// every returned answer is an fp64 KKT point of the same active set the fp64
// path finds.
//
// Replaces, batched: matrix_ops.c matrix_invert (LU + explicit inverse,
// :487-630) and matrix_mult (:235-271) on the solver path of
// qp_solvers.c:103-319.
#include <type_traits>

#include "qpb_common.h"
#include "qpb.h"

namespace qpb {
namespace mx {

constexpr int NP = 32;                     // padded n
constexpr int L_SIZE = NP * (NP + 1) / 2;  // 528 floats: L packed rows
constexpr int OFF_L = 0;
constexpr int OFF_R = L_SIZE;              // 528: R[i][j] at j*NP + i (fp32, zero diagonal)
constexpr int OFF_X = OFF_R + NP * NP;     // 1552: fp32 exchange row (NP) + s_p, |D_p|^2
constexpr int OFF_D = OFF_X + NP + 8;      // 1592 (8-B aligned): fp64 area, 64 doubles
constexpr int SLOTF = OFF_D + 2 * 64;      // 1720 floats = 6,880 B per wave
constexpr int RST = 36;                    // fp32 staging row stride (16-B aligned rows)
static_assert(NP * RST <= OFF_X, "load staging fits in L + R");
static_assert(OFF_D % 4 == 0, "fp64 area 16-byte aligned");
constexpr float kDepTol32 = 1e-10f;  // |d2|^2 <= kDepTol32 |d|^2  <=>  z = 0 (fp32 noise ~1e-14)
constexpr float kFeas32 = 1e-6f;     // fp32 violation threshold (relative); fp64 verifies against feas_tol
constexpr int kRefine = 3;           // fp64 refinement steps (at most; stops once converged)
constexpr int32_t kRedo = 100;       // internal status: re-solve in fp64
#ifndef QPB_MX_OCC
#define QPB_MX_OCC 3  // waves per SIMD
#endif
#ifndef QPB_MX_STAGE
#define QPB_MX_STAGE 3  // diagnostic builds: 0 fp32 only, 1 + initial x, 2 + refinement, 3 + verification
#endif

__device__ __forceinline__ float readlane_f(float v, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}
__device__ __forceinline__ double readlane_d(double v, int lane) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const int lo = __builtin_amdgcn_readlane((int)(unsigned)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(unsigned)(b >> 32), lane);
  return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
// exact min over the 64 lanes (wave-uniform)
__device__ __forceinline__ float wave_minf(float v) {
  v = __builtin_fminf(v, dppf<kRowRor + 8>(v));
  v = __builtin_fminf(v, dppf<kRowRor + 4>(v));
  v = __builtin_fminf(v, dppf<kRowRor + 2>(v));
  v = __builtin_fminf(v, dppf<kRowRor + 1>(v));
  const float a = readlane_f(v, 0), b = readlane_f(v, 16), c = readlane_f(v, 32), d = readlane_f(v, 48);
  return __builtin_fminf(__builtin_fminf(a, b), __builtin_fminf(c, d));
}
// sum over lanes 0-31 (wave-uniform; xor butterfly inside each 16-lane row)
__device__ __forceinline__ float half_sumf(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x141>(v);
  v += dppf<0x140>(v);
  return readlane_f(v, 0) + readlane_f(v, 16);
}
__device__ __forceinline__ double wave_maxd(double v) {
  v = __builtin_fmax(v, ror<8>(v));
  v = __builtin_fmax(v, ror<4>(v));
  v = __builtin_fmax(v, ror<2>(v));
  v = __builtin_fmax(v, ror<1>(v));
  const double a = readlane_d(v, 0), b = readlane_d(v, 16), c = readlane_d(v, 32), d = readlane_d(v, 48);
  return __builtin_fmax(__builtin_fmax(a, b), __builtin_fmax(c, d));
}
__device__ __forceinline__ bool wave_any(bool p) { return __ballot(p) != 0; }
__device__ __forceinline__ void pinf(float &v) { asm volatile("" : "+v"(v)); }
// a finite fp32 key whose low 6 mantissa bits carry a lane index
__device__ __forceinline__ float pack_key64f(float v, int idx) {
  return __builtin_bit_cast(float, (__builtin_bit_cast(uint32_t, v) & ~63u) | (uint32_t)idx);
}
constexpr float kBigF = 3.4028234663852886e38f;

// E . (fp32 vector in LDS)
__device__ __forceinline__ float dot_xchf(const float (&E)[NP], const float *x) {
  float a0 = 0.f, a1 = 0.f;
#pragma unroll
  for (int j = 0; j < NP; j += 4) {
    const float4 v = *reinterpret_cast<const float4 *>(&x[j]);
    a0 = __builtin_fmaf(E[j], v.x, a0);
    a1 = __builtin_fmaf(E[j + 1], v.y, a1);
    a0 = __builtin_fmaf(E[j + 2], v.z, a0);
    a1 = __builtin_fmaf(E[j + 3], v.w, a1);
  }
  return a0 + a1;
}

// fp64 dot of a global fp64 row (n entries) with the fp64 vector in LDS;
// eight loads in flight at a time (all 32 at once would need 64 VGPRs)
__device__ __forceinline__ double row_dot(const double *__restrict__ row, int n, const double *xd) {
  asm volatile("" : "+v"(row));  // per-call loads (see at_w)
  double a0 = 0.0, a1 = 0.0;
#pragma unroll
  for (int j0 = 0; j0 < NP; j0 += 8) {
    double r[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) r[t] = row[j0 + t < n ? j0 + t : 0];
#pragma unroll
    for (int t = 0; t < 8; t += 2) {
      const double2 xv = *reinterpret_cast<const double2 *>(&xd[j0 + t]);
      a0 = __builtin_fma(j0 + t < n ? r[t] : 0.0, xv.x, a0);
      a1 = __builtin_fma(j0 + t + 1 < n ? r[t + 1] : 0.0, xv.y, a1);
    }
  }
  return a0 + a1;
}

__host__ __device__ constexpr int lrow(int i) { return i * (i + 1) / 2; }

// (R^T R)^{-1} c over the q active positions (position j in lane j), fp64
// arithmetic with the fp32 R (column-major, zero diagonal) and its diagonal
// in registers (ird = 1 / R_ll as fp64)
__device__ __forceinline__ double minv(double c, int q, int l, const float *R, double ird) {
  const int lc = l & (NP - 1);
  double acc = (l < q) ? c : 0.0, yl = 0.0;
  for (int i = 0; i < q; ++i) {  // R^T y = c (forward)
    const double yi = readlane_d(acc * ird, i);
    if (l == i) yl = yi;
    acc = __builtin_fma(-((l > i && l < q) ? (double)R[lc * NP + i] : 0.0), yi, acc);
  }
  acc = yl;
  double zl = 0.0;
  for (int j = q - 1; j >= 0; --j) {  // R z = y (backward)
    const double zj = readlane_d(acc * ird, j);
    if (l == j) zl = zj;
    acc = __builtin_fma(-((l < j) ? (double)R[j * NP + lc] : 0.0), zj, acc);
  }
  return l < q ? zl : 0.0;
}

// sum_k w_k A[iam_k][l] over the active positions (lanes l < n), fp64.
// Each position's row is one coalesced load across the lanes; the loads go
// out eight at a time before their FMAs (a load-use per position would
// expose one L2 / Infinity-Cache round trip per active constraint).
__device__ __forceinline__ double at_w(const double *__restrict__ Aq, int n, int q, int iam, double w, int l) {
  // a fresh base pointer per call: the loads are loop-invariant across the
  // refinement steps, and hoisted out of the loop they would pin up to 64 VGPRs
  asm volatile("" : "+s"(Aq));
  double s0 = 0.0, s1 = 0.0;
  const int lc = l < n ? l : 0;
  for (int k0 = 0; k0 < q; k0 += 8) {  // wave-uniform
    double a[8], u[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int kk = k0 + t < q ? k0 + t : q - 1;  // clamped: a duplicate row with u = 0
      const int row = __builtin_amdgcn_readlane(iam, kk);
      u[t] = k0 + t < q ? readlane_d(w, kk) : 0.0;
      a[t] = Aq[row * n + lc];
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      if (t % 2 == 0) s0 = __builtin_fma(u[t], a[t], s0);
      else s1 = __builtin_fma(u[t], a[t], s1);
    }
  }
  return l < n ? s0 + s1 : 0.0;
}

template <int OCC>
__global__ __launch_bounds__(64, OCC) void gi_mixed_kernel(
    const double *__restrict__ Hg, const double *__restrict__ fg, const double *__restrict__ Ag,
    const double *__restrict__ bg, double *__restrict__ xg, double *__restrict__ lamg, uint32_t *__restrict__ actg,
    int32_t *__restrict__ statg, int32_t *__restrict__ itg, int n, int m, long long batch, int max_iter,
    double feas_tol) {
  __shared__ __attribute__((aligned(16))) float lds[SLOTF];
  const int l = threadIdx.x;
  const long long g = blockIdx.x;
  if (g >= batch) return;
  float *Lp = lds + OFF_L;
  float *R = lds + OFF_R;
  float *xch = lds + OFF_X;
  double *xd = reinterpret_cast<double *>(lds + OFF_D);  // fp64 exchange (64)

  const double *Hq = Hg + g * (long long)n * n;
  const double *Aq = m > 0 ? Ag + g * (long long)m * n : Hq;
  const double *bq = m > 0 ? bg + g * (long long)m : Hq;
  const bool rowok = l < m;

  // ------------------------------------------------------------------ load
  // coalesced flat fp64 reads (lane l takes element i*64 + l), staged in LDS
  // as fp32 rows of stride RST, read back one row per lane (as qpb_gi_wave.hip)
  float Lr[NP], E[NP];
  const double bv = bq[rowok ? l : 0];
  const double fv = fg[g * n + (l < n ? l : 0)];
  {
    const int nn = n * n, h0 = (m < NP ? m : NP) * n, h1 = m * n - h0;
    double hv[16], av[2][16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int e = i * 64 + l;
      hv[i] = Hq[min(e, nn - 1)];
      av[0][i] = Aq[max(min(e, h0 - 1), 0)];
      av[1][i] = Aq[max(h0 + min(e, h1 - 1), 0)];
    }
    const int q0 = 64 / n, r0 = 64 - q0 * n;
    const int rl = l / n, cl = l - rl * n;
    auto stage = [&](const double (&v)[16]) {
      int r = rl, c = cl;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        lds[min(r, NP) * RST + c] = (float)v[i];
        c += r0;
        r += q0;
        if (c >= n) {
          c -= n;
          ++r;
        }
      }
    };
    // dst = keep ? staged row : (first ? 0 : dst)
    auto fetch_row = [&](float (&dst)[NP], int row, bool keep, bool first) {
#pragma unroll
      for (int j = 0; j < NP; j += 4) {
        const float4 v = *reinterpret_cast<const float4 *>(&lds[row * RST + j]);
        const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) dst[j + i] = keep ? vv[i] : (first ? 0.f : dst[j + i]);
      }
    };
#pragma unroll
    for (int i = 0; i < ((NP + 1) * RST + 255) / 256; ++i)
      if (i * 256 + 4 * l < (NP + 1) * RST)
        *reinterpret_cast<float4 *>(&lds[i * 256 + 4 * l]) = make_float4(0.f, 0.f, 0.f, 0.f);
    wave_lds_sync();
    stage(av[0]);
    wave_lds_sync();
    fetch_row(E, l & (NP - 1), l < NP && rowok, true);
    wave_lds_sync();
    if (m > NP) {
      stage(av[1]);
      wave_lds_sync();
      fetch_row(E, l & (NP - 1), l >= NP && rowok, false);
      wave_lds_sync();
    }
    stage(hv);
    wave_lds_sync();
    fetch_row(Lr, l & (NP - 1), l < n, true);
    wave_lds_sync();
  }

  float nrm2 = 0.f;
#pragma unroll
  for (int j = 0; j < NP; ++j) nrm2 = __builtin_fmaf(E[j], E[j], nrm2);
  const float bl = rowok ? (float)bv : 0.f;
  const float invn = nrm2 > 0.f ? __builtin_amdgcn_rsqf(nrm2) : 0.f;
  const float thr = (rowok && nrm2 > 0.f) ? -kFeas32 * (1.f + __builtin_fabsf(bl) * invn) : -__builtin_huge_valf();
  const bool infeasible0 = wave_any(rowok && nrm2 == 0.f && bl < -kFeas32 * (1.f + __builtin_fabsf(bl)));
  const float fl = l < n ? (float)fv : 0.f;

  // ---- fp32 sweep: H = L L^T, D = A L^{-T}, y = L^{-1} f, s = b + D y
  bool spd = true;
  float ya = fl, s = bl;
  unroll<NP>([&](auto K) {
    constexpr int k = K;
    if (k >= n) return;  // wave-uniform: padded columns stay zero
    __builtin_amdgcn_sched_barrier(0);
    wave_lds_sync();
    if (l < NP) xch[l] = Lr[k];  // column k = pivot row k by symmetry
    wave_lds_sync();
    const float akk = xch[k];
    spd = spd && (akk > 0.f);
    const float ik = __builtin_amdgcn_rsqf(akk);
    const float ik2 = ik * ik;
    const float c = Lr[k] * ik2;
    const float e = E[k];
    const float e2 = e * ik2;
    Lr[k] *= ik;
    E[k] = e * ik;
    constexpr int j0 = (k + 1) / 4 * 4;
    unroll<(NP - j0) / 4>([&](auto P) {
      constexpr int j = j0 + 4 * P;
      const float4 v = *reinterpret_cast<const float4 *>(&xch[j]);
      const float vv[4] = {v.x, v.y, v.z, v.w};
      unroll<4>([&](auto I) {
        constexpr int jj = j + I;
        if constexpr (jj >= k + 1) {
          Lr[jj] = __builtin_fmaf(-c, vv[I], Lr[jj]);
          E[jj] = __builtin_fmaf(-e2, vv[I], E[jj]);
        }
      });
    });
    const float fk = readlane_f(ya, k);
    ya = __builtin_fmaf(-c, fk, ya);
    s = __builtin_fmaf(E[k], fk * ik, s);  // D[l][k] final: s += D[l][k] y_k
  });
  // L -> LDS (fp32 packed rows; descending j, in-order DS, clamped tail)
  unroll<NP>([&](auto J) {
    constexpr int j = NP - 1 - J;
    if (l < NP) Lp[lrow(l) + j <= L_SIZE - 1 ? lrow(l) + j : L_SIZE - 1] = Lr[j];
    wave_lds_sync();
  });
  float dn = 0.f;
#pragma unroll
  for (int j = 0; j < NP; ++j) dn = __builtin_fmaf(E[j], E[j], dn);

  // ------------------------------------------------------ fp32 active-set loop
  wave_lds_sync();
  for (int j = 0; j < NP; ++j) R[j * NP + (l & (NP - 1))] = 0.f;
  int q = 0;
  float um = 0.f, rdg = 0.f, invRd = 0.f;
  int iam = -1;
  bool act = false;
  int status = !spd ? QPB_NOT_SPD : (infeasible0 ? QPB_INFEASIBLE : QPB_MAX_ITER);
  bool done = !spd || infeasible0;
  bool selecting = true;
  int p = 0;
  float up = 0.f;
  int it = 0;
  wave_lds_sync();
  while (!done && it < max_iter) {
    ++it;
    if (selecting) {
      const float v = s * invn;
      const bool viol = !act && v < thr;
      const float key = wave_minf(viol ? pack_key64f(v, l) : kBigF);
      if (!(key < 0.f)) {
        status = QPB_OK;
        break;
      }
      p = __builtin_amdgcn_readfirstlane((int)(__builtin_bit_cast(uint32_t, key) & 63u));
      up = 0.f;
      selecting = false;
    }
    wave_lds_sync();
    if (l == p) {
#pragma unroll
      for (int j = 0; j < NP; j += 4) *reinterpret_cast<float4 *>(&xch[j]) = make_float4(E[j], E[j + 1], E[j + 2], E[j + 3]);
      xch[NP] = s;
      xch[NP + 1] = dn;
    }
    wave_lds_sync();
    const float Dpl = xch[l & (NP - 1)];
    const float Dpq = xch[q < NP ? q : 0];
    const float sp = xch[NP];
    const float dd = xch[NP + 1];
    wave_lds_sync();
    if (l < q) xch[l] = 0.f;
    const float nd2 = half_sumf((l & (NP - 1)) >= q ? Dpl * Dpl : 0.f);
    const float dl = (l < NP) ? -Dpl : 0.f;
    wave_lds_sync();
    // r = R^{-1} d1 over the active positions
    float rm = 0.f;
    if (q > 0) {
      float acc = (l < q) ? dl : 0.f;
      for (int j = q - 1; j >= 0; --j) {
        const float rj = readlane_f(acc * invRd, j);
        acc = __builtin_fmaf(-R[j * NP + (l & (NP - 1))], rj, acc);
      }
      rm = acc * invRd;
    }
    float t1 = kBigF;
    int k = 0;
    if (q > 0) {
      const bool cand = l < q && rm > 0.f;
      const float ratio = um / rm;
      t1 = wave_minf(cand ? ratio : kBigF);
      const unsigned long long hit = __ballot(cand && ratio == t1);
      k = hit ? (int)__builtin_ctzll(hit) : 0;
    }
    const float t2 = (nd2 > kDepTol32 * dd) ? -sp / nd2 : kBigF;
    const float t = t1 < t2 ? t1 : t2;
    if (!(t < kBigF)) {
      status = QPB_INFEASIBLE;
      break;
    }
    if (t2 < kBigF) s = __builtin_fmaf(t, dot_xchf(E, xch), s);
    um = __builtin_fmaf(-t, rm, um);
    up += t;
    if (t2 <= t1) {
      // ADD p: Householder on columns q.. (v = d2 + alpha e_q)
      const float nrm = __builtin_sqrtf(nd2);
      const float alpha = Dpq <= 0.f ? -nrm : nrm;
      const float beta = 1.f / __builtin_fmaf(alpha, Dpq, nd2);
      wave_lds_sync();
      if (l == q) xch[q] = Dpq + alpha;
      wave_lds_sync();
      const float w = beta * dot_xchf(E, xch);
#pragma unroll
      for (int j = 0; j < NP; j += 4) {
        const float4 v = *reinterpret_cast<const float4 *>(&xch[j]);
        E[j] = __builtin_fmaf(-w, v.x, E[j]);
        E[j + 1] = __builtin_fmaf(-w, v.y, E[j + 1]);
        E[j + 2] = __builtin_fmaf(-w, v.z, E[j + 2]);
        E[j + 3] = __builtin_fmaf(-w, v.w, E[j + 3]);
      }
      if (l < NP) R[q * NP + l] = (l < q) ? dl : 0.f;
      if (l == q) {
        rdg = alpha;
        invRd = 1.f / alpha;
        iam = p;
        um = up;
      }
      if (l == p) act = true;
      ++q;
      selecting = true;
    } else {
      // DROP active position k
      const int c = __builtin_amdgcn_readlane(iam, k);
      if (l == c) act = false;
      const float un = __shfl(um, (l + 1) & 63);
      const int in = __shfl(iam, (l + 1) & 63);
      if (l >= k && l < q - 1) {
        um = un;
        iam = in;
      } else if (l == q - 1) {
        um = 0.f;
        iam = -1;
      }
      const int lc = l & (NP - 1);
      wave_lds_sync();
      if (l < q) R[l * NP + l] = rdg;
      const bool shift = l >= k && l < q - 1;
      for (int i = 0; i < q; ++i) {
        wave_lds_sync();
        const float nx = R[((lc + 1) & (NP - 1)) * NP + i];
        wave_lds_sync();
        if (shift) R[l * NP + i] = nx;
        else if (l == q - 1) R[l * NP + i] = 0.f;
      }
      for (int j = k; j < q - 1; ++j) {
        wave_lds_sync();
        const float a = R[j * NP + j], bb = R[j * NP + j + 1];
        const float ir = __builtin_amdgcn_rsqf(__builtin_fmaf(a, a, bb * bb));
        const float cj = a * ir, sj = bb * ir;
        const float rj = R[lc * NP + j], rj1 = R[lc * NP + j + 1];
        wave_lds_sync();
        if (l >= j && l < q - 1) {
          R[l * NP + j] = __builtin_fmaf(cj, rj, sj * rj1);
          R[l * NP + j + 1] = (l == j) ? 0.f : __builtin_fmaf(-sj, rj, cj * rj1);
        }
        unroll<NP - 1>([&](auto JJ) {
          constexpr int jj = JJ;
          if (jj == j) {
            const float e0 = E[jj], e1 = E[jj + 1];
            E[jj] = __builtin_fmaf(cj, e0, sj * e1);
            E[jj + 1] = __builtin_fmaf(-sj, e0, cj * e1);
            asm volatile("; rot %0" ::"n"(jj));
          }
        });
      }
      wave_lds_sync();
      if (l < NP) R[l * NP + q - 1] = 0.f;
      --q;
      wave_lds_sync();
      const float dg = (l < q) ? R[l * NP + l] : 0.f;
      wave_lds_sync();
      if (l < q) R[l * NP + l] = 0.f;
      rdg = dg;
      invRd = (l < q) ? 1.f / dg : 0.f;
    }
  }

  // ------------------------------------------- fp64 refinement of the KKT system
  bool redo = status != QPB_OK;
  double xl = 0.0, lam = (l < q) ? (double)um : 0.0;
  if (!redo && QPB_MX_STAGE >= 1) {
    const int h = l >> 5, c = l & (NP - 1);
    // explicit fp32 U = R^{-1} (upper triangular, M^{-1} = U U^T): lane j
    // solves R u = e_j right-looking over the columns of R (contiguous in
    // LDS); the diagonal of R goes through LDS first
    wave_lds_sync();
    if (l < NP) xch[l] = (l < q) ? rdg : 1.f;
    wave_lds_sync();
    {
      float U[NP];
#pragma unroll
      for (int k = 0; k < NP; ++k) U[k] = 0.f;
      unroll<NP>([&](auto II) {
        constexpr int i = NP - 1 - II;
        if (i >= q) return;  // wave-uniform
        wave_lds_sync();
        int cc = c;
        asm volatile("" : "+v"(cc));
        const float ui = ((cc == i) ? 1.f : U[i]) * __builtin_amdgcn_rcpf(xch[i]);
        U[i] = ui;
        unroll<i>([&](auto K) {
          constexpr int k = K;
          U[k] = __builtin_fmaf(-R[i * NP + k], ui, U[k]);
        });
        unroll<i + 1>([&](auto K) {
          constexpr int k = K;
          pinf(U[k]);
        });
      });
      wave_lds_sync();  // every lane has read R: U overwrites it, column j by lane j
      if (l < q) {
#pragma unroll
        for (int k = 0; k < NP; k += 4)
          *reinterpret_cast<float4 *>(&R[l * NP + k]) = make_float4(U[k], U[k + 1], U[k + 2], U[k + 3]);
      }
      wave_lds_sync();
    }
    // explicit fp32 H^{-1} = L^{-T} L^{-1}: lane l solves for column c (= row
    // c), L's entries read from LDS as broadcasts (rows >= n of L are zero)
    wave_lds_sync();
    float Hi[NP];
    unroll<NP>([&](auto K) {  // L y = e_c
      constexpr int k = K;
      // one row of L at a time: the ordering point keeps the step's LDS reads
      // from being hoisted (all 528 would be live at once), the opaque copy
      // of c keeps the lane test from becoming 32 hoisted SGPR masks
      wave_lds_sync();
      int cc = c;
      asm volatile("" : "+v"(cc));
      float acc = (cc == k) ? 1.f : 0.f;
      unroll<k>([&](auto I) {
        constexpr int i = I;
        acc = __builtin_fmaf(-Lp[lrow(k) + i], Hi[i], acc);
      });
      const float dk = Lp[lrow(k) + k];
      Hi[k] = k < n ? acc * __builtin_amdgcn_rcpf(dk) : 0.f;
      asm volatile("" : "+v"(Hi[k]));  // materialised here: IR passes would sink the step's FMAs
    });
    // the backward pass reads the same entries again: this ordering point
    // keeps the compiler from holding all 528 across the two passes
    wave_lds_sync();
    unroll<NP>([&](auto KK) {  // L^T z = y
      constexpr int k = NP - 1 - KK;
      wave_lds_sync();
      float acc = Hi[k];
      unroll<NP - 1 - k>([&](auto I) {
        constexpr int i = k + 1 + I;
        acc = __builtin_fmaf(-Lp[lrow(i) + k], Hi[i], acc);
      });
      const float dk = Lp[lrow(k) + k];
      Hi[k] = k < n ? acc * __builtin_amdgcn_rcpf(dk) : 0.f;
      asm volatile("" : "+v"(Hi[k]));
    });
    // (H^{-1} r)_c, r broadcast through LDS (lanes < 32 hold components)
    auto hinv_apply = [&](double r) -> double {
      wave_lds_sync();
      if (l < NP) xd[l] = (l < n) ? r : 0.0;
      wave_lds_sync();
      double a0 = 0.0, a1 = 0.0;
#pragma unroll
      for (int j = 0; j < NP; j += 2) {
        if (j % 8 == 0) wave_lds_sync();  // eight reads in flight at a time (register budget)
        const double2 v = *reinterpret_cast<const double2 *>(&xd[j]);
        // opaque copies: the fp64 conversions of H^{-1} stay inside each call
        // (hoisted out of the refinement loop they would hold 64 VGPRs)
        float h0 = Hi[j], h1 = Hi[j + 1];
        asm volatile("" : "+v"(h0), "+v"(h1));
        a0 = __builtin_fma((double)h0, v.x, a0);
        a1 = __builtin_fma((double)h1, v.y, a1);
      }
      return (c < n) ? a0 + a1 : 0.0;
    };
    // (H x)_c in fp64.  H is read two rows per load instruction (coalesced):
    // lane l gets H[2i+h][c] = H[c][2i+h] (symmetric), half of row c, so the
    // dot is a half-row partial plus the other half's (lane ^ 32).  Re-read
    // per call (L2 / Infinity Cache): held across the refinement it would
    // pin 32 VGPRs.
    auto h_mul = [&](double x) -> double {
      wave_lds_sync();
      if (l < NP) xd[l] = (l < n) ? x : 0.0;
      wave_lds_sync();
      const double *Hp = Hq;
      asm volatile("" : "+s"(Hp));
      double a = 0.0;
#pragma unroll
      for (int i0 = 0; i0 < NP / 2; i0 += 8) {
        double hv[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int r = 2 * (i0 + t) + h;
          const bool ok = r < n && c < n;
          const double v = Hp[ok ? r * n + c : 0];
          hv[t] = ok ? v : 0.0;
        }
        wave_lds_sync();
#pragma unroll
        for (int t = 0; t < 8; ++t) a = __builtin_fma(hv[t], xd[2 * (i0 + t) + h], a);
      }
      const double o = __shfl_xor(a, 32);
      return (c < n) ? a + o : 0.0;
    };
    // (U U^T c) over the positions, fp64 arithmetic, c broadcast through LDS
    auto minv2 = [&](double cv) -> double {
      wave_lds_sync();
      if (l < NP) xd[l] = (l < q) ? cv : 0.0;
      wave_lds_sync();
      double w = 0.0;  // w_j = sum_k U[k][j] c_k, lane j reads its column
#pragma unroll
      for (int k = 0; k < NP; k += 2) {
        if (k % 8 == 0) wave_lds_sync();
        const double2 v = *reinterpret_cast<const double2 *>(&xd[k]);
        w = __builtin_fma((double)R[c * NP + k], v.x, w);
        w = __builtin_fma((double)R[c * NP + k + 1], v.y, w);
      }
      wave_lds_sync();
      if (l < NP) xd[l] = (l < q) ? w : 0.0;
      wave_lds_sync();
      double z = 0.0;  // z_i = sum_j U[i][j] w_j, lane i reads row i (strided)
#pragma unroll
      for (int j = 0; j < NP; j += 2) {
        if (j % 8 == 0) wave_lds_sync();
        const double2 v = *reinterpret_cast<const double2 *>(&xd[j]);
        z = __builtin_fma((double)R[j * NP + c], v.x, z);
        z = __builtin_fma((double)R[(j + 1) * NP + c], v.y, z);
      }
      return (l < q) ? z : 0.0;
    };
    const double *arow = Aq + (l < q && iam >= 0 ? iam : 0) * n;
    const double bw = (l < q && iam >= 0) ? bq[iam] : 0.0;
    // x = -H^{-1} (f + A_W^T lam)
    xl = -hinv_apply(fv + at_w(Aq, n, q, iam, lam, l));
    const double x_init = xl;
    // Refinement.  The error after a step is ~ kappa * (that step's
    // correction), kappa the observed contraction (corr_s / corr_{s-1});
    // stop once that estimate is below 1e-12
    double corr = 1.0, corr_prev = 1.0;
    bool converged = false;
    for (int step = 0; step < (QPB_MX_STAGE >= 2 ? kRefine : 0) && !converged; ++step) {
      // r1 = -f - H x - A_W^T lam; one A_W product per step: c = A_W (x + v) - b_W
      const double hx = h_mul(xl);
      const double r1 = (l < n) ? -(fv + hx + at_w(Aq, n, q, iam, lam, l)) : 0.0;
      const double v = hinv_apply(r1);
      wave_lds_sync();
      if (l < NP) xd[l] = (l < n) ? xl + v : 0.0;
      wave_lds_sync();
      const double cc = (l < q) ? row_dot(arow, n, xd) - bw : 0.0;
      const double dlam = minv2(cc);
      const double dx = v - hinv_apply(at_w(Aq, n, q, iam, dlam, l));
      xl += dx;
      lam += dlam;
      corr_prev = corr;
      corr = wave_maxd(l < n ? __builtin_fabs(dx) : 0.0) / (1.0 + wave_maxd(l < n ? __builtin_fabs(xl) : 0.0));
      converged = corr <= 1e-13 || (step > 0 && corr * (corr / corr_prev) <= 1e-12);
    }
    // ---- fp64 verification: lam >= 0, refinement converged, and every
    // inactive row feasible.  A row whose fp32 normalised slack is beyond the
    // fp32 solution's error (tau) is feasible in fp64 too; the others are
    // checked in fp64 (their A rows re-read).
    if (QPB_MX_STAGE >= 3) {
      wave_lds_sync();
      if (l < NP) xd[l] = (l < n) ? xl : 0.0;
      wave_lds_sync();
      const double xa = wave_maxd(l < n ? __builtin_fabs(xl) : 0.0);
      const double dxi = wave_maxd(l < n ? __builtin_fabs(xl - x_init) : 0.0);
      const double tau = 1e-3 * (1.0 + xa) + 64.0 * dxi;
      bool bad = false;
      if (rowok && !act && nrm2 > 0.f && (double)(s * invn) < tau) {
        const double *ar = Aq + l * n;
        double an = 0.0;
        // clamped loads, all issued before the sum (the empty asm consumes
        // them): a guarded load per j became a branch with its own wait
        // (NP serial round trips)
        double av[NP];
#pragma unroll
        for (int j = 0; j < NP; ++j) av[j] = ar[j < n ? j : 0];
#pragma unroll
        for (int j = 0; j < NP; ++j) asm volatile("" : "+v"(av[j]));
#pragma unroll
        for (int j = 0; j < NP; ++j) an = j < n ? __builtin_fma(av[j], av[j], an) : an;
        const double sl = bv - row_dot(ar, n, xd);
        bad = sl < -feas_tol * (__builtin_sqrt(an) + __builtin_fabs(bv));
      }
      const double lmax = wave_maxd(l < q ? __builtin_fabs(lam) : 0.0);
      if (l < q && lam < 0.0) {
        if (lam < -1e-9 * (1.0 + lmax)) bad = true;
        lam = 0.0;
      }
      bad = bad || !(__builtin_fabs(xl) < kInf) || !converged;
      redo = wave_any(bad);
    }
  }

  // ------------------------------------------------------------- outputs
  wave_lds_sync();
  double *lamb = xd;
  lamb[l] = 0.0;
  wave_lds_sync();
  if (l < q && iam >= 0) lamb[iam] = lam;
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
    statg[g] = redo ? kRedo : QPB_OK;
    if (itg) itg[g] = it;
  }
}

}  // namespace mx
}  // namespace qpb

// the fp64 kernel over the QPs the mixed kernel marked (qpb_gi_wave.hip)
extern "C" hipError_t qpb_launch_gi_wave_redo(const qpb_desc *d, const double *H, const double *f, const double *A,
                                              const double *b, double *x, double *lam, uint32_t *active,
                                              int32_t *status, int32_t *iters, hipStream_t stream);

extern "C" hipError_t qpb_launch_gi_mixed(const qpb_desc *d, const double *H, const double *f, const double *A,
                                          const double *b, double *x, double *lam, uint32_t *active,
                                          int32_t *status, int32_t *iters, hipStream_t stream) {
  const int max_iter = d->max_iter > 0 ? d->max_iter : 4 * (d->n + d->m) + 8;
  const double tol = d->feas_tol > 0 ? d->feas_tol : 1e-10;
  hipLaunchKernelGGL(qpb::mx::gi_mixed_kernel<QPB_MX_OCC>, dim3((unsigned)d->batch), dim3(64), 0, stream, H, f, A, b, x, lam,
                     active, status, iters, d->n, d->m, (long long)d->batch, max_iter, tol);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || (d->flags & QPB_FLAG_DIAG_NO_REDO)) return e;
  // the marked QPs again, in fp64 (every other wave of this launch exits at once)
  return qpb_launch_gi_wave_redo(d, H, f, A, b, x, lam, active, status, iters, stream);
}
