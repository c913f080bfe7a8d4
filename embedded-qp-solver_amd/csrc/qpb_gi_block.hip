// qpb_gi_block.hip -- active-set QP kernel for 32 < n <= 128, m <= 256 (gfx950).
//
// BASELINE config 4 sizes (n = 128, m = 256).  Same method as qpb_gi.hip
// (dual active set of Goldfarb & Idnani on D = A L^{-T}), one QP per
// 1024-thread workgroup (four wavefronts per SIMD):
//   the 4 lanes of quad r own row r of D, 32 columns each, in registers
//   (row dot products combine the quarters with two DPP quad_perm steps);
//   LDS holds one 128 x 128 fp64 matrix (128 KiB): H while it is factorised
//   in place (right-looking, the whole workgroup on each rank-1 update),
//   then L (lower triangle) while D = A L^{-T} is formed, then R
//   (column-major, zero diagonal) through the active-set loop.  L is
//   recomputed from H at the end for x = -H^{-1} (f + A^T lam).
// The serial pieces of an iteration (argmin, the back substitution with R,
// the ratio test, Givens sweeps) run on wavefront 0 with v_readlane
// broadcasts; the O(m n) updates of D run on every thread.  All control flow
// is workgroup-uniform (values taken from LDS after a barrier).
#include "qpb_common.h"
#include "qpb.h"

namespace qpb {
namespace blk {

constexpr int NB = 128;   // padded n
constexpr int MB = 256;   // rows of D
constexpr int NT = 1024;  // threads: four per row (one quad)
constexpr int HW = NB / 4;  // columns per thread
constexpr int XS = 2 * NB + 64;  // exchange area (doubles)
constexpr double kDepTol = 1e-24;

__device__ __forceinline__ double readlane_d(double v, int lane) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const int lo = __builtin_amdgcn_readlane((int)(unsigned)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(unsigned)(b >> 32), lane);
  return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_min64(double v) {
  v = row_min(v);
  const double a = readlane_d(v, 0), b = readlane_d(v, 16), c = readlane_d(v, 32), d = readlane_d(v, 48);
  return __builtin_fmin(__builtin_fmin(a, b), __builtin_fmin(c, d));
}
// min over the workgroup of a key with a 8-bit row index in its low mantissa bits
__device__ __forceinline__ double pack_key256(double v, int idx) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  return __builtin_bit_cast(double, (b & ~255ull) | (unsigned long long)idx);
}
__device__ __forceinline__ int key_index256(double k) { return (int)(__builtin_bit_cast(unsigned long long, k) & 255ull); }

// sum over the quad (the 4 quarters of a row): xor butterfly, bitwise equal
// on the 4 lanes
__device__ __forceinline__ double quad_sum(double v) {
  v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
  v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]
  return v;
}
// lane Q of the quad to all 4
template <int Q>
__device__ __forceinline__ double quad_bcast(double v) {
  return __builtin_amdgcn_mov_dpp(v, Q | (Q << 2) | (Q << 4) | (Q << 6), 0xF, 0xF, true);
}
// row . u: this thread's 32 columns against u[0..32) (its quarter of an LDS
// vector, 16-byte pairs), summed over the quad -- identical on its 4 lanes
__device__ __forceinline__ double dot_lds(const double (&E)[HW], const double *u) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
#pragma unroll
  for (int j = 0; j < HW; j += 4) {
    const double2 v0 = *reinterpret_cast<const double2 *>(&u[j]);
    const double2 v1 = *reinterpret_cast<const double2 *>(&u[j + 2]);
    a0 = __builtin_fma(E[j], v0.x, a0);
    a1 = __builtin_fma(E[j + 1], v0.y, a1);
    a2 = __builtin_fma(E[j + 2], v1.x, a2);
    a3 = __builtin_fma(E[j + 3], v1.y, a3);
  }
  return quad_sum((a0 + a1) + (a2 + a3));
}

// Cholesky of the n x n matrix in M (row-major, stride NB) in place, lower
// triangle = L (true diagonal); returns false if a pivot is <= 0.  Every
// thread updates elements of the trailing matrix.
__device__ bool chol_lds(double *M, double *X, int n, int tid) {
  __shared__ int bad;
  if (tid == 0) bad = 0;
  __syncthreads();
  for (int k = 0; k < n; ++k) {
    const double akk = M[k * NB + k];
    if (!(akk > 0.0)) {
      if (tid == 0) bad = 1;
      __syncthreads();
      return false;
    }
    const double ik = rsq(akk);
    // column k below the diagonal scaled; kept in X for the rank-1 update
    for (int i = k + 1 + tid; i < n; i += NT) {
      const double v = M[i * NB + k] * ik;
      X[i] = v;
    }
    __syncthreads();
    if (tid == 0) M[k * NB + k] = akk * ik;
    for (int i = k + 1 + tid; i < n; i += NT) M[i * NB + k] = X[i];
    // trailing lower triangle (i, j), k < j <= i < n: thread t takes column
    // k + 1 + (t mod 128) and every 8th row from k + 1 + t / 128
    {
      const int j = k + 1 + (tid & (NB - 1));
      if (j < n) {
        const double xj = X[j];
        for (int i = k + 1 + (tid >> 7); i < n; i += NT / NB)
          if (j <= i) M[i * NB + j] = __builtin_fma(-X[i], xj, M[i * NB + j]);
      }
    }
    __syncthreads();
  }
  return bad == 0;
}

__global__ __launch_bounds__(1024, 1) void gi_block_kernel(
    const double *__restrict__ Hg, const double *__restrict__ fg, const double *__restrict__ Ag,
    const double *__restrict__ bg, double *__restrict__ xg, double *__restrict__ lamg, uint32_t *__restrict__ actg,
    int32_t *__restrict__ statg, int32_t *__restrict__ itg, int n, int m, long long batch, int max_iter,
    double feas_tol) {
  __shared__ double Mx[NB * NB];  // H -> L (transposed) -> R -> H -> L
  __shared__ double X[XS];        // exchange area
  __shared__ double Ld[NB];       // 1 / L_kk
  __shared__ int sh_i[8], actv[MB];
  __shared__ double sh_d[24];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int row = tid >> 2, h = tid & 3, c0 = h * HW;
  const long long g = blockIdx.x;
  if (g >= batch) return;  // whole workgroup
  const double *Hq = Hg + g * (long long)n * n;
  const double *Aq = m > 0 ? Ag + g * (long long)m * n : Hq;
  const double *bq = m > 0 ? bg + g * (long long)m : Hq;
  const bool rowok = row < m;

  // ---------------------------------------------------------------- setup
  for (int e = tid; e < NB * NB; e += NT) Mx[e] = 0.0;
  for (int e = tid; e < XS; e += NT) X[e] = 0.0;
  __syncthreads();
  for (int e = tid; e < n * n; e += NT) Mx[(e / n) * NB + e % n] = Hq[e];
  __syncthreads();
  const bool spd = chol_lds(Mx, X, n, tid);
  int status = spd ? QPB_MAX_ITER : QPB_NOT_SPD;
  // rows of A after the factorisation (not live across it)
  const double bl = rowok ? bq[row] : 0.0;
  double E[HW];
  {
    const int ra = rowok ? row : 0;
#pragma unroll
    for (int j = 0; j < HW; ++j) {
      const int c = c0 + j;
      const double a = Aq[ra * n + (c < n ? c : 0)];
      E[j] = (rowok && c < n) ? a : 0.0;
    }
  }
  double na2 = 0.0;  // |a_r|^2 for the normalised slack
  {
    double a = 0.0;
#pragma unroll
    for (int j = 0; j < HW; ++j) a = __builtin_fma(E[j], E[j], a);
    na2 = quad_sum(a);
  }
  const double invn = na2 > 0.0 ? rsq(na2) : 0.0;
  const double thr = (rowok && na2 > 0.0) ? -feas_tol * (1.0 + __builtin_fabs(bl) * invn) : -kInf;

  // L^T into the upper triangle (row k of Mx = column k of L below the
  // diagonal, zeros elsewhere), 1/L_kk into Ld
  __syncthreads();
  for (int e = tid; e < NB * NB; e += NT) {
    const int r = e / NB, c = e % NB;
    if (c > r) Mx[e] = Mx[c * NB + r];
  }
  for (int k = tid; k < NB; k += NT) Ld[k] = k < n ? 1.0 / Mx[k * NB + k] : 0.0;
  __syncthreads();
  for (int e = tid; e < NB * NB; e += NT) {
    const int r = e / NB, c = e % NB;
    if (c <= r) Mx[e] = 0.0;
  }
  __syncthreads();
  // D = A L^{-T}: step k scales column k (held by half k / 64) and updates
  // every column from row k of the transposed L
  if (spd) {
    unroll<NB>([&](auto K) {
      constexpr int k = K, ho = k / HW, kl = k % HW;
      // (steps k >= n are no-ops: 1/L_kk and row k of L^T are zero there)
      __builtin_amdgcn_sched_barrier(0);
      int lo = k * NB + c0;  // opaque per step: keeps this step's LDS reads inside it
      asm volatile("" : "+v"(lo));
      const double e = quad_bcast<ho>(E[kl] * Ld[k]);
      E[kl] = h == ho ? e : E[kl];
#pragma unroll
      for (int j = 0; j < HW; j += 2) {
        const double2 lv = *reinterpret_cast<const double2 *>(&Mx[lo + j]);
        E[j] = __builtin_fma(-lv.x, e, E[j]);
        E[j + 1] = __builtin_fma(-lv.y, e, E[j + 1]);
        pin(E[j]);
        pin(E[j + 1]);
      }
    });
  }
  // y = L^{-1} f on wave 0 (lane i: components i, i + 64) into X[0..n)
  __syncthreads();
  if (wv == 0 && spd) {
    double a0 = lane < n ? fg[g * n + lane] : 0.0, a1 = lane + 64 < n ? fg[g * n + lane + 64] : 0.0;
    for (int k = 0; k < n; ++k) {
      const double yk = (k < 64 ? readlane_d(a0, k) : readlane_d(a1, k - 64)) * Ld[k];
      if (lane == 0) X[k] = yk;
      a0 = __builtin_fma(-Mx[k * NB + lane], yk, a0);        // L[lane][k], zero unless lane > k
      a1 = __builtin_fma(-Mx[k * NB + lane + 64], yk, a1);
    }
  }
  __syncthreads();
  double s = bl + dot_lds(E, X + c0);  // s = b + D y
  double dn;                           // |D_r|^2
  {
    double a = 0.0;
#pragma unroll
    for (int j = 0; j < HW; ++j) a = __builtin_fma(E[j], E[j], a);
    dn = quad_sum(a);
  }
  if (tid == 0) sh_i[0] = 0;
  __syncthreads();
  if (h == 0 && rowok && na2 == 0.0 && bl < -feas_tol * (1.0 + __builtin_fabs(bl))) sh_i[0] = 1;
  __syncthreads();
  bool done = !spd;
  if (spd && sh_i[0]) {
    status = QPB_INFEASIBLE;
    done = true;
  }
  __syncthreads();

  // --------------------------------------------------------- active set
  double *R = Mx;  // column-major NB x NB, zero diagonal
  for (int e = tid; e < NB * NB; e += NT) R[e] = 0.0;
  int q = 0, it = 0, p = 0;
  bool selecting = true, act = false;
  double up = 0.0;
  // wave 0 keeps the active positions: lane i holds positions i and i + 64
  double um0 = 0.0, um1 = 0.0, rdg0 = 0.0, rdg1 = 0.0;
  int iam0 = -1, iam1 = -1;
  __syncthreads();
  while (!done && it < max_iter) {
    ++it;
    if (selecting) {
      const double v = s * invn;
      const double key = wave_min64((h == 0 && !act && v < thr) ? pack_key256(v, row) : kBig);
      if (lane == 0) sh_d[wv] = key;
      __syncthreads();
      double kmin = sh_d[0];
#pragma unroll
      for (int w = 1; w < NT / 64; ++w) kmin = __builtin_fmin(kmin, sh_d[w]);
      __syncthreads();
      if (!(kmin < 0.0)) {
        status = QPB_OK;
        break;
      }
      p = key_index256(kmin);
      up = 0.0;
      selecting = false;
    }
    // row p of D, s_p, |D_p|^2 through X; d2 = D[p, q:] in X[NB..2NB)
    if (row == p) {
#pragma unroll
      for (int j = 0; j < HW; j += 2)
        *reinterpret_cast<double2 *>(&X[c0 + j]) = make_double2(E[j], E[j + 1]);
      if (h == 0) {
        X[2 * NB] = s;
        X[2 * NB + 1] = dn;
      }
    }
    __syncthreads();
    for (int j = tid; j < NB; j += NT) X[NB + j] = j >= q ? X[j] : 0.0;
    const double sp = X[2 * NB], dd = X[2 * NB + 1];
    __syncthreads();
    // wave 0: |d2|^2, r = R^{-1} d1, the ratio test
    if (wv == 0) {
      const double d2a = X[NB + lane], d2b = X[NB + lane + 64];
      double nd2 = row_sum(d2a * d2a + d2b * d2b);
      nd2 = (readlane_d(nd2, 0) + readlane_d(nd2, 16)) + (readlane_d(nd2, 32) + readlane_d(nd2, 48));
      double acc0 = lane < q ? -X[lane] : 0.0, acc1 = lane + 64 < q ? -X[lane + 64] : 0.0;
      const double ir0 = lane < q ? 1.0 / rdg0 : 0.0, ir1 = lane + 64 < q ? 1.0 / rdg1 : 0.0;
      for (int j = q - 1; j >= 0; --j) {
        const double rj = j < 64 ? readlane_d(acc0 * ir0, j) : readlane_d(acc1 * ir1, j - 64);
        acc0 = __builtin_fma(-R[j * NB + lane], rj, acc0);
        acc1 = __builtin_fma(-R[j * NB + lane + 64], rj, acc1);
      }
      const double r0 = acc0 * ir0, r1 = acc1 * ir1;
      double t1 = kBig;
      int k = 0;
      if (q > 0) {
        // the packed keys only pick k; the step is position k's exact ratio
        const double q0 = um0 / r0, q1 = um1 / r1;
        const double k0 = (lane < q && r0 > 0.0) ? pack_key256(q0, lane) : kBig;
        const double k1 = (lane + 64 < q && r1 > 0.0) ? pack_key256(q1, lane + 64) : kBig;
        const double tk = wave_min64(__builtin_fmin(k0, k1));
        k = key_index256(tk);
        const double tx = k < 64 ? readlane_d(q0, k) : readlane_d(q1, k - 64);
        t1 = tk < kBig ? tx : kBig;
      }
      const double t2 = (nd2 > kDepTol * dd) ? -sp / nd2 : kBig;
      const double t = t1 < t2 ? t1 : t2;
      um0 = __builtin_fma(-t, r0, um0);
      um1 = __builtin_fma(-t, r1, um1);
      if (lane == 0) {
        sh_d[16] = t;
        sh_d[17] = t2;
        sh_d[18] = t1;
        sh_d[19] = nd2;
        sh_i[1] = k;
      }
    }
    __syncthreads();
    const double t = sh_d[16], t2 = sh_d[17], t1 = sh_d[18], nd2 = sh_d[19];
    const int kdrop = sh_i[1];
    __syncthreads();
    if (!(t < kBig)) {
      status = QPB_INFEASIBLE;
      break;
    }
    if (t2 < kBig) s = __builtin_fma(t, dot_lds(E, X + NB + c0), s);
    up += t;
    if (t2 <= t1) {
      // ADD p: Householder on columns q.. (v = d2 + alpha e_q, see qpb_gi.hip)
      const double Dpq = X[q];
      const double nrm = sqrt(nd2);
      const double alpha = Dpq <= 0.0 ? -nrm : nrm;
      const double beta = 1.0 / __builtin_fma(alpha, Dpq, nd2);
      __syncthreads();
      if (tid == 0) X[NB + q] = Dpq + alpha;
      if (tid < q) R[q * NB + tid] = -X[tid];  // new column q of R: d1 above the diagonal
      __syncthreads();
      const double w = beta * dot_lds(E, X + NB + c0);
#pragma unroll
      for (int j = 0; j < HW; j += 2) {
        const double2 v = *reinterpret_cast<const double2 *>(&X[NB + c0 + j]);
        E[j] = __builtin_fma(-w, v.x, E[j]);
        E[j + 1] = __builtin_fma(-w, v.y, E[j + 1]);
      }
      if (wv == 0) {
        if (lane == q) {
          rdg0 = alpha;
          iam0 = p;
          um0 = up;
        }
        if (lane + 64 == q) {
          rdg1 = alpha;
          iam1 = p;
          um1 = up;
        }
      }
      if (row == p) act = true;
      ++q;
      selecting = true;
      __syncthreads();
    } else {
      // DROP position kdrop.  The diagonal goes back into R first (old
      // position order), positions kdrop.. move down by one (wave 0), column
      // kdrop is deleted, Givens rotations restore the triangle (the same
      // rotations on D's columns), and the new diagonal is taken out.
      if (wv == 0) {
        if (lane < q) R[lane * NB + lane] = rdg0;
        if (lane + 64 < q) R[(lane + 64) * NB + lane + 64] = rdg1;
        const int c = kdrop < 64 ? __builtin_amdgcn_readlane(iam0, kdrop) : __builtin_amdgcn_readlane(iam1, kdrop - 64);
        if (lane == 0) sh_i[2] = c;
        const double un0 = __shfl(um0, (lane + 1) & 63), un1 = __shfl(um1, (lane + 1) & 63);
        const int in0 = __shfl(iam0, (lane + 1) & 63), in1 = __shfl(iam1, (lane + 1) & 63);
        const double um64 = readlane_d(um1, 0);
        const int iam64 = __builtin_amdgcn_readlane(iam1, 0);
        const int p0 = lane, p1 = lane + 64;
        if (p0 >= kdrop && p0 < q - 1) {
          um0 = lane == 63 ? um64 : un0;
          iam0 = lane == 63 ? iam64 : in0;
        } else if (p0 == q - 1) {
          um0 = 0.0;
          iam0 = -1;
        }
        if (p1 >= kdrop && p1 < q - 1) {
          um1 = un1;
          iam1 = in1;
        } else if (p1 == q - 1) {
          um1 = 0.0;
          iam1 = -1;
        }
      }
      __syncthreads();
      if (row == sh_i[2]) act = false;
      // column l <- column l + 1 for kdrop <= l < q - 1 (ascending; rows in parallel)
      for (int l = kdrop; l < q - 1; ++l) {
        if (tid < q) R[l * NB + tid] = R[(l + 1) * NB + tid];
        __syncthreads();
      }
      if (tid < NB) R[(q - 1) * NB + tid] = 0.0;
      __syncthreads();
      for (int j = kdrop; j < q - 1; ++j) {
        const double a = R[j * NB + j], bb = R[j * NB + j + 1];
        const double ir = rsq(__builtin_fma(a, a, bb * bb));
        const double cj = a * ir, sj = bb * ir;
        const int l = tid;  // column
        double rj = 0.0, rj1 = 0.0;
        if (l >= j && l < q - 1) {
          rj = R[l * NB + j];
          rj1 = R[l * NB + j + 1];
        }
        __syncthreads();
        if (l >= j && l < q - 1) {
          R[l * NB + j] = __builtin_fma(cj, rj, sj * rj1);
          R[l * NB + j + 1] = (l == j) ? 0.0 : __builtin_fma(-sj, rj, cj * rj1);
        }
        // the same rotation on columns j, j+1 of every D row
        if (j % HW == HW - 1) {  // the pair straddles quarters j / 32 and j / 32 + 1
          const int hq = j / HW;
          const double next0 = __shfl_down(E[0], 1), prev31 = __shfl_up(E[HW - 1], 1);
          if (h == hq) E[HW - 1] = __builtin_fma(cj, E[HW - 1], sj * next0);
          if (h == hq + 1) E[0] = __builtin_fma(-sj, prev31, cj * E[0]);
        } else {
          // branch-free: the rotation at this quarter's local pair, identity
          // (exactly) at the others
          const int jj = j - c0;
          unroll<HW - 1>([&](auto JJ) {
            constexpr int jl = JJ;
            const bool hit = jj == jl;
            const double cm = hit ? cj : 1.0, sm = hit ? sj : 0.0;
            const double e0 = E[jl], e1 = E[jl + 1];
            E[jl] = __builtin_fma(cm, e0, sm * e1);
            E[jl + 1] = __builtin_fma(-sm, e0, cm * e1);
          });
        }
        __syncthreads();
      }
      if (tid < NB) R[tid * NB + q - 1] = 0.0;  // row q - 1
      --q;
      __syncthreads();
      if (wv == 0) {
        rdg0 = lane < q ? R[lane * NB + lane] : 0.0;
        rdg1 = lane + 64 < q ? R[(lane + 64) * NB + lane + 64] : 0.0;
      }
      __syncthreads();
      if (tid < q) R[tid * NB + tid] = 0.0;
      __syncthreads();
    }
  }

  // ------------------------------------------------------------- outputs
  __syncthreads();
  for (int j = tid; j < XS; j += NT) X[j] = 0.0;
  if (h == 0) actv[row] = act ? 1 : 0;
  __syncthreads();
  if (wv == 0) {
    if (lane < q && iam0 >= 0) X[iam0] = um0;
    if (lane + 64 < q && iam1 >= 0) X[iam1] = um1;
  }
  __syncthreads();
  if (h == 0 && rowok) lamg[g * m + row] = X[row];
  const int words = (m + 31) / 32;
  if (tid < words && m > 0) {
    uint32_t wbits = 0;
    for (int b = 0; b < 32; ++b) wbits |= (uint32_t)(actv[32 * tid + b] & 1) << b;
    actg[g * words + tid] = wbits;
  }
  // g = f + A^T lam (thread i < n: component i); L from H again
  double gi = 0.0;
  if (tid < n) {
    gi = fg[g * n + tid];
    for (int r = 0; r < m; ++r) {
      const double u = X[r];
      if (u != 0.0) gi = __builtin_fma(u, Aq[r * n + tid], gi);
    }
  }
  __syncthreads();
  for (int e = tid; e < n * n; e += NT) Mx[(e / n) * NB + e % n] = Hq[e];
  double *Y = X + NB;  // g, outside the Cholesky's scratch X[0..n)
  if (tid < n) Y[tid] = gi;
  __syncthreads();
  chol_lds(Mx, X, n, tid);  // succeeded before: same input, same arithmetic
  __syncthreads();
  // forward L y = g and backward L^T x = -y on wave 0 (L row-major lower)
  if (wv == 0 && spd) {
    double a0 = lane < n ? Y[lane] : 0.0, a1 = lane + 64 < n ? Y[lane + 64] : 0.0;
    for (int k = 0; k < n; ++k) {
      const double yk = (k < 64 ? readlane_d(a0, k) : readlane_d(a1, k - 64)) / Mx[k * NB + k];
      if (k < 64 && lane == k) a0 = yk;
      if (k >= 64 && lane == k - 64) a1 = yk;
      if (lane > k) a0 = __builtin_fma(-Mx[lane * NB + k], yk, a0);
      if (lane + 64 > k && lane + 64 < n) a1 = __builtin_fma(-Mx[(lane + 64) * NB + k], yk, a1);
    }
    for (int k = n - 1; k >= 0; --k) {
      const double xk = (k < 64 ? readlane_d(a0, k) : readlane_d(a1, k - 64)) / Mx[k * NB + k];
      if (k < 64 && lane == k) a0 = xk;
      if (k >= 64 && lane == k - 64) a1 = xk;
      if (lane < k) a0 = __builtin_fma(-Mx[k * NB + lane], xk, a0);
      if (lane + 64 < k) a1 = __builtin_fma(-Mx[k * NB + lane + 64], xk, a1);
    }
    const double x0 = -a0, x1 = -a1;
    const bool bad = (lane < n && !(__builtin_fabs(x0) < kInf)) || (lane + 64 < n && !(__builtin_fabs(x1) < kInf));
    if (lane < n) xg[g * n + lane] = x0;
    if (lane + 64 < n) xg[g * n + lane + 64] = x1;
    if (status == QPB_OK && __ballot(bad) != 0) status = QPB_NUMERICAL;
    if (lane == 0) {
      statg[g] = status;
      if (itg) itg[g] = it;
    }
  } else if (tid == 0) {
    statg[g] = status;
    if (itg) itg[g] = it;
  }
}

}  // namespace blk
}  // namespace qpb

extern "C" hipError_t qpb_launch_gi_block(const qpb_desc *d, const double *H, const double *f, const double *A,
                                          const double *b, double *x, double *lam, uint32_t *active,
                                          int32_t *status, int32_t *iters, hipStream_t stream) {
  const int max_iter = d->max_iter > 0 ? d->max_iter : 4 * (d->n + d->m) + 8;
  const double tol = d->feas_tol > 0 ? d->feas_tol : 1e-10;
  hipLaunchKernelGGL(qpb::blk::gi_block_kernel, dim3((unsigned)d->batch), dim3(qpb::blk::NT), 0, stream, H, f, A, b,
                     x, lam, active, status, iters, d->n, d->m, (long long)d->batch, max_iter, tol);
  return hipGetLastError();
}
