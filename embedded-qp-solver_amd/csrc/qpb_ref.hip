// qpb_ref.hip -- reference-semantics kernels and the
// batched quadratic-form evaluation (qp.c:9-27).
//
// Batched GPU replicas of the reference solvers, operation for operation:
//   newton_method_with_line_search   qp_solvers.c:103-144
//   admm                             qp_solvers.c:255-319 (rho = 1, alpha = 1,
//                                    returns x, x0 ignored)
//   gradient_descent_with_line_search qp_solvers.c:65-101
// with the explicit inverse of matrix_invert (partial-pivot LU, matrix_ops.c:
// 487-536, per-column forward/back substitution :594-625), the Armijo test's
// f(x + 2 alpha d) quirk (qp_solvers.c:21-35 called from :50-56), matrix_norm's
// sequential sum of squares (:632-656) and matrix_mult's sequential k-sums
// (:235-271).  This file is compiled with -ffp-contract=off: the reference
// (gcc -O2, x86-64, no FMA) rounds every product and every sum, and so do
// these kernels, in the same order.
//
// Layout: thread i owns row i.
//   n <= 64: one QP per 64-thread workgroup; P, the LU / inverse and two n x n
//   scratch matrices for the per-column solves (thread t keeps its column's
//   vectors in column t: conflict-free) and the n-vectors in LDS.
//   64 < n <= 128 (the reference's N_DIM is any compile-time size; SURVEY §6
//   times refC at n = 128): 128-thread workgroups walking the batch, as many
//   per CU as their LDS allows (one at n = 128), each with ONE n x n matrix X
//   in LDS at column stride ld = n | 1 (odd: walks along a row and along a
//   column across the threads are both conflict-free).  X holds in turn the
//   matrix being factorised (the LU in place), the per-column solves' W and
//   then V (in place: V[nn] overwrites W[nn] once it is read), and P for the
//   solver's loop.  The LU factors and, for Newton, the inverse (row
//   products, coalesced) go to a 2 n^2 slice per workgroup in global memory,
//   which stays in L2; the solves stage LU row nn into an LDS row buffer (one
//   element per thread, loaded a step ahead), read there by every thread at
//   the same address.  Every sequential sum and the LU's row update run in
//   RC-aligned chunks, loads ahead of the arithmetic, with no branch inside a
//   chunk (X has ref_npad(n) columns so a chunk never leaves it).  Rounds 3-4
//   kept all four matrices in a global slice with 8 workgroups per CU: one
//   dependent memory round trip per multiply-add, 128-156 ms for configs[3]'s
//   Newton replicas (74 ms now).
//   128 < n <= 1024 (round 6: the compat layer's N_DIM above 128, SURVEY's
//   16-bit dimension fields): 1024-thread workgroups, one thread per row as
//   for n <= 64, the four matrices (P, the LU, W, V) in a 4 n^2 slice of global
//   memory per workgroup and only the n-vectors in LDS; the pivot search
//   reduces over the sixteen wavefronts through LDS.  The n <= 64 code runs
//   unchanged on those addresses.
// The arithmetic is the same code in the same order in every layout: only the
// addresses, and the grouping of loads ahead of the stores, change.
#include "qpb_common.h"
#include "qpb.h"

namespace qpb {

constexpr int REF_MAXN = 1024;
constexpr int REF_LDS_MAXN = 64;  // n above this: the one-matrix layout (X) below
constexpr int REF_BIG_MAXN = 128;  // n above this: the global layout below
constexpr int REF_BIG_NT = 128;
constexpr int REF_HUGE_NT = 1024;  // 128 < n <= 1024: one thread per row, the matrices in global memory
constexpr int REF_HUGE_WS_MATS = 4;  // P, the LU, W, V per workgroup
constexpr int REF_WS_MATS = 2;  // big layout, per workgroup: the LU factors (row-major), V (column-major)
constexpr int REF_MAX_WG_PER_CU = 8;
__host__ __device__ constexpr int ref_ld(int n) { return n | 1; }
// the big layout's X has ref_npad(n) columns (rows of W / V): every RC-chunk
// of a row or column stays inside it
__host__ __device__ constexpr int ref_npad(int n) { return (n + 15) & ~15; }

// an n x n matrix in any layout: element (r, c) at p[r * rs + c * cs]
struct Mat {
  double *p;
  int rs, cs;
  __device__ __forceinline__ double &operator()(int r, int c) const { return p[r * rs + c * cs]; }
};

struct RefShared {
  Mat P, V;            // the solver's P and the inverse (layout depends on the path)
  double *M, *W, *Vr;  // n <= 64: LU, W, V row-major in LDS
  double *X, *Mg;      // n > 64: the LDS matrix, the global LU copy
  double *rowbuf;      // n > 64: two staged LU rows (2 npad); the LU's dummy store slots
  int ld;
  double *x, *g, *d, *t0, *t1, *t2;  // n each
  double *scal;                       // scalars broadcast by thread 0
  double *red;                        // cross-wave reduction slots (2)
  int *perm, *redi;
};

// The sequential sums below keep the reference's order (k ascending, one
// rounding per product and per sum); their operands are loaded RC at a time
// ahead of the arithmetic (one memory latency per RC terms, not per term).
constexpr int RC = 16;

// prod_i = sum_k A(i, k) * v[k], k ascending (matrix_mult, matrix_ops.c:262-270)
__device__ __forceinline__ double row_dot(const Mat &A, const double *v, int i, int n) {
  double acc = 0.0;
  int k = 0;
  for (; k + RC <= n; k += RC) {
    double a[RC], b[RC];
#pragma unroll
    for (int u = 0; u < RC; ++u) {
      a[u] = A(i, k + u);
      b[u] = v[k + u];
    }
#pragma unroll
    for (int u = 0; u < RC; ++u) acc += a[u] * b[u];
  }
  for (; k < n; ++k) acc += A(i, k) * v[k];
  return acc;
}

// matrix_scalar_prod (matrix_ops.c:295-297): sequential
__device__ __forceinline__ double seq_dot(const double *a, const double *b, int n) {
  double acc = 0.0;
  int k = 0;
  for (; k + RC <= n; k += RC) {
    double x[RC], y[RC];
#pragma unroll
    for (int u = 0; u < RC; ++u) {
      x[u] = a[k + u];
      y[u] = b[k + u];
    }
#pragma unroll
    for (int u = 0; u < RC; ++u) acc += x[u] * y[u];
  }
  for (; k < n; ++k) acc += a[k] * b[k];
  return acc;
}

// matrix_norm (matrix_ops.c:647-655)
__device__ __forceinline__ double seq_norm(const double *a, int n) {
  double acc = 0.0;
  int k = 0;
  for (; k + RC <= n; k += RC) {
    double x[RC];
#pragma unroll
    for (int u = 0; u < RC; ++u) x[u] = a[k + u];
#pragma unroll
    for (int u = 0; u < RC; ++u) {
      double t = x[u];
      t *= t;
      acc += t;
    }
  }
  for (; k < n; ++k) {
    double t = a[k];
    t *= t;
    acc += t;
  }
  return __builtin_sqrt(acc);
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, lane);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), lane);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// matrix_lup_decompose (matrix_ops.c:487-536) in place on M, the permutation
// in S.perm.  NT threads (64: one wavefront; 128: two, reduced through LDS);
// thread i updates row i.
template <int NT>
__device__ void ref_lu(RefShared &S, const Mat &M, int n) {
  const int tid = threadIdx.x;
  if (tid < n) S.perm[tid] = tid;
  __syncthreads();
  for (int k = 0; k + 1 < n; ++k) {  // :507
    // matrix_lup_pivot :449-470: the first row attaining the largest |M[i][k]|
    // (a strict `>` scan from piv = 0), found by an exact max over the
    // workgroup and the lowest thread holding it
    double v = 0.0;
    if (tid >= k && tid < n) {
      v = M(tid, k);
      v = v < 0 ? -v : v;
    }
    double piv;
    int pidx;
    if constexpr (NT > 64) {
      // the wave's max (fmin of -v over the DPP rows, then the four rows:
      // fmin / fmax drop a NaN as the strict `>` scan skips it), its lowest
      // thread at the max, then the waves' pairs through LDS with ONE
      // barrier (lower waves win ties: lower rows; a NaN wave max loses)
      double m = -row_min(-v);
      m = __builtin_fmax(__builtin_fmax(readlane_d(m, 0), readlane_d(m, 16)),
                         __builtin_fmax(readlane_d(m, 32), readlane_d(m, 48)));
      const unsigned long long hit = __ballot(tid >= k && tid < n && v == m);
      const int w = tid >> 6;
      if ((tid & 63) == 0) {
        S.red[w] = m;
        S.redi[w] = hit ? (tid & ~63) + __builtin_ctzll(hit) : 1 << 30;
      }
      __syncthreads();
      piv = S.red[0];
      pidx = S.redi[0];
#pragma unroll
      for (int w2 = 1; w2 < NT / 64; ++w2) {
        const double mw = S.red[w2];
        if (mw > piv || piv != piv) {
          pidx = S.redi[w2];
          piv = __builtin_fmax(piv, mw);
        }
      }
    } else {
      piv = v;
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) piv = __builtin_fmax(piv, __shfl_xor(piv, off));
      const unsigned long long hit = __ballot(tid >= k && tid < n && v == piv);
      pidx = __builtin_ctzll(hit);
    }
    if (!(piv > 0.0)) break;  // singular: the reference prints and returns (:511-515)
    if (tid == 0) {  // permutation_swap :434-447
      const int tmp = S.perm[pidx];
      S.perm[pidx] = S.perm[k];
      S.perm[k] = tmp;
    }
    if (tid < n) {  // matrix_row_permute :472-485 (thread tid swaps column tid)
      const double a = M(pidx, tid), b = M(k, tid);
      M(pidx, tid) = b;
      M(k, tid) = a;
    }
    __syncthreads();
    if (tid > k && tid < n) {  // :523-533
      const int i = tid;
      double tmp = M(i, k);
      tmp /= M(k, k);
      M(i, k) = tmp;
      // the row's update RC entries at a time: their loads first, then the
      // arithmetic and the stores (one LDS latency per RC entries)
      if constexpr (NT == REF_BIG_NT) {
        // the big layout: RC-aligned chunks over the padded columns, no
        // branch anywhere (a branch per guarded load made every join wait
        // for all outstanding LDS reads): entries j <= k and j >= n are
        // computed and stored to this thread's dummy slot
        const int npad = ref_npad(n);
        double *dummy = S.rowbuf + tid;
        for (int j0 = (k + 1) & ~(RC - 1); j0 < npad; j0 += RC) {
          double a[RC], b[RC];
#pragma unroll
          for (int u = 0; u < RC; ++u) {
            a[u] = M(i, j0 + u);
            b[u] = M(k, j0 + u);
          }
#pragma unroll
          for (int u = 0; u < RC; ++u) {
            double t = a[u];
            t -= tmp * b[u];
            const int j = j0 + u;
            *((j > k && j < n) ? &M(i, j) : dummy) = t;
          }
        }
      } else
      for (int j0 = k + 1; j0 < n; j0 += RC) {
        double a[RC], b[RC];
#pragma unroll
        for (int u = 0; u < RC; ++u)
          if (j0 + u < n) {
            a[u] = M(i, j0 + u);
            b[u] = M(k, j0 + u);
          }
#pragma unroll
        for (int u = 0; u < RC; ++u)
          if (j0 + u < n) {
            double t = a[u];
            t -= tmp * b[u];
            M(i, j0 + u) = t;
          }
      }
    }
    // the big layout: the next step's pivot search reads only the thread's
    // own row, and its barrier comes before anything reads another thread's row
    if constexpr (NT != REF_BIG_NT) __syncthreads();
  }
  if constexpr (NT == REF_BIG_NT) __syncthreads();
}

// In-place explicit inverse (matrix_invert, matrix_ops.c:551-630), n <= 64
// (NT = 64, LDS) or 128 < n <= 1024 (NT = 1024, global): S.M -> S.Vr.
// Thread i: row i in the LU, column i in the solves.
template <int NT>
__device__ void ref_invert_small(RefShared &S, int n) {
  const Mat M{S.M, n, 1};
  ref_lu<NT>(S, M, n);
  // per-column solves (:594-619): thread i solves for column i; its w/v
  // vectors are column i of W/V, so V ends up as the inverse (:621-625)
  const int tid = threadIdx.x;
  if (tid < n) {
    const int i = tid;
    for (int nn = 0; nn < n; ++nn) {
      double t = 0.0;
      for (int k = 0; k + 1 <= nn; ++k) t += M(nn, k) * S.W[k * n + i];
      const double e = (S.perm[nn] == i) ? 1.0 : 0.0;
      S.W[nn * n + i] = e - t;
    }
    for (int nn = n - 1; nn >= 0; --nn) {
      double t = 0.0;
      for (int k = nn + 1; k < n; ++k) t += M(nn, k) * S.Vr[k * n + i];
      S.Vr[nn * n + i] = (S.W[nn * n + i] - t) / M(nn, nn);
    }
  }
  __syncthreads();
  S.V = Mat{S.Vr, n, 1};
}

// The same for 64 < n <= 128: the matrix in X (column-major, stride ld) on
// entry; the LU factors go to S.Mg (row-major) and the inverse ends in X
// row-major (S.V = X with row stride ld).
__device__ void ref_invert_big(RefShared &S, int n) {
  const int tid = threadIdx.x;
  const int ld = S.ld;
  ref_lu<REF_BIG_NT>(S, Mat{S.X, 1, ld}, n);
  for (int e = tid; e < n * n; e += REF_BIG_NT) {
    const int r = e / n, c = e - r * n;
    S.Mg[e] = S.X[c * ld + r];
  }
  __syncthreads();
  // per-column solves (:594-619), thread i on column i of W, then of V in its
  // place: entry nn of the column at X[nn * ld + i] (contiguous across the
  // threads).  Row nn of the LU is staged from the global copy into an LDS
  // row buffer (double-buffered, one element per thread, loaded a step ahead)
  // and read there by every thread at the same address.
  double *rb0 = S.rowbuf, *rb1 = S.rowbuf + ref_npad(n);
  double *col = S.X + tid;
  const double *Mg = S.Mg;
  double pre = tid < n ? Mg[tid] : 0.0;  // row 0
  for (int nn = 0; nn < n; ++nn) {
    double *buf = (nn & 1) ? rb1 : rb0;
    if (tid < n) buf[tid] = pre;
    if (nn + 1 < n && tid < n) pre = Mg[(nn + 1) * n + tid];
    __syncthreads();
    if (tid < n) {
      // RC terms per step, all loaded ahead; the last, partial chunk adds
      // its terms k < nn by a select (no branch per term)
      double t = 0.0;
      for (int k0 = 0; k0 < nn; k0 += RC) {
        double mv[RC], wv[RC];
#pragma unroll
        for (int u = 0; u < RC; ++u) {
          mv[u] = buf[k0 + u];
          wv[u] = col[(k0 + u) * ld];
        }
        if (k0 + RC <= nn) {
#pragma unroll
          for (int u = 0; u < RC; ++u) t += mv[u] * wv[u];
        } else {
#pragma unroll
          for (int u = 0; u < RC; ++u) {
            const double tn = t + mv[u] * wv[u];
            t = (k0 + u < nn) ? tn : t;
          }
        }
      }
      const double e = (S.perm[nn] == tid) ? 1.0 : 0.0;
      col[nn * ld] = e - t;
    }
  }
  pre = tid < n ? Mg[(n - 1) * n + tid] : 0.0;
  __syncthreads();  // the last forward step's readers are done with its buffer
  for (int nn = n - 1; nn >= 0; --nn) {
    double *buf = (nn & 1) ? rb1 : rb0;
    if (tid < n) buf[tid] = pre;
    if (nn > 0 && tid < n) pre = Mg[(nn - 1) * n + tid];
    __syncthreads();
    if (tid < n) {
      // terms k = nn + 1 .. n - 1 in RC-aligned chunks; the first and the
      // last chunk select their terms
      double t = 0.0;
      for (int k0 = (nn + 1) & ~(RC - 1); k0 < n; k0 += RC) {
        double mv[RC], vv[RC];
#pragma unroll
        for (int u = 0; u < RC; ++u) {
          mv[u] = buf[k0 + u];
          vv[u] = col[(k0 + u) * ld];
        }
        if (k0 > nn && k0 + RC <= n) {
#pragma unroll
          for (int u = 0; u < RC; ++u) t += mv[u] * vv[u];
        } else {
#pragma unroll
          for (int u = 0; u < RC; ++u) {
            const double tn = t + mv[u] * vv[u];
            t = (k0 + u > nn && k0 + u < n) ? tn : t;
          }
        }
      }
      col[nn * ld] = (col[nn * ld] - t) / buf[nn];
    }
  }
  __syncthreads();
  S.V = Mat{S.X, ld, 1};
}

// f(x) = 1/2 x^T (P x) + q^T x + r (quadratic_form_eval, qp.c:9-27); xv in LDS;
// uses S.t2 as the P x temporary; result broadcast in S.scal[slot].
// The two sequential dots run on threads 0 and 1 at once (each in the
// reference's order), then thread 0 combines them as the reference does.
// `extra` (>= 0): thread 2 also computes fx + C2 * (t0 . t1) into scal[extra]
// (the Armijo right-hand side, independent of f(x)).
template <int NT>
__device__ double ref_eval(RefShared &S, const double *q, const double *xv, int n, int slot, int extra = -1,
                           double fx = 0.0) {
  const int tid = threadIdx.x;
  if (tid < n) S.t2[tid] = row_dot(S.P, xv, tid, n);
  __syncthreads();
  if (tid == 0) S.scal[4] = seq_dot(xv, S.t2, n);
  else if (tid == 1) S.scal[5] = seq_dot(q, xv, n);
  else if (tid == 2 && extra >= 0) S.scal[extra] = fx + 1e-4 * seq_dot(S.t0, S.t1, n);  // C2 (qp_solvers.c:9)
  __syncthreads();
  if (tid == 0) {
    double a = 0.5 * S.scal[4];
    a += S.scal[5];
    a += 0.0;  // r = 0 in every reference call path (main.c:12)
    S.scal[slot] = a;
  }
  __syncthreads();
  return S.scal[slot];
}

// grad f(x) = P x + q into out (quadratic_form_eval_grad, qp.c:29-44)
template <int NT>
__device__ void ref_grad(RefShared &S, const double *q, const double *xv, double *out, int n) {
  const int tid = threadIdx.x;
  if (tid < n) {
    const double px = row_dot(S.P, xv, tid, n);
    out[tid] = px + q[tid];
  }
  __syncthreads();
}

// line_search + armijo (qp_solvers.c:21-63); d in S.d, x in S.x; returns alpha
template <int NT>
__device__ double ref_line_search(RefShared &S, const double *q, int n) {
  const int tid = threadIdx.x;
  const double C1 = 0.9;  // C2 = 1e-4 (qp_solvers.c:9) is applied in ref_eval
  const double fx = ref_eval<NT>(S, q, S.x, n, 1);
  ref_grad<NT>(S, q, S.x, S.t0, n);  // grad_fx
  double alpha = 1.0;            // ALPHA0_* (:11-12)
  // The reference loop has no trial cap (:51); alpha *= 0.9 reaches 0 (and
  // then the Armijo test holds) after ~7000 trials for finite data.  The cap
  // only stops non-finite data from spinning the GPU forever.
  for (int trial = 0; trial < 20000; ++trial) {
    if (tid < n) {
      const double da = alpha * S.d[tid];  // d_alpha = copy(d); scalar_mult(alpha)
      S.t1[tid] = da;
    }
    __syncthreads();
    if (tid < n) S.g[tid] = (S.x[tid] + S.t1[tid]) + S.t1[tid];  // lhs_arg = xk + d_alpha, xk = x + d_alpha
    __syncthreads();
    const double lhs = ref_eval<NT>(S, q, S.g, n, 2, 3, fx);  // and rhs = fx + C2 (grad . d_alpha) in scal[3]
    const double rhs = S.scal[3];
    if (lhs <= rhs) break;
    alpha *= C1;
  }
  return alpha;
}

// LDS (and workspace) carving shared by the solver and the invert kernels.
// n <= 64: [P n^2 (solver only)] [M W V 3 n^2] in `sm`.  n > 64: [X n ld] in
// `sm`, the LU copy and V in the workgroup's 2 n^2 slice of `ws`.  The
// n-vectors, scalars and ints follow.
template <int NT>
__device__ __forceinline__ void ref_carve(RefShared &S, double *sm, double *ws, int n, bool with_p) {
  const int nn2 = n * n;
  double *cur = sm;
  if constexpr (NT == REF_BIG_NT) {
    S.ld = ref_ld(n);
    S.X = cur;
    cur += ref_npad(n) * S.ld;
    S.rowbuf = cur;
    cur += 2 * ref_npad(n);
    S.Mg = ws + (size_t)blockIdx.x * REF_WS_MATS * nn2;
    S.P = Mat{S.X, 1, S.ld};  // where P is loaded (column-major)
  } else if constexpr (NT == REF_HUGE_NT) {
    // the n <= 64 layout's matrices in the workgroup's global slice
    double *gm = ws + (size_t)blockIdx.x * REF_HUGE_WS_MATS * nn2;
    S.ld = n;
    S.P = Mat{gm, n, 1};
    S.M = gm + nn2;
    S.W = gm + 2 * nn2;
    S.Vr = gm + 3 * nn2;
  } else {
    S.ld = n;
    if (with_p) {
      S.P = Mat{cur, n, 1};
      cur += nn2;
    }
    S.M = cur;
    S.W = cur + nn2;
    S.Vr = cur + 2 * nn2;
    cur += 3 * nn2;
  }
  // n-vectors packed at stride n: the LDS per QP sets the occupancy
  // (n = 16: 9.6 KB, 16 workgroups per CU)
  S.x = cur;
  S.g = S.x + n;
  S.d = S.g + n;
  S.t0 = S.d + n;
  S.t1 = S.t0 + n;
  S.t2 = S.t1 + n;
  S.scal = S.t2 + 4 * n;  // q, u, z sit between t2 and the scalars
  S.red = S.scal + 8;
  S.perm = reinterpret_cast<int *>(S.red + (NT / 64 > 2 ? NT / 64 : 2));  // one reduction slot per wave
  S.redi = S.perm + n;
}

// the matrix the invert starts from: P (+ rho on the diagonal for ADMM),
// row-major in LDS (n <= 64) or column-major in X
template <int NT>
__device__ __forceinline__ void ref_load_m(RefShared &S, const double *Pq, int n, double diag) {
  const int tid = threadIdx.x;
  const int nn2 = n * n;
  if constexpr (NT == REF_BIG_NT) {
    for (int e = tid; e < nn2; e += NT) {
      const int r = e / n, c = e - r * n;
      S.X[c * S.ld + r] = Pq[e];
    }
  } else {
    for (int e = tid; e < nn2; e += NT) S.M[e] = S.P.p[e];
  }
  __syncthreads();
  if (diag != 0.0) {  // R = P + rho I (qp_solvers.c:285-291)
    double *mii = NT == REF_BIG_NT ? &S.X[tid * S.ld + tid] : &S.M[tid * n + tid];
    if (tid < n) *mii = *mii + diag;
    __syncthreads();
  }
}

// One QP of the reference solvers (thread i owns row i)
template <int NT>
__device__ void ref_solve_one(double *sm, double *ws, int mode, int n, long long g, int iterations, double box_min,
                              double box_max, const double *__restrict__ Pg, const double *__restrict__ qg,
                              const double *__restrict__ x0g, double *__restrict__ xg, int32_t *__restrict__ itg) {
  const int tid = threadIdx.x;
  RefShared S;
  const int nn2 = n * n;
  ref_carve<NT>(S, sm, ws, n, true);
  double *q = S.t2 + n;
  double *u = q + n;
  double *z = u + n;
  const double *Pq = Pg + g * (long long)nn2;
  // P row-major (n <= 64: LDS; n > 128: global); for 64 < n <= 128 it is loaded after the invert
  if constexpr (NT != REF_BIG_NT) {
    for (int e = tid; e < nn2; e += NT) S.P.p[e] = Pq[e];
  }
  if (tid < n) {
    q[tid] = qg[g * n + tid];
    S.x[tid] = (mode != QPB_REF_ADMM) ? x0g[g * n + tid] : 0.0;
  }
  __syncthreads();
  int it = 0;

  if (mode == QPB_REF_NEWTON || mode == QPB_REF_GD) {
    const double MIN_GRAD = 1e-1;  // MIN_GRAD_GRAD / MIN_GRAD_NEWTON (:14-15)
    if (mode == QPB_REF_NEWTON) {  // hessian_inv = invert(copy(P)) (:115-117)
      ref_load_m<NT>(S, Pq, n, 0.0);
      if constexpr (NT == REF_BIG_NT) {
        ref_invert_big(S, n);
        // V to the global slice (column-major: coalesced row products), P into X
        double *Vg = S.Mg + nn2;
        for (int e = tid; e < nn2; e += NT) {
          const int c = e / n, r = e - c * n;
          Vg[e] = S.X[r * S.ld + c];
        }
        __syncthreads();
        S.V = Mat{Vg, 1, n};
      } else {
        ref_invert_small<NT>(S, n);
      }
    }
    if constexpr (NT == REF_BIG_NT) {
      for (int e = tid; e < nn2; e += NT) {
        const int r = e / n, c = e - r * n;
        S.X[c * S.ld + r] = Pq[e];
      }
      S.P = Mat{S.X, 1, S.ld};
      __syncthreads();
    }
    for (; it < iterations; ++it) {
      ref_grad<NT>(S, q, S.x, S.g, n);
      if (tid == 0) S.scal[0] = seq_norm(S.g, n);
      __syncthreads();
      if (MIN_GRAD > S.scal[0]) break;  // :83 / :125
      if (tid < n) {
        double dv = (mode == QPB_REF_NEWTON) ? row_dot(S.V, S.g, tid, n) : S.g[tid];  // matrix_mult / copy
        dv = -1.0 * dv;                                                               // scalar_mult(d, -1)
        S.d[tid] = dv;
      }
      __syncthreads();
      const double alpha = ref_line_search<NT>(S, q, n);
      if (tid < n) {
        const double da = alpha * S.d[tid];  // scalar_mult(d, alpha)
        S.x[tid] = S.x[tid] + da;            // matrix_add(x, x, d)
      }
      __syncthreads();
    }
  } else {  // ADMM (:255-319)
    const double rho = 1.0, alpha = 1.0, abstol = 1e-4, restol = 1e-2;
    if (tid < n) {
      z[tid] = 0.0;
      u[tid] = 0.0;
    }
    ref_load_m<NT>(S, Pq, n, rho);  // R = P + rho I (:285-291)
    if constexpr (NT == REF_BIG_NT)
      ref_invert_big(S, n);  // R^{-1} in X (:292)
    else
      ref_invert_small<NT>(S, n);
    const double sq = __builtin_sqrt((double)n);
    // admm_update_x's right-hand side rho (z - u) - q (:146-159) is each
    // thread's own entry, so it is formed at the end of the previous
    // iteration, into the other half of a double buffer (t1 / t2: the current
    // one is still being read by every thread's row product)
    if (tid < n) {
      double y1 = z[tid] - u[tid];
      y1 = rho * y1;
      y1 = y1 - q[tid];
      S.t1[tid] = y1;
    }
    __syncthreads();
    for (; it < iterations; ++it) {
      double *ycur = (it & 1) ? S.t2 : S.t1, *ynext = (it & 1) ? S.t1 : S.t2;
      if (tid < n) {
        const double zold = z[tid];
        const double xv = row_dot(S.V, ycur, tid, n);
        S.x[tid] = xv;
        double xh = alpha * xv;  // admm_update_x_hat (:161-174)
        const double tz = (1.0 - alpha) * zold;
        xh = xh + tz;
        double tt = xh + u[tid];  // admm_update_z (:176-190): max with lb, then min with ub
        tt = tt > box_min ? tt : box_min;
        const double zn = tt > box_max ? box_max : tt;
        z[tid] = zn;
        const double du = xh - zn;  // admm_update_u (:192-203)
        const double un = u[tid] + du;
        u[tid] = un;
        S.g[tid] = xv - zn;  // for admm_r_norm
        double ds = zn - zold;
        ds = -rho * ds;  // admm_s_norm (:219-231)
        S.d[tid] = ds;
        double y1 = zn - un;  // the next iteration's admm_update_x right-hand side
        y1 = rho * y1;
        y1 = y1 - q[tid];
        ynext[tid] = y1;
      }
      __syncthreads();
      // the five norms (each the reference's sequential sum) on five threads at once
      if (tid < 5) {
        const double *v = tid == 0 ? S.g : tid == 1 ? S.d : tid == 2 ? S.x : tid == 3 ? z : u;
        S.scal[2 + tid] = seq_norm(v, n);
      }
      __syncthreads();
      // the stopping test, evaluated identically by every thread (:233-253)
      const double r_norm = S.scal[2], s_norm = S.scal[3];
      const double norm_x = S.scal[4], norm_z = S.scal[5];
      const double norm_max = norm_x > norm_z ? norm_x : norm_z;
      const double eps_pri = sq * abstol + restol * norm_max;
      const double norm_u = S.scal[6];
      const double eps_dual = sq * abstol + restol * rho * norm_u;
      if (r_norm < eps_pri && s_norm < eps_dual) {
        ++it;
        break;
      }
    }
  }
  if (tid < n) xg[g * n + tid] = S.x[tid];
  if (tid == 0 && itg) itg[g] = it;
}

// NT = 64: one workgroup per QP, everything in LDS.  NT = 128: the big
// layout (X in LDS, the LU and V in the workgroup's slice of `ws`); the grid
// walks the batch.
template <int NT>
__global__ __launch_bounds__(NT) void ref_kernel(int mode, int n, long long batch, int iterations,
                                                 double box_min, double box_max, const double *__restrict__ Pg,
                                                 const double *__restrict__ qg, const double *__restrict__ x0g,
                                                 double *__restrict__ xg, int32_t *__restrict__ itg,
                                                 double *__restrict__ ws) {
  extern __shared__ double sm[];
  for (long long g = blockIdx.x; g < batch; g += gridDim.x) {
    ref_solve_one<NT>(sm, ws, mode, n, g, iterations, box_min, box_max, Pg, qg, x0g, xg, itg);
    __syncthreads();  // LDS and workspace are reused by the next QP
  }
}

// f(x) = 1/2 x^T (P x) + q^T x + r with the reference's order of operations:
// tmp = matrix_mult(P, x) (sequential k), 0.5 * scalar_prod(x, tmp), + q.x, + r.
__global__ void qf_eval_kernel(int n, long long batch, const double *__restrict__ P, const double *__restrict__ q,
                               double r, const double *__restrict__ x, double *__restrict__ out) {
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= batch) return;
  const double *Pq = P + g * (long long)n * n;
  const double *xq = x + g * n;
  const double *qq = q + g * n;
  double xa = 0.0;
  for (int i = 0; i < n; ++i) {
    double acc = 0.0;
    for (int k = 0; k < n; ++k) acc += Pq[i * n + k] * xq[k];
    xa += xq[i] * acc;
  }
  double a = 0.5 * xa;
  double qa = 0.0;
  for (int k = 0; k < n; ++k) qa += qq[k] * xq[k];
  a += qa;
  a += r;
  out[g] = a;
}

// Batched matrix_invert (matrix_ops.c:551-630) on its own: P -> P^{-1} per
// QP, the same LU + per-column solves the Newton / ADMM replicas run.
template <int NT>
__global__ __launch_bounds__(NT) void ref_invert_kernel(int n, long long batch, const double *__restrict__ Pg,
                                                        double *__restrict__ Vg, double *__restrict__ ws) {
  extern __shared__ double sm[];
  const int tid = threadIdx.x;
  const int nn2 = n * n;
  for (long long g = blockIdx.x; g < batch; g += gridDim.x) {
    RefShared S;
    ref_carve<NT>(S, sm, ws, n, false);
    const double *Pq = Pg + g * (long long)nn2;
    if constexpr (NT == REF_BIG_NT) {
      ref_load_m<NT>(S, Pq, n, 0.0);
      ref_invert_big(S, n);
    } else {
      for (int e = tid; e < nn2; e += NT) S.M[e] = Pq[e];
      __syncthreads();
      ref_invert_small<NT>(S, n);
    }
    double *Vq = Vg + g * (long long)nn2;
    for (int e = tid; e < nn2; e += NT) {
      const int r = e / n, c = e - r * n;
      Vq[e] = S.V(r, c);
    }
    __syncthreads();
  }
}

}  // namespace qpb

namespace {
// LDS bytes of one workgroup: the matrices ([P n^2] [M W V 3 n^2] for
// n <= 64; X = n ld for n > 64) + 9 vectors + 8 scalars + 2 reduction slots
// (doubles), perm + 2 (ints)
size_t ref_lds_bytes(int n, bool with_p) {
  const size_t nn2 = (size_t)n * n;
  if (n > qpb::REF_BIG_MAXN)  // the matrices live in the workspace; 16 reduction slots
    return sizeof(double) * (9 * (size_t)n + 8 + 16) + sizeof(int) * ((size_t)n + 16);
  const size_t mats = n <= qpb::REF_LDS_MAXN ? (with_p ? nn2 : 0) + 3 * nn2 : (size_t)qpb::ref_npad(n) * (qpb::ref_ld(n) + 2);
  return sizeof(double) * (mats + 9 * (size_t)n + 10) + sizeof(int) * ((size_t)n + 2);
}
// 128 < n <= 1024: one 1024-thread workgroup per CU at most, each with a
// 4 n^2 slice of the cached workspace, the grid capped so that the slices
// stay within 2 GiB (64 workgroups at n = 1024)
hipError_t ref_huge_launch(long long batch, int n, hipStream_t stream,
                           const std::function<void(unsigned grid, double *ws)> &launch) {
  int dev = 0, cus = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return e;
  const size_t slice = (size_t)qpb::REF_HUGE_WS_MATS * (size_t)n * n * sizeof(double);
  long long cap = (long long)((2ull << 30) / slice);
  if (cap < 1) cap = 1;
  if (cap > cus) cap = cus;
  const unsigned grid = (unsigned)(batch < cap ? batch : cap);
  return qpb_with_workspace(stream, (size_t)grid * slice, [&](void *p) {
    launch(grid, static_cast<double *>(p));
    return hipGetLastError();
  });
}
// n > 64: as many workgroups per CU as their LDS allows (one at n = 128, at
// most REF_MAX_WG_PER_CU) walk the batch, each with its 2 n^2 slice of the
// cached workspace; `launch` queues the kernel while the cache is locked
hipError_t ref_big_launch(long long batch, int n, size_t lds, hipStream_t stream,
                          const std::function<void(unsigned grid, double *ws)> &launch) {
  int dev = 0, cus = 0, lds_cu = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  // the CU's LDS, from the device (160 KiB on gfx950)
  if (e == hipSuccess) e = hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev);
  if (e != hipSuccess) return e;
  long long per_cu = (long long)((size_t)lds_cu / lds);
  if (per_cu < 1) per_cu = 1;
  if (per_cu > qpb::REF_MAX_WG_PER_CU) per_cu = qpb::REF_MAX_WG_PER_CU;
  const long long slots = (long long)cus * per_cu;
  const unsigned grid = (unsigned)(batch < slots ? batch : slots);
  return qpb_with_workspace(stream, (size_t)grid * qpb::REF_WS_MATS * (size_t)n * n * sizeof(double), [&](void *p) {
    launch(grid, static_cast<double *>(p));
    return hipGetLastError();
  });
}
template <class K>
hipError_t allow_lds(K kern, size_t lds) {
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (lds <= 64 * 1024) return hipSuccess;
  return hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)lds);
}
}  // namespace

extern "C" hipError_t qpb_launch_ref_invert(int n, long long batch, const double *P, double *Pinv,
                                            hipStream_t stream) {
  if (n > qpb::REF_MAXN) return hipErrorInvalidValue;
  if (batch == 0) return hipSuccess;
  const size_t lds = ref_lds_bytes(n, false);
  if (n <= qpb::REF_LDS_MAXN) {
    hipError_t e = allow_lds(&qpb::ref_invert_kernel<64>, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(qpb::ref_invert_kernel<64>, dim3((unsigned)batch), dim3(64), lds, stream, n, batch, P, Pinv,
                       nullptr);
  } else if (n > qpb::REF_BIG_MAXN) {
    hipError_t e = allow_lds(&qpb::ref_invert_kernel<qpb::REF_HUGE_NT>, lds);
    if (e == hipSuccess)
      e = ref_huge_launch(batch, n, stream, [&](unsigned grid, double *ws) {
        hipLaunchKernelGGL(qpb::ref_invert_kernel<qpb::REF_HUGE_NT>, dim3(grid), dim3(qpb::REF_HUGE_NT), lds, stream,
                           n, batch, P, Pinv, ws);
      });
    if (e != hipSuccess) return e;
  } else {
    hipError_t e = allow_lds(&qpb::ref_invert_kernel<128>, lds);
    if (e == hipSuccess)
      e = ref_big_launch(batch, n, lds, stream, [&](unsigned grid, double *ws) {
        hipLaunchKernelGGL(qpb::ref_invert_kernel<128>, dim3(grid), dim3(128), lds, stream, n, batch, P, Pinv, ws);
      });
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

extern "C" hipError_t qpb_launch_qf_eval(int n, long long batch, const double *P, const double *q, double r,
                                         const double *x, double *out, hipStream_t stream) {
  const long long blocks = (batch + 255) / 256;
  hipLaunchKernelGGL(qpb::qf_eval_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, n, batch, P, q, r, x, out);
  return hipGetLastError();
}

extern "C" hipError_t qpb_launch_ref(const qpb_ref_desc *d, const double *P, const double *q, const double *x0,
                                     double *x, int32_t *iters, hipStream_t stream) {
  if (d->n > qpb::REF_MAXN) return hipErrorInvalidValue;
  if (d->batch == 0) return hipSuccess;
  const int n = d->n;
  const size_t lds = ref_lds_bytes(n, true);
  if (n <= qpb::REF_LDS_MAXN) {
    hipError_t e = allow_lds(&qpb::ref_kernel<64>, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(qpb::ref_kernel<64>, dim3((unsigned)d->batch), dim3(64), lds, stream, d->mode, n,
                       (long long)d->batch, d->iterations, d->box_min, d->box_max, P, q, x0, x, iters, nullptr);
  } else if (n > qpb::REF_BIG_MAXN) {
    hipError_t e = allow_lds(&qpb::ref_kernel<qpb::REF_HUGE_NT>, lds);
    if (e == hipSuccess)
      e = ref_huge_launch(d->batch, n, stream, [&](unsigned grid, double *ws) {
        hipLaunchKernelGGL(qpb::ref_kernel<qpb::REF_HUGE_NT>, dim3(grid), dim3(qpb::REF_HUGE_NT), lds, stream,
                           d->mode, n, (long long)d->batch, d->iterations, d->box_min, d->box_max, P, q, x0, x, iters,
                           ws);
      });
    if (e != hipSuccess) return e;
  } else {
    hipError_t e = allow_lds(&qpb::ref_kernel<128>, lds);
    if (e == hipSuccess)
      e = ref_big_launch(d->batch, n, lds, stream, [&](unsigned grid, double *ws) {
        hipLaunchKernelGGL(qpb::ref_kernel<128>, dim3(grid), dim3(128), lds, stream, d->mode, n, (long long)d->batch,
                           d->iterations, d->box_min, d->box_max, P, q, x0, x, iters, ws);
      });
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}
