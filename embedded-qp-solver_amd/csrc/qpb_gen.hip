// qpb_gen.hip -- on-device batched input generators.
//
// 1. The reference's own generator, bit for bit (qpb_ref_generate):
//    srand(seed) once, then per QP in main.c:37-39 order
//      P  = matirx_random_pos_def   (matrix_ops.c:699-734: B = matrix_random,
//                                    B^T B by the sequential-k matrix_mult of
//                                    :235-271, scaled by 1/(max n))
//      q  = matrix_random, x0 = matrix_random      (U[min, max] each)
//    with random_number = min + rand() * (max - min) / RAND_MAX (:677-681)
//    and glibc's TYPE_3 rand().  QP k starts at output k * (n^2 + 2n) of the
//    stream: every QP finds its position by jump-ahead, so a batch (or any
//    shard [first, first + batch) of it) is produced in parallel and is
//    identical to the sequential reference run.
//
//    glibc TYPE_3 (stdlib/random_r.c): after srandom_r the 31-word window
//    obeys s[t] = s[t-31] + s[t-3] (mod 2^32); rand() returns s >> 1 and the
//    first 310 results are discarded.  The recurrence is linear, so
//    s[T] = sum_j c_j s[j] with sum_j c_j x^j = x^T mod (x^31 - x^28 - 1)
//    over Z/2^32: square-and-multiply on 31-coefficient polynomials.
//
// 2. The benchmark families (qpb_generate): a counter-based Philox4x32-10
//    stream keyed by (seed, QP index), so any shard of a batch is identical
//    to the same QPs of the full batch; H = B^T B / (1e3 n) + shift I with
//    the n x n product on the matrix cores (v_mfma_f64_16x16x4_f64).
#include "qpb_common.h"
#include "qpb.h"

namespace qpb {
namespace gen {

constexpr int DEG = 31;  // glibc TYPE_3 degree, separation 3

// c <- c * c mod (x^31 - x^28 - 1)
__device__ __forceinline__ void poly_sqr(uint32_t (&c)[DEG]) {
  uint32_t p[2 * DEG - 1];
#pragma unroll
  for (int i = 0; i < 2 * DEG - 1; ++i) p[i] = 0;
#pragma unroll
  for (int i = 0; i < DEG; ++i)
#pragma unroll
    for (int j = 0; j < DEG; ++j) p[i + j] += c[i] * c[j];
  // x^d = x^(d-3) + x^(d-31) for d >= 31, from the top down
#pragma unroll
  for (int d = 2 * DEG - 2; d >= DEG; --d) {
    p[d - 3] += p[d];
    p[d - DEG] += p[d];
  }
#pragma unroll
  for (int i = 0; i < DEG; ++i) c[i] = p[i];
}

// c <- x * c mod (x^31 - x^28 - 1)
__device__ __forceinline__ void poly_mulx(uint32_t (&c)[DEG]) {
  const uint32_t top = c[DEG - 1];
#pragma unroll
  for (int i = DEG - 1; i > 0; --i) c[i] = c[i - 1];
  c[0] = top;
  c[DEG - 3] += top;
}

// srandom_r's window: s[j] = r[3 + j] (the first 31 terms obeying the recurrence)
__host__ __device__ inline void glibc_base(uint32_t seed, uint32_t (&s)[DEG]) {
  int32_t r[34];
  int32_t word = (int32_t)seed;
  if (word == 0) word = 1;
  r[0] = word;
  for (int i = 1; i < 31; ++i) {
    const int32_t hi = word / 127773, lo = word % 127773;
    word = 16807 * lo - 2836 * hi;
    if (word < 0) word += 2147483647;
    r[i] = word;
  }
  for (int i = 31; i < 34; ++i) r[i] = r[i - 31];
  for (int j = 0; j < DEG; ++j) s[j] = (uint32_t)r[3 + j];
}

// one thread per QP: raw draws of QP k (B row-major into P, then q, x0)
__global__ __launch_bounds__(64) void ref_draws_kernel(int n, long long batch, unsigned long long first,
                                                       unsigned seed, double pmin, double pmax, double qmin,
                                                       double qmax, double xmin, double xmax, double *__restrict__ P,
                                                       double *__restrict__ q, double *__restrict__ x0) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= batch) return;
  uint32_t base[DEG];
  glibc_base(seed, base);
  const unsigned long long D = (unsigned long long)n * n + 2ull * n;
  // output o of rand() is s[341 + o] >> 1; the window preceding the first
  // draw of this QP starts at s[T0], T0 = 341 + (first + k) D - 31
  const unsigned long long T0 = 310ull + (first + (unsigned long long)k) * D;
  uint32_t c[DEG];
#pragma unroll
  for (int i = 0; i < DEG; ++i) c[i] = i == 0 ? 1u : 0u;
  for (int b = 63 - __builtin_clzll(T0 | 1); b >= 0; --b) {  // left-to-right binary powering of x
    poly_sqr(c);
    if ((T0 >> b) & 1) poly_mulx(c);
  }
  uint32_t w[DEG];  // w[j] = s[T0 + j]
#pragma unroll
  for (int j = 0; j < DEG; ++j) {
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < DEG; ++i) v += c[i] * base[i];
    w[j] = v;
    poly_mulx(c);
  }
  double *Pk = P + k * (long long)n * n;
  double *qk = q + k * (long long)n;
  double *xk = x0 + k * (long long)n;
  const int nn = n * n;
  const int D32 = (int)D;
  // blocks of 31: updating w[i] in place for i = 0..30 is exactly
  // s[t] = s[t-31] + s[t-3] (w[(i+28)%31] already holds s[t-3]), with
  // compile-time indices (the window stays in registers)
  for (int o = 0; o < D32;) {
#pragma unroll
    for (int i = 0; i < DEG; ++i) {
      w[i] += w[(i + DEG - 3) % DEG];
      if (o < D32) {
        const double r = (double)(w[i] >> 1);
        if (o < nn) Pk[o] = pmin + r * (pmax - pmin) / 2147483647.0;
        else if (o < nn + n) qk[o - nn] = qmin + r * (qmax - qmin) / 2147483647.0;
        else xk[o - nn - n] = xmin + r * (xmax - xmin) / 2147483647.0;
        ++o;
      }
    }
  }
}

// one workgroup per QP (64 threads; 256 when n > 64): P <- B^T B / (pmax n),
// the reference's operation order (k ascending, product rounded then added:
// matrix_mult :235-271, compiled with -ffp-contract=off like the reference
// build)
__global__ __launch_bounds__(256) void ref_posdef_kernel(int n, long long batch, double pmax,
                                                        double *__restrict__ P) {
  extern __shared__ double Bs[];
  const long long k = blockIdx.x;
  if (k >= batch) return;
  double *Pk = P + k * (long long)n * n;
  for (int i = threadIdx.x; i < n * n; i += blockDim.x) Bs[i] = Pk[i];
  __syncthreads();
  const double scale = 1.0 / (pmax * n);
  for (int e = threadIdx.x; e < n * n; e += blockDim.x) {
    const int i = e / n, j = e % n;
    double acc = 0.0;
    for (int t = 0; t < n; ++t) acc = acc + Bs[t * n + i] * Bs[t * n + j];
    Pk[e] = acc * scale;
  }
}

// ---------------------------------------------------------------- Philox
// Philox4x32-10 (Salmon et al., SC'11), counter (element block, QP lo, QP hi,
// purpose), key (seed lo, seed hi)
__host__ __device__ inline void philox(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1;
    c[3] = (uint32_t)p0;
    c[0] = n0;
    c[2] = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}
// element e of stream `purpose` of QP g: a double in [0, 1) with 53 random bits
__host__ __device__ inline double uniform(unsigned long long seed, unsigned long long g, uint32_t purpose,
                                          uint32_t e) {
  uint32_t c[4] = {e >> 1, (uint32_t)g, (uint32_t)(g >> 32), purpose};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const uint32_t hi = (e & 1) ? c[2] : c[0], lo = (e & 1) ? c[3] : c[1];
  return ((double)(hi >> 5) * 67108864.0 + (double)(lo >> 6)) * (1.0 / 9007199254740992.0);
}
enum : uint32_t { kStreamB = 0, kStreamF = 1, kStreamA = 2, kStreamBvec = 3 };

// one wave per QP.  H = B^T B / (1e3 n) + shift I on the matrix cores: per
// 16 x 16 tile, K in steps of 4; lane l feeds A[i = l&15][k = l>>4] =
// B[k][i] and B[k][j = l&15] (v_mfma_f64_16x16x4_f64, C/D: col = l&15,
// row = (l>>4) + 4 r).  For n > 16 the B matrix is staged in the A output
// (m >= n rows) and re-read per tile; for n <= 16 it never leaves registers.
__global__ __launch_bounds__(64) void family_kernel(int n, int m, long long batch, unsigned long long first,
                                                    unsigned long long seed, int family, double shift, double box,
                                                    double *__restrict__ H, double *__restrict__ f,
                                                    double *__restrict__ A, double *__restrict__ b) {
  const long long k = blockIdx.x;
  if (k >= batch) return;
  const unsigned long long g = first + (unsigned long long)k;
  const int l = threadIdx.x;
  const int li = l & 15, lk = l >> 4;
  double *Hk = H + k * (long long)n * n;
  double *Ak = A + k * (long long)m * n;
  const bool staged = n > 16;
  auto bval = [&](int kk, int i) -> double {  // B[kk][i], zero padding outside n
    if (kk >= n || i >= n) return 0.0;
    if (staged) return Ak[kk * n + i];
    return -1e3 + 2e3 * uniform(seed, g, kStreamB, (uint32_t)(kk * n + i));
  };
  if (staged) {
    for (int e = l; e < n * n; e += 64) Ak[e] = -1e3 + 2e3 * uniform(seed, g, kStreamB, (uint32_t)e);
    __threadfence_block();
    __syncthreads();
  }
  const int nt = (n + 15) / 16;
  const double scale = 1e3 * n;
  // upper tiles only; each result is stored at (row, col) and (col, row), so
  // H is exactly symmetric
  for (int ti = 0; ti < nt; ++ti)
    for (int tj = ti; tj < nt; ++tj) {
      using d4 = __attribute__((__vector_size__(4 * sizeof(double)))) double;
      d4 acc = {0.0, 0.0, 0.0, 0.0};
      for (int k4 = 0; k4 < n; k4 += 4) {
        const double a = bval(k4 + lk, ti * 16 + li);
        const double bb = ti == tj ? a : bval(k4 + lk, tj * 16 + li);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = ti * 16 + lk + 4 * r, col = tj * 16 + li;
        if (row < n && col < n && row <= col) {
          const double h = acc[r] / scale + (row == col ? shift : 0.0);
          Hk[row * n + col] = h;
          Hk[col * n + row] = h;
        }
      }
    }
  if (staged) {
    __syncthreads();  // every lane done with the staged B before A is written
  }
  for (int i = l; i < n; i += 64) f[k * (long long)n + i] = -1e3 + 2e3 * uniform(seed, g, kStreamF, (uint32_t)i);
  if (family == 0) {  // box |x_i| <= box as the dense rows [I; -I]
    for (int e = l; e < m * n; e += 64) {
      const int row = e / n, col = e % n;
      Ak[e] = row < n ? (row == col ? 1.0 : 0.0) : (row - n == col ? -1.0 : 0.0);
    }
    for (int i = l; i < m; i += 64) b[k * (long long)m + i] = box;
  } else {  // dense: rows ~ N(0, I) normalised, b ~ U[0.1, 1) box (x = 0 strictly feasible)
    for (int row = l; row < m; row += 64) {
      double nrm = 0.0;
      for (int col = 0; col < n; ++col) {
        const uint32_t e = (uint32_t)(row * n + col);
        // Box-Muller on the pair (2e, 2e+1) of the A stream, cosine branch
        const double u1 = uniform(seed, g, kStreamA, 2 * e), u2 = uniform(seed, g, kStreamA, 2 * e + 1);
        const double z = sqrt(-2.0 * log(1.0 - u1)) * cos(6.283185307179586 * u2);
        Ak[row * n + col] = z;
        nrm += z * z;
      }
      const double inv = 1.0 / sqrt(nrm);
      for (int col = 0; col < n; ++col) Ak[row * n + col] *= inv;
      b[k * (long long)m + row] = (0.1 + 0.9 * uniform(seed, g, kStreamBvec, (uint32_t)row)) * box;
    }
  }
}

}  // namespace gen
}  // namespace qpb

extern "C" hipError_t qpb_launch_generate(int n, int m, long long batch, unsigned long long first,
                                          unsigned long long seed, int family, double shift, double box, double *H,
                                          double *f, double *A, double *b, hipStream_t stream) {
  if (batch == 0) return hipSuccess;
  hipLaunchKernelGGL(qpb::gen::family_kernel, dim3((unsigned)batch), dim3(64), 0, stream, n, m, batch, first, seed,
                     family, shift, box, H, f, A, b);
  return hipGetLastError();
}

extern "C" hipError_t qpb_launch_ref_generate(int n, long long batch, unsigned long long first, unsigned seed,
                                              const double *range, double *P, double *q, double *x0,
                                              hipStream_t stream) {
  if (batch == 0) return hipSuccess;
  const unsigned grid1 = (unsigned)((batch + 63) / 64);
  hipLaunchKernelGGL(qpb::gen::ref_draws_kernel, dim3(grid1), dim3(64), 0, stream, n, batch, first, seed, range[0],
                     range[1], range[2], range[3], range[4], range[5], P, q, x0);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t lds = (size_t)n * n * sizeof(double);  // B of one QP (n = 128: 128 KiB)
  if (lds > 64 * 1024) {
    e = hipFuncSetAttribute(reinterpret_cast<const void *>(&qpb::gen::ref_posdef_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(qpb::gen::ref_posdef_kernel, dim3((unsigned)batch), dim3(n > 64 ? 256 : 64), lds, stream, n,
                     batch, range[1], P);
  return hipGetLastError();
}
