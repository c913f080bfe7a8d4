// qpb_ref.hip -- reference-semantics kernels and the
// batched quadratic-form evaluation (qp.c:9-27).
//
// Compiled with -ffp-contract=off: the reference's arithmetic (gcc -O2,
// x86-64, no FMA) rounds every product and sum separately, and these kernels
// reproduce its operation order.
#include "qpb_common.h"
#include "qpb.h"

namespace qpb {

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

}  // namespace qpb

extern "C" hipError_t qpb_launch_qf_eval(int n, long long batch, const double *P, const double *q, double r,
                                         const double *x, double *out, hipStream_t stream) {
  const long long blocks = (batch + 255) / 256;
  hipLaunchKernelGGL(qpb::qf_eval_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, n, batch, P, q, r, x, out);
  return hipGetLastError();
}

extern "C" hipError_t qpb_launch_ref(const qpb_ref_desc *, const double *, const double *, const double *, double *,
                                     int32_t *, hipStream_t) {
  return hipErrorNotSupported;  // reference-semantics kernels: next milestone
}
