// qpb_api.hip -- the C-ABI of include/qpb.h: argument checking, launches,
// host-pointer convenience wrappers.  No computation happens here: every
// solve runs in the HIP kernels (qpb_gi.hip, qpb_ref.hip); there is no CPU
// fallback -- without a usable HIP device the calls fail with
// QPB_ERR_NO_DEVICE / QPB_ERR_HIP.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "qpb.h"
#include "qpb_common.h"  // kSectionSlots, kSections

extern "C" hipError_t qpb_launch_gi(const qpb_desc *d, const double *H, const double *f, const double *A,
                                    const double *b, double *x, double *lam, uint32_t *active,
                                    int32_t *status, int32_t *iters, hipStream_t stream);
extern "C" hipError_t qpb_launch_gi_sections(const qpb_desc *d, const double *H, const double *f, const double *A,
                                             const double *b, double *x, double *lam, uint32_t *active,
                                             int32_t *status, int32_t *iters, unsigned long long *sections,
                                             hipStream_t stream);
extern "C" hipError_t qpb_launch_gi_wave_sections(const qpb_desc *d, const double *H, const double *f,
                                                  const double *A, const double *b, double *x, double *lam,
                                                  uint32_t *active, int32_t *status, int32_t *iters,
                                                  unsigned long long *sections, hipStream_t stream);
extern "C" hipError_t qpb_launch_gi_wave(const qpb_desc *d, const double *H, const double *f, const double *A,
                                         const double *b, double *x, double *lam, uint32_t *active, int32_t *status,
                                         int32_t *iters, hipStream_t stream);
extern "C" hipError_t qpb_launch_gi_mixed(const qpb_desc *d, const double *H, const double *f, const double *A,
                                          const double *b, double *x, double *lam, uint32_t *active,
                                          int32_t *status, int32_t *iters, hipStream_t stream);
extern "C" hipError_t qpb_launch_gi_gram(const qpb_desc *d, const double *H, const double *f, const double *A,
                                         const double *b, double *x, double *lam, uint32_t *active,
                                         int32_t *status, int32_t *iters, unsigned long long *sections,
                                         hipStream_t stream);
extern "C" hipError_t qpb_launch_gi_box(const qpb_desc *d, const double *H, const double *f, const double *lb,
                                        const double *ub, double *x, double *lam, uint32_t *active, int32_t *status,
                                        int32_t *iters, hipStream_t stream);
extern "C" hipError_t qpb_launch_gi_gram_box(const qpb_desc *d, const double *H, const double *f, const double *lb,
                                             const double *ub, double *x, double *lam, uint32_t *active,
                                             int32_t *status, int32_t *iters, hipStream_t stream);
extern "C" hipError_t qpb_launch_gi_wave_box(const qpb_desc *d, const double *H, const double *f, const double *lb,
                                             const double *ub, double *x, double *lam, uint32_t *active,
                                             int32_t *status, int32_t *iters, hipStream_t stream);
extern "C" hipError_t qpb_launch_ref(const qpb_ref_desc *d, const double *P, const double *q,
                                     const double *x0, double *x, int32_t *iters, hipStream_t stream);
extern "C" hipError_t qpb_launch_qf_eval(int n, long long batch, const double *P, const double *q, double r,
                                         const double *x, double *out, hipStream_t stream);
extern "C" hipError_t qpb_launch_ref_invert(int n, long long batch, const double *P, double *Pinv,
                                            hipStream_t stream);

extern "C" hipError_t qpb_launch_ref_generate(int n, long long batch, unsigned long long first, unsigned seed,
                                              const double *range, double *P, double *q, double *x0,
                                              hipStream_t stream);
extern "C" hipError_t qpb_launch_generate(int n, int m, long long batch, unsigned long long first,
                                          unsigned long long seed, int family, double shift, double box, double *H,
                                          double *f, double *A, double *b, hipStream_t stream);

static thread_local char g_err[512] = "";

static int fail(int code, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

// error reporting for the host-only C parts of the library (qpb_wire.c)
extern "C" __attribute__((visibility("hidden"))) void qpb_set_error(int code, const char *msg) {
  fail(code, "%s", msg);
}

static int hip_fail(hipError_t e, const char *what) {
  return fail(QPB_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

// The device census is taken once per process (a HIP runtime query per solve
// cost ~8 us of host time on every launch); a process without a device keeps
// failing with QPB_ERR_NO_DEVICE.
static int device_census(void) {
  static const int count = [] {
    int c = 0;
    return hipGetDeviceCount(&c) == hipSuccess ? c : 0;
  }();
  return count;
}

static int check_device(void) {
  if (device_census() <= 0) return fail(QPB_ERR_NO_DEVICE, "no HIP device available");
  return 0;
}

// QPs per launch: a launch's grid holds at most 2^32 - 1 work-items, so each
// kernel family takes at most 2^32 / (threads per QP) QPs per launch (minus a
// margin); larger batches are split into consecutive launches on the stream.
static long long chunk_qps(int n, int m, int flags = 0) {
  if (n <= 16 && m <= 32 && !(flags & QPB_FLAG_DIAG_WAVE)) return 1LL << 27;  // 16 lanes per QP
  if (n <= 32 && m <= 64) return 1LL << 25;  // 64 lanes per QP
  return 1LL << 21;                          // n <= 128: one workgroup per CU walks the QPs (bounded chunks)
}

static int check_desc(const qpb_desc *d) {
  if (!d) return fail(QPB_ERR_INVALID_ARG, "desc is NULL");
  if (d->batch < 0) return fail(QPB_ERR_INVALID_ARG, "batch < 0");
  if (d->n < 1 || d->m < 0) return fail(QPB_ERR_INVALID_ARG, "n must be >= 1 and m >= 0");
  if (d->n > QPB_MAX_N || d->m > QPB_MAX_M)
    return fail(QPB_ERR_UNSUPPORTED, "n=%d m=%d outside this build's kernels (n<=%d, m<=%d)", d->n, d->m,
                QPB_MAX_N, QPB_MAX_M);
  return 0;
}

extern "C" int qpb_solve(const qpb_desc *d, const double *H, const double *f, const double *A,
                         const double *b, double *x, double *lam, uint32_t *active, int32_t *status,
                         int32_t *iters, void *stream) {
  int rc = check_desc(d);
  if (rc) return rc;
  if (d->batch == 0) return 0;
  if (!H || !f || !x || !status) return fail(QPB_ERR_INVALID_ARG, "H, f, x and status are required");
  if (d->m > 0 && (!A || !b || !lam || !active))
    return fail(QPB_ERR_INVALID_ARG, "A, b, lam and active are required when m > 0");
  rc = check_device();
  if (rc) return rc;
  // n <= 16, m <= 32: four QPs per wavefront; n <= 32, m <= 64: one QP per
  // wavefront; larger: one QP per workgroup
  const long long n = d->n, m = d->m, w = (m + 31) / 32, step = chunk_qps(d->n, d->m, d->flags);
  for (long long k0 = 0; k0 < d->batch; k0 += step) {
    qpb_desc c = *d;
    c.batch = d->batch - k0 < step ? d->batch - k0 : step;
    const double *Hc = H + k0 * n * n, *fc = f + k0 * n;
    const double *Ac = m ? A + k0 * m * n : A, *bc = m ? b + k0 * m : b;
    double *xc = x + k0 * n, *lc = m ? lam + k0 * m : lam;
    uint32_t *ac = m ? active + k0 * w : active;
    int32_t *sc = status + k0, *ic = iters ? iters + k0 : iters;
    hipError_t e;
    if (d->n <= 16 && d->m <= 32 && !(d->flags & QPB_FLAG_DIAG_WAVE))
      e = qpb_launch_gi(&c, Hc, fc, Ac, bc, xc, lc, ac, sc, ic, (hipStream_t)stream);
    else if (d->n > 16 && d->n <= 32 && d->m <= 64 && (d->flags & QPB_FLAG_MIXED))
      e = qpb_launch_gi_mixed(&c, Hc, fc, Ac, bc, xc, lc, ac, sc, ic, (hipStream_t)stream);
    else if (d->n <= 32 && d->m <= 64)
      e = qpb_launch_gi_wave(&c, Hc, fc, Ac, bc, xc, lc, ac, sc, ic, (hipStream_t)stream);
    else
      e = qpb_launch_gi_gram(&c, Hc, fc, Ac, bc, xc, lc, ac, sc, ic, nullptr, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "qpb_solve launch");
  }
  return 0;
}

extern "C" int qpb_solve_box(const qpb_desc *d, const double *H, const double *f, const double *lb,
                             const double *ub, double *x, double *lam, uint32_t *active, int32_t *status,
                             int32_t *iters, void *stream) {
  int rc = check_desc(d);
  if (rc) return rc;
  if (d->m != 2 * d->n) return fail(QPB_ERR_INVALID_ARG, "qpb_solve_box: m must be 2n (got n=%d m=%d)", d->n, d->m);
  if (d->batch == 0) return 0;
  if (!H || !f || !x || !lam || !active || !status)
    return fail(QPB_ERR_INVALID_ARG, "H, f, x, lam, active and status are required");
  rc = check_device();
  if (rc) return rc;
  // n <= 16: four QPs per wavefront (qpb_gi_box.hip), at most 2^27 QPs per
  // launch (2^32 work-items); 16 < n <= 32: one QP per wavefront (the BOX
  // instantiation of qpb_gi_wave.hip), 2^25; 32 < n <= 128: one QP per
  // workgroup (the BOX instantiation of qpb_gi_gram.hip, a persistent grid)
  const long long n = d->n, w = (2 * n + 31) / 32, step = n <= 16 ? 1LL << 27 : 1LL << 25;
  for (long long k0 = 0; k0 < d->batch; k0 += step) {
    qpb_desc c = *d;
    c.batch = d->batch - k0 < step ? d->batch - k0 : step;
    hipError_t e = (n <= 16 ? qpb_launch_gi_box : n <= 32 ? qpb_launch_gi_wave_box : qpb_launch_gi_gram_box)(
        &c, H + k0 * n * n, f + k0 * n, lb ? lb + k0 * n : lb, ub ? ub + k0 * n : ub, x + k0 * n, lam + k0 * 2 * n,
        active + k0 * w, status + k0, iters ? iters + k0 : iters, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "qpb_solve_box launch");
  }
  return 0;
}

extern "C" int qpb_solve_sections(const qpb_desc *d, const double *H, const double *f, const double *A,
                                  const double *b, double *x, double *lam, uint32_t *active, int32_t *status,
                                  int32_t *iters, unsigned long long *sections, int64_t sections_len,
                                  void *stream) {
  int rc = check_desc(d);
  if (rc) return rc;
  static_assert(QPB_SECTIONS_LEN == qpb::kSectionSlots * qpb::kSections, "sections buffer shape");
  if (sections && sections_len < QPB_SECTIONS_LEN)
    return fail(QPB_ERR_INVALID_ARG, "sections: the buffer must hold QPB_SECTIONS_LEN (256 x 20) counters");
  if (d->batch == 0) return 0;
  const bool n16 = d->n == 16 && d->m > 16 && d->m <= 32, wave = d->n > 16 && d->n <= 32 && d->m <= 64;
  const bool gram = !(d->n <= 32 && d->m <= 64) && d->batch <= chunk_qps(d->n, d->m);
  if (!(n16 || wave || gram) || !sections)
    return fail(QPB_ERR_UNSUPPORTED, "sections: n=16 with 16<m<=32, 16<n<=32 with m<=64, or the n<=128 class");
  rc = check_device();
  if (rc) return rc;
  hipError_t e;
  if (n16)
    e = qpb_launch_gi_sections(d, H, f, A, b, x, lam, active, status, iters, sections, (hipStream_t)stream);
  else if (wave)
    e = qpb_launch_gi_wave_sections(d, H, f, A, b, x, lam, active, status, iters, sections, (hipStream_t)stream);
  else
    e = qpb_launch_gi_gram(d, H, f, A, b, x, lam, active, status, iters, sections, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "qpb_solve_sections launch");
  return 0;
}

// ---- host-pointer wrappers -------------------------------------------------
struct DevBuf {
  void *p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

static hipError_t up(DevBuf &b, const void *src, size_t bytes) {
  if (!src || !bytes) return hipSuccess;
  hipError_t e = hipMalloc(&b.p, bytes);
  if (e != hipSuccess) return e;
  return hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice);
}
static hipError_t alloc(DevBuf &b, const void *dst, size_t bytes) {
  if (!dst || !bytes) return hipSuccess;
  return hipMalloc(&b.p, bytes);
}
static hipError_t down(void *dst, const DevBuf &b, size_t bytes) {
  if (!dst || !bytes) return hipSuccess;
  return hipMemcpy(dst, b.p, bytes, hipMemcpyDeviceToHost);
}

#define HIPCHK(expr, what)                  \
  do {                                      \
    hipError_t e_ = (expr);                 \
    if (e_ != hipSuccess) return hip_fail(e_, what); \
  } while (0)

extern "C" int qpb_solve_host(const qpb_desc *d, const double *H, const double *f, const double *A,
                              const double *b, double *x, double *lam, uint32_t *active, int32_t *status,
                              int32_t *iters) {
  int rc = check_desc(d);
  if (rc) return rc;
  if (d->batch == 0) return 0;
  rc = check_device();
  if (rc) return rc;
  const size_t B = (size_t)d->batch, n = d->n, m = d->m, w = (m + 31) / 32;
  DevBuf dH, df, dA, db, dx, dl, da, ds, di;
  HIPCHK(up(dH, H, B * n * n * 8), "H");
  HIPCHK(up(df, f, B * n * 8), "f");
  HIPCHK(up(dA, m ? A : nullptr, B * m * n * 8), "A");
  HIPCHK(up(db, m ? b : nullptr, B * m * 8), "b");
  HIPCHK(alloc(dx, x, B * n * 8), "x");
  HIPCHK(alloc(dl, m ? lam : nullptr, B * m * 8), "lam");
  HIPCHK(alloc(da, m ? active : nullptr, B * w * 4), "active");
  HIPCHK(alloc(ds, status, B * 4), "status");
  HIPCHK(alloc(di, iters, B * 4), "iters");
  rc = qpb_solve(d, (double *)dH.p, (double *)df.p, (double *)dA.p, (double *)db.p, (double *)dx.p,
                 (double *)dl.p, (uint32_t *)da.p, (int32_t *)ds.p, (int32_t *)di.p, nullptr);
  if (rc) return rc;
  HIPCHK(hipDeviceSynchronize(), "qpb_solve_host kernel");
  HIPCHK(down(x, dx, B * n * 8), "x D2H");
  HIPCHK(down(m ? lam : nullptr, dl, B * m * 8), "lam D2H");
  HIPCHK(down(m ? active : nullptr, da, B * w * 4), "active D2H");
  HIPCHK(down(status, ds, B * 4), "status D2H");
  HIPCHK(down(iters, di, B * 4), "iters D2H");
  return 0;
}

static int check_ref(const qpb_ref_desc *d) {
  if (!d) return fail(QPB_ERR_INVALID_ARG, "desc is NULL");
  if (d->batch < 0 || d->n < 1 || d->iterations < 0) return fail(QPB_ERR_INVALID_ARG, "bad n/batch/iterations");
  if (d->mode != QPB_REF_NEWTON && d->mode != QPB_REF_ADMM && d->mode != QPB_REF_GD)
    return fail(QPB_ERR_INVALID_ARG, "unknown ref mode %d", d->mode);
  if (d->n > QPB_REF_MAX_N) return fail(QPB_ERR_UNSUPPORTED, "qpb_ref_solve: n=%d > %d", d->n, QPB_REF_MAX_N);
  return 0;
}

extern "C" int qpb_ref_solve(const qpb_ref_desc *d, const double *P, const double *q, const double *x0,
                             double *x, int32_t *iters, void *stream) {
  int rc = check_ref(d);
  if (rc) return rc;
  if (d->batch == 0) return 0;
  if (!P || !q || !x || (!x0 && d->mode != QPB_REF_ADMM)) return fail(QPB_ERR_INVALID_ARG, "P, q, x0, x required");
  rc = check_device();
  if (rc) return rc;
  // n <= 64: one 64-thread workgroup per QP, at most 2^25 QPs per launch
  // (n > 64: a grid of one workgroup per CU walks the batch)
  const long long n = d->n, step = 1LL << 25;
  for (long long k0 = 0; k0 < d->batch; k0 += step) {
    qpb_ref_desc c = *d;
    c.batch = d->batch - k0 < step ? d->batch - k0 : step;
    hipError_t e = qpb_launch_ref(&c, P + k0 * n * n, q + k0 * n, x0 ? x0 + k0 * n : x0, x + k0 * n,
                                  iters ? iters + k0 : iters, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "qpb_ref_solve launch");
  }
  return 0;
}

extern "C" int qpb_ref_solve_host(const qpb_ref_desc *d, const double *P, const double *q, const double *x0,
                                  double *x, int32_t *iters) {
  int rc = check_ref(d);
  if (rc) return rc;
  if (d->batch == 0) return 0;
  rc = check_device();
  if (rc) return rc;
  const size_t B = (size_t)d->batch, n = d->n;
  DevBuf dP, dq, dx0, dx, di;
  HIPCHK(up(dP, P, B * n * n * 8), "P");
  HIPCHK(up(dq, q, B * n * 8), "q");
  HIPCHK(up(dx0, x0, B * n * 8), "x0");
  HIPCHK(alloc(dx, x, B * n * 8), "x");
  HIPCHK(alloc(di, iters, B * 4), "iters");
  rc = qpb_ref_solve(d, (double *)dP.p, (double *)dq.p, (double *)dx0.p, (double *)dx.p, (int32_t *)di.p,
                     nullptr);
  if (rc) return rc;
  HIPCHK(hipDeviceSynchronize(), "qpb_ref_solve_host kernel");
  HIPCHK(down(x, dx, B * n * 8), "x D2H");
  HIPCHK(down(iters, di, B * 4), "iters D2H");
  return 0;
}

extern "C" int qpb_matrix_invert(int32_t n, int64_t batch, const double *P, double *Pinv, void *stream) {
  if (n < 1 || batch < 0) return fail(QPB_ERR_INVALID_ARG, "bad qpb_matrix_invert arguments");
  if (n > QPB_REF_MAX_N) return fail(QPB_ERR_UNSUPPORTED, "qpb_matrix_invert: n=%d > %d", n, QPB_REF_MAX_N);
  if (batch == 0) return 0;
  if (!P || !Pinv) return fail(QPB_ERR_INVALID_ARG, "P and Pinv are required");
  int rc = check_device();
  if (rc) return rc;
  const long long nn = (long long)n * n, step = 1LL << 25;  // one 64-thread workgroup per matrix
  for (long long k0 = 0; k0 < batch; k0 += step) {
    const long long c = batch - k0 < step ? batch - k0 : step;
    hipError_t e = qpb_launch_ref_invert(n, c, P + k0 * nn, Pinv + k0 * nn, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "qpb_matrix_invert launch");
  }
  return 0;
}

extern "C" int qpb_qf_eval(int32_t n, int64_t batch, const double *P, const double *q, double r, const double *x,
                           double *out, void *stream) {
  if (n < 1 || batch < 0 || !P || !q || !x || !out) return fail(QPB_ERR_INVALID_ARG, "bad qpb_qf_eval arguments");
  if (batch == 0) return 0;
  int rc = check_device();
  if (rc) return rc;
  hipError_t e = qpb_launch_qf_eval(n, batch, P, q, r, x, out, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "qpb_qf_eval launch");
  return 0;
}

extern "C" int qpb_ref_generate(const qpb_ref_gen_desc *d, double *P, double *q, double *x0, void *stream) {
  if (!d) return fail(QPB_ERR_INVALID_ARG, "desc is NULL");
  if (d->n < 1 || d->batch < 0) return fail(QPB_ERR_INVALID_ARG, "n must be >= 1 and batch >= 0");
  if (d->n > QPB_MAX_N) return fail(QPB_ERR_UNSUPPORTED, "qpb_ref_generate: n=%d > %d", d->n, QPB_MAX_N);
  if (d->batch > (1LL << 25))  // one 64-thread workgroup per QP: 2^32 work-items per launch
    return fail(QPB_ERR_UNSUPPORTED, "batch > 2^25 QPs per generator call (split it with `first`)");
  if (d->batch > 0 && (!P || !q || !x0)) return fail(QPB_ERR_INVALID_ARG, "NULL output pointer");
  int rc = check_device();
  if (rc) return rc;
  const double range[6] = {d->p_min, d->p_max, d->q_min, d->q_max, d->x_min, d->x_max};
  hipError_t e = qpb_launch_ref_generate(d->n, d->batch, d->first, d->seed, range, P, q, x0, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "qpb_ref_generate launch");
  return 0;
}

extern "C" int qpb_generate(const qpb_gen_desc *d, double *H, double *f, double *A, double *b, void *stream) {
  if (!d) return fail(QPB_ERR_INVALID_ARG, "desc is NULL");
  if (d->n < 1 || d->m < 1 || d->batch < 0) return fail(QPB_ERR_INVALID_ARG, "n, m must be >= 1 and batch >= 0");
  if (d->family != QPB_FAMILY_BOX && d->family != QPB_FAMILY_DENSE)
    return fail(QPB_ERR_INVALID_ARG, "unknown family %d", d->family);
  if (d->family == QPB_FAMILY_BOX && d->m != 2 * d->n)
    return fail(QPB_ERR_INVALID_ARG, "the box family has m = 2n (got n=%d m=%d)", d->n, d->m);
  if (d->n > 128) return fail(QPB_ERR_UNSUPPORTED, "qpb_generate: n=%d > 128", d->n);
  if (d->n > 16 && d->m < d->n) return fail(QPB_ERR_UNSUPPORTED, "qpb_generate: n > 16 needs m >= n");
  if (d->batch > (1LL << 25))  // one 64-thread workgroup per QP: 2^32 work-items per launch
    return fail(QPB_ERR_UNSUPPORTED, "batch > 2^25 QPs per generator call (split it with `first`)");
  if (d->batch > 0 && (!H || !f || !A || !b)) return fail(QPB_ERR_INVALID_ARG, "NULL output pointer");
  int rc = check_device();
  if (rc) return rc;
  hipError_t e = qpb_launch_generate(d->n, d->m, d->batch, d->first, d->seed, d->family, d->shift, d->box, H, f, A,
                                     b, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "qpb_generate launch");
  return 0;
}

extern "C" int qpb_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return 0;
  return c;
}

extern "C" int qpb_set_device(int device) {
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  return 0;
}

extern "C" int qpb_synchronize(void *stream) {
  hipError_t e = stream ? hipStreamSynchronize((hipStream_t)stream) : hipDeviceSynchronize();
  if (e != hipSuccess) return hip_fail(e, "synchronize");
  return 0;
}

extern "C" const char *qpb_last_error(void) { return g_err; }

// the hot kernel revision is part of the string: profiles/pmc_traffic.json is
// only trusted for the revision it was measured on (bench.py)
extern "C" const char *qpb_version(void) { return "qpb 0.12 (gfx950; gi_dense v11.5: dual steepest-edge select -s/|D[r,q:]| with a nonzero key floor, dependency scale clamped to FLT_MAX, setup slacks from the sweep's DPP-read f, output stores under the A-row loads, DPP-fused slack product and Householder update, Householder product as u + alpha D[:,q], exact ratio step, one-trip loads and x gather, 3 waves/SIMD and 12 per CU (12,608 B of LDS per wave: the exchange row in R's column 0, Givens parameters in registers), built without machine LICM; gi_box v2.2: lb <= x <= ub, A implicit, dual steepest-edge select with a nonzero key floor, DPP-fused slack and Householder products, one-pass R column shift, 12 waves per CU; gi_wave v6.7 (+ BOX, n <= 32; absent bounds as +inf slacks): x solves with the components captured in LDS (no lane masks, no SGPR spills), dual steepest-edge select with a nonzero key floor, ratio reduction only when a partial step is possible, active A rows for x gathered 16 at a time, DPP-fused sweep, slack product, Householder update and back substitution (no LDS vector reads), Householder product as u + alpha D[:,q], odd-stride R with the exchange row in its column 0 (12 waves per CU), one-trip A gather for x, split setup sweep, 3 waves/SIMD; gi_gram v4.5 (+ BOX, n <= 128: qpb_solve_box with A generated in place) n<=128 on fp64 MFMA, no next-QP prefetch, lane ids opaque per iteration (2 VGPR spills instead of 29), active set as Q1 rows and Z = R^{-1} (parallel passes only), |u|^2 published with the key, broadcast row products, conflict-free diagonal-tile inverses, one-trip loads, cached workspace launched under its lock; ref v6: n <= 1024 (above 128: 1024-thread workgroups, the matrices in a global workspace slice), 64 < n <= 128 one LDS matrix per workgroup (LU, W / V, P in turn), LU rows staged for the solves, branch-free chunked sums)"; }
