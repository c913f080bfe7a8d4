/*
 * qpb.h -- batched dense QP solver for AMD MI355X (gfx950): the C-ABI.
 *
 * Plain C, plain pointers and sizes.  This is the drop-in boundary for the
 * reference's hot path (YangLingyuan/Embedded-qp-solver):
 *
 *   reference (one QP, CPU, fp64)                       replaced by
 *   --------------------------------------------------  ----------------------
 *   qp_solvers.h:4-16  gradient_descent_with_line_search qpb_ref_solve(QPB_REF_GD)
 *                      newton_method_with_line_search    qpb_ref_solve(QPB_REF_NEWTON)
 *                      admm (box = config.h:29-30)       qpb_ref_solve(QPB_REF_ADMM)
 *   test/qp_ref.py:35  solve_qp(P, q, G=0, h=0)          qpb_solve(m = 0)
 *   north_star active-set over (H, f, A, b)              qpb_solve(m > 0)
 *   (absent from the reference: SURVEY.md §0)
 *   qp.h:19-24         quadratic_form_eval / _eval_grad  qpb_qf_eval
 *
 * The single-QP reference API itself (qp.h, qp_solvers.h, matrix_ops.h,
 * kmalloc.h, matrix_type.h) is re-exported, layout-compatible, by the compat
 * headers in include/compat/ on top of these entry points.
 *
 * Problem (per QP, fp64):   min 1/2 x^T H x + f^T x   s.t.   A x <= b
 *   H  n x n row-major, symmetric positive definite (the reference's P,
 *      qp.h:8-13; must be symmetric -- the kernels read the full matrix)
 *   f  n        (the reference's q)
 *   A  m x n row-major, b  m   (a box lb <= x <= ub is A = [I; -I], b = [ub; -lb])
 * Batched layout: QP k's arrays are contiguous at H + k*n*n, f + k*n,
 * A + k*m*n, b + k*m (array-of-structures, the reference's row-major
 * struct _matrix elements, matrix_type.h:20-23, one after another).
 *
 * Outputs:
 *   x       n per QP
 *   lam     m per QP: Lagrange multipliers, H x + f + A^T lam = 0, lam >= 0
 *   active  ceil(m/32) uint32 words per QP: bit i set <=> row i in the final
 *           active set
 *   status  one int32 per QP (qpb_status); never aborts the batch
 *   iters   one int32 per QP (active-set iterations), may be NULL
 *
 * All array pointers passed to qpb_solve / qpb_ref_solve are DEVICE pointers
 * (hipMalloc'd or torch CUDA tensors) and the call is asynchronous on
 * `stream` (a hipStream_t, NULL = default stream).  The *_host variants take
 * host pointers and synchronise.
 * Return value: 0 on success, a negative qpb_error on an invalid call.
 * Thread-safe: no global state besides the per-thread last-error string.
 */
#ifndef QPB_H
#define QPB_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* qpb_version() reports "qpb MAJOR.MINOR (...)" */
#define QPB_VERSION_MAJOR 0
#define QPB_VERSION_MINOR 12

/* limits of this build's kernels: n <= 16, m <= 32 one QP per 16-lane DPP
 * row (qpb_gi.hip); n <= 32, m <= 64 one QP per wavefront (qpb_gi_wave.hip);
 * n <= 128, m <= 256 one QP per 512-thread workgroup, one workgroup per CU
 * walking the batch (qpb_gi_gram.hip) */
#define QPB_MAX_N 128
#define QPB_MAX_M 256
/* the reference-semantics replicas (qpb_ref_solve, qpb_matrix_invert) and the
 * compat solvers on them: n <= 1024 (above 128 the matrices live in a global
 * workspace, one 1024-thread workgroup per QP, qpb_ref.hip) */
#define QPB_REF_MAX_N 1024

typedef enum qpb_status {
	QPB_OK = 0,         /* KKT point found (within feas_tol) */
	QPB_MAX_ITER = 1,   /* iteration cap reached */
	QPB_NOT_SPD = 2,    /* Cholesky of H failed (pivot <= 0) */
	QPB_INFEASIBLE = 3, /* constraints proven infeasible */
	QPB_NUMERICAL = 4   /* non-finite result */
} qpb_status;

typedef enum qpb_error {
	QPB_SUCCESS = 0,
	QPB_ERR_INVALID_ARG = -1,
	QPB_ERR_UNSUPPORTED = -2, /* size outside this build's kernels */
	QPB_ERR_HIP = -3,         /* HIP runtime error (see qpb_last_error) */
	QPB_ERR_NO_DEVICE = -4
} qpb_error;

/* diagnostic flag: every QP k reads the inputs of QP (k mod 512) -- kernel
 * time without HBM latency (outputs are still written for every k) */
#define QPB_FLAG_DIAG_L2 1
/* flag values 4 and 8 (round-2 diagnostic builds of the n <= 16 kernel) are
 * retired: accepted and ignored */
/* diagnostic flag (n <= 16): every QP k reads the inputs of QP (k mod 16384),
 * a 107 MB working set that stays Infinity-Cache resident across launches */
#define QPB_FLAG_DIAG_MALL 16

/* n in (16, 32], m <= 64 (BASELINE configs[4]): mixed precision -- the
 * active set is found in fp32 (factorisation and iterations), then x and lam
 * are refined in fp64 on the KKT system of that active set (fp32 factors,
 * fp64 residuals) and verified in fp64 (feasibility of every row, lam >= 0,
 * converged refinement).  QPs that fail verification are re-solved by the
 * fp64 kernel in a second launch, so results meet the fp64 path's bars.
 * Ignored outside that size class. */
#define QPB_FLAG_MIXED 32
/* diagnostic flag (with QPB_FLAG_MIXED): skip the fp64 re-solve; QPs that
 * would be re-solved keep status 100 (measures the re-solve fraction) */
#define QPB_FLAG_DIAG_NO_REDO 64

/* flag value 128 (the round-1 n <= 128 kernel) is retired: accepted and ignored */
/* diagnostic flag (n <= 16, m <= 32): solve with the one-QP-per-wavefront
 * kernel of the n <= 32 class (qpb_gi_wave.hip) instead of four QPs per
 * wavefront -- the group-size-1 endpoint of the lockstep model (DESIGN.md
 * §2.1); same answers within the parity bars, not a faster path */
#define QPB_FLAG_DIAG_WAVE 256

typedef struct qpb_desc {
	int32_t n;        /* variables, 1..QPB_MAX_N */
	int32_t m;        /* rows of A x <= b, 0..QPB_MAX_M (0: unconstrained) */
	int64_t batch;    /* number of QPs */
	int32_t max_iter; /* <= 0: default 4*(n+m)+8 */
	int32_t flags;    /* 0; QPB_FLAG_DIAG_L2 = diagnostic (see below) */
	double feas_tol;  /* <= 0: default 1e-10 (relative, per row) */
} qpb_desc;

/* Batched active-set solve (dual Goldfarb-Idnani method, one QP per 16-lane
 * row of a wavefront).  Device pointers; asynchronous on `stream`. */
int qpb_solve(const qpb_desc *desc, const double *H, const double *f,
	      const double *A, const double *b, double *x, double *lam,
	      uint32_t *active, int32_t *status, int32_t *iters, void *stream);

/* Same with host pointers (allocates device buffers, copies, synchronises). */
int qpb_solve_host(const qpb_desc *desc, const double *H, const double *f,
		   const double *A, const double *b, double *x, double *lam,
		   uint32_t *active, int32_t *status, int32_t *iters);

/* Box-constrained batched solve, lb <= x <= ub: the constraint class of the
 * reference's admm() (qp_solvers.c:146-319, bounds config.h:29-30), solved
 * exactly with A = [I; -I], b = [ub; -lb] kept implicit (qpb_gi_box.hip for
 * n <= 16, four QPs per wavefront; the BOX form of qpb_gi_wave.hip for
 * 16 < n <= 32, one QP per wavefront; the BOX form of qpb_gi_gram.hip for
 * 32 < n <= 128, one QP per workgroup).  Replaces admm()'s box QP the way
 * qpb_solve replaces the dense path.  desc->n <= QPB_MAX_N (128;
 * QPB_ERR_UNSUPPORTED above); desc->m must be 2n.  lb, ub: B x n, either may be NULL,
 * and +-inf entries are absent bounds.  lam: B x 2n (upper bounds' multipliers
 * first, then the lower bounds'); active: B x ceil(2n/32) uint32 words in the
 * same row order -- ONE word per QP for n <= 16, TWO for 16 < n <= 32, up to
 * EIGHT at n = 128 (size it as qpb_solve's ceil(m/32) with m = 2n; the n > 16
 * kernels write every word);
 * x, status, iters as qpb_solve.  Device pointers; asynchronous on `stream`. */
int qpb_solve_box(const qpb_desc *desc, const double *H, const double *f,
		  const double *lb, const double *ub, double *x, double *lam,
		  uint32_t *active, int32_t *status, int32_t *iters, void *stream);

/* Reference-semantics solvers (qp_solvers.c replicas). */
typedef enum qpb_ref_mode {
	QPB_REF_NEWTON = 1, /* qp_solvers.c:103-144 (explicit LU inverse, Armijo quirk) */
	QPB_REF_ADMM = 2,   /* qp_solvers.c:255-319 (rho = 1, alpha = 1, returns x) */
	QPB_REF_GD = 3      /* qp_solvers.c:65-101 */
} qpb_ref_mode;

typedef struct qpb_ref_desc {
	int32_t n;          /* variables (N_DIM of the reference) */
	int32_t mode;       /* qpb_ref_mode */
	int64_t batch;
	int32_t iterations; /* the reference's `iterations` argument */
	int32_t flags;      /* reserved, 0 */
	double box_min;     /* ADMM box (config.h:29-30 ADMM_BOX_CONSTRAINT_MIN/MAX) */
	double box_max;
} qpb_ref_desc;

/* P n*n, q n, x0 n per QP (device), 1 <= n <= QPB_REF_MAX_N; writes x n per
 * QP and the iteration count per QP (may be NULL).  x0 is ignored by ADMM, as in the reference
 * (qp_solvers.c:256). */
int qpb_ref_solve(const qpb_ref_desc *desc, const double *P, const double *q,
		  const double *x0, double *x, int32_t *iters, void *stream);

int qpb_ref_solve_host(const qpb_ref_desc *desc, const double *P,
		       const double *q, const double *x0, double *x,
		       int32_t *iters);

/* Batched matrix_invert (matrix_ops.c:551-630): Pinv = P^{-1} per matrix,
 * n <= 128, device pointers, n*n doubles each.  The reference's partial-pivot
 * LU (first strict maximum, physical row swaps, :434-536) and per-column
 * forward / back solves, unfused, in its order: bitwise equal to the
 * reference's result.  n <= QPB_REF_MAX_N.  A singular pivot stops the LU as in the reference
 * (:511-515); the result is then garbage, as there. */
int qpb_matrix_invert(int32_t n, int64_t batch, const double *P, double *Pinv,
		      void *stream);

/* f(x) = 1/2 x^T P x + q^T x + r per QP (qp.c:9-27), batched, device. */
int qpb_qf_eval(int32_t n, int64_t batch, const double *P, const double *q,
		double r, const double *x, double *out, void *stream);

/* Diagnostic: same solve (n = 16 with 16 < m <= 32, or 16 < n <= 32 with
 * m <= 64) by a build of the kernel with s_memrealtime stamps (100 MHz); adds
 * each wavefront's ticks per kernel section into row (workgroup index mod 256)
 * of sections[256][20] (zero it first; sum the rows for the totals).
 * sections_len is the device buffer's length in elements: below
 * QPB_SECTIONS_LEN the call fails with QPB_ERR_INVALID_ARG (no write).
 * n = 16: load, cholesky, substitution, init, select, exchange, back-solve,
 * step, add, drop, loop-exit, output.  16 < n <= 32: load, sweep, init,
 * select, exchange, back-solve, step, add, drop, loop-exit, x, stores. */
#define QPB_SECTIONS_LEN (256 * 20)
int qpb_solve_sections(const qpb_desc *desc, const double *H, const double *f,
		       const double *A, const double *b, double *x, double *lam,
		       uint32_t *active, int32_t *status, int32_t *iters,
		       unsigned long long *sections, int64_t sections_len, void *stream);

/* ------------------------------------------------------------------------
 * On-device input generators.
 *
 * qpb_ref_generate: the reference's generator bit for bit -- srand(seed),
 * then per QP P = matirx_random_pos_def (matrix_ops.c:699-734), q, x0 =
 * matrix_random (main.c:37-39 order), glibc TYPE_3 rand().  QPs
 * [first, first + batch) of that sequence (each QP jumps ahead to its own
 * offset), so any shard equals the same QPs of one sequential run.
 * P n*n, q n, x0 n per QP, device pointers.  1 <= n <= 128.             */
typedef struct qpb_ref_gen_desc {
	int32_t n;      /* N_DIM */
	uint32_t seed;  /* srand() argument */
	int64_t batch;
	uint64_t first; /* index of the first QP in the sequence */
	double p_min, p_max; /* random_pos_def range (main.c:37: -1e3, 1e3) */
	double q_min, q_max; /* q range (main.c:38) */
	double x_min, x_max; /* x0 range (main.c:39) */
} qpb_ref_gen_desc;

int qpb_ref_generate(const qpb_ref_gen_desc *desc, double *P, double *q, double *x0, void *stream);

/* qpb_generate: the benchmark families of SURVEY.md §8d from a counter-based
 * Philox4x32-10 stream keyed by (seed, QP index): QP first + k of any launch
 * is the same QP.  H = B^T B / (1e3 n) + shift I with B ~ U[-1e3, 1e3]^{n x n}
 * (product on the fp64 matrix cores), f ~ U[-1e3, 1e3];
 *   QPB_FAMILY_BOX:   A = [I; -I] (m = 2n), b = box
 *   QPB_FAMILY_DENSE: rows of A ~ N(0, I) normalised, b ~ U[0.1, 1) box
 * Device pointers H n*n, f n, A m*n, b m per QP.  1 <= n <= 128; for
 * n > 16, m >= n (B is staged in A's rows).                             */
typedef enum qpb_family { QPB_FAMILY_BOX = 0, QPB_FAMILY_DENSE = 1 } qpb_family;

typedef struct qpb_gen_desc {
	int32_t n, m;
	int64_t batch;
	uint64_t first; /* QP index of the first QP generated */
	uint64_t seed;
	int32_t family; /* qpb_family */
	int32_t flags;  /* reserved, 0 */
	double shift;   /* added to H's diagonal (0: the heavy-tailed "ref" family) */
	double box;     /* box half-width / b scale */
} qpb_gen_desc;

int qpb_generate(const qpb_gen_desc *desc, double *H, double *f, double *A, double *b, void *stream);

/* ------------------------------------------------------------------------
 * Wire format, host memory, native-endian fp64.
 * The reference's single QP (test/test.c:108-126 -> test/qp_ref.py:8-30):
 *     [n][P n*n][q n]
 * Batched:  [n][m][B] then B records [H n*n][f n][A m*n][b m].
 * qpb_wire_write emits the reference form when m == 0 and batch == 1; the
 * readers accept both (told apart by the file size).                    */
int qpb_wire_write(const char *path, int32_t n, int32_t m, int64_t batch, const double *H, const double *f,
		   const double *A, const double *b);
int qpb_wire_read_header(const char *path, int32_t *n, int32_t *m, int64_t *batch);
/* H B*n*n, f B*n, A B*m*n, b B*m host buffers sized from the header */
int qpb_wire_read(const char *path, double *H, double *f, double *A, double *b);

/* housekeeping */
int qpb_device_count(void);
int qpb_set_device(int device);
int qpb_synchronize(void *stream);
/* Scratch buffers are cached per (device, stream) and reused across calls
 * (the n <= 128 kernels and the reference replicas at n > 64 need one);
 * this synchronises those streams and frees them all.  The cache frees a
 * stream's buffer stream-ordered ON that stream, so release a stream's
 * buffer (qpb_release_stream_workspace) before destroying the stream.  Calls
 * from several host threads are safe, sharing a stream included: a buffer is
 * handed to a launch only while the cache is locked. */
int qpb_release_workspaces(void);
int qpb_release_stream_workspace(void *stream);
const char *qpb_last_error(void);
const char *qpb_version(void);

#ifdef __cplusplus
}
#endif

#endif /* QPB_H */
