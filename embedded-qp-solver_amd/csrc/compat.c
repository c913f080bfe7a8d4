/*
 * compat.c -- the reference's single-QP C API (qp.h, qp_solvers.h,
 * matrix_ops.h, kmalloc.h of YangLingyuan/Embedded-qp-solver) re-implemented
 * on top of the batched C-ABI, so a reference caller (its main.c /
 * test/test.c) builds against include/compat and links libqpb.so unchanged.
 *
 *   solvers      gradient_descent_with_line_search / newton_method_with_line_search
 *                / admm  ->  qpb_ref_solve_host(batch = 1): the GPU
 *                reference-semantics kernels (qpb_ref.hip).  No CPU solver.
 *   objects      kmalloc pools, struct _matrix, struct _quadratic_form: host
 *                memory with the reference's layouts (matrix_type.h, qp.h).
 *   matrix ops   single-matrix host utilities with the reference's semantics
 *                (row-major, sequential sums, partial-pivot LU inverse).
 *
 * N_DIM and the ADMM box are compile-time constants of the reference; the
 * library takes them at kmalloc_init() (a macro for qpb_compat_init in
 * kmalloc.h), so one library serves every N_DIM.  Not thread-safe, like the
 * reference (global pools).
 */
#define _DEFAULT_SOURCE /* initstate / setstate */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "matrix_ops.h"
#include "qp.h"
#include "qp_solvers.h"
#include "qpb.h"

#undef kmalloc_init

/* ---------------------------------------------------------------- pools */
#define POOL_NXN 64
#define POOL_NX1 256
#define POOL_QF 16

struct slot {
	union {
		struct _matrix m;
		struct _quadratic_form qf;
	} v;
	int used;
};

static unsigned g_ndim = 48;
static double g_box_min = -1e12, g_box_max = 1e12;
static int g_init;
static struct slot g_nxn[POOL_NXN], g_nx1[POOL_NX1], g_qf[POOL_QF];
static double *g_nxn_store, *g_nx1_store;

/* The sanitizer build (Makefile target asan) gives every pool matrix its own
 * heap block, so an access past one matrix's elements is a heap overflow
 * AddressSanitizer reports, not a silent read of the neighbouring matrix. */
#if defined(__SANITIZE_ADDRESS__)
#define QPB_POOL_PER_SLOT 1
#elif defined(__has_feature)
#if __has_feature(address_sanitizer)
#define QPB_POOL_PER_SLOT 1
#endif
#endif
#ifndef QPB_POOL_PER_SLOT
#define QPB_POOL_PER_SLOT 0
#endif

static void pool_release(void)
{
#if QPB_POOL_PER_SLOT
	if (g_init) {
		for (int i = 0; i < POOL_NXN; i++)
			free(g_nxn[i].v.m.elements);
		for (int i = 0; i < POOL_NX1; i++)
			free(g_nx1[i].v.m.elements);
	}
#endif
	free(g_nxn_store);
	free(g_nx1_store);
	g_nxn_store = g_nx1_store = NULL;
}

void qpb_compat_init(unsigned n_dim, double admm_box_min, double admm_box_max)
{
	/* The reference packs N_DIM into 16 bits (matrix_type.h:14-17): its host
	 * matrix library (matrix_mult, matrix_invert, matrix_norm, the pools)
	 * works at any N_DIM up to 65535, and so does this one.  Only the three
	 * qp_solvers.h solvers run on the batched GPU replicas, which take
	 * n <= QPB_REF_MAX_N (1024); they refuse a larger N_DIM with the reason (run_ref). */
	if (n_dim == 0 || n_dim > 0xFFFFu) {
		fprintf(stderr, "kmalloc_init: N_DIM = %u is outside 1..65535 (the 16-bit dimension fields of "
				"struct _matrix, matrix_type.h)\n", n_dim);
		exit(EXIT_FAILURE);
	}
	pool_release();
	g_ndim = n_dim;
	g_box_min = admm_box_min;
	g_box_max = admm_box_max;
#if !QPB_POOL_PER_SLOT
	g_nxn_store = calloc((size_t)POOL_NXN * n_dim * n_dim, sizeof(double));
	g_nx1_store = calloc((size_t)POOL_NX1 * n_dim, sizeof(double));
	if (!g_nxn_store || !g_nx1_store) {
		/* the reference's pools are static arrays sized by N_DIM: a size
		 * that does not fit is fatal there too */
		fprintf(stderr, "kmalloc_init: N_DIM = %u: the matrix pools (%d n x n, %d n x 1) do not fit in memory\n",
			n_dim, POOL_NXN, POOL_NX1);
		exit(EXIT_FAILURE);
	}
#endif
	for (int i = 0; i < POOL_NXN; i++) {
		g_nxn[i].used = 0;
		g_nxn[i].v.m.elements = QPB_POOL_PER_SLOT ? calloc((size_t)n_dim * n_dim, sizeof(double))
							  : g_nxn_store + (size_t)i * n_dim * n_dim;
	}
	for (int i = 0; i < POOL_NX1; i++) {
		g_nx1[i].used = 0;
		g_nx1[i].v.m.elements = QPB_POOL_PER_SLOT ? calloc(n_dim, sizeof(double))
							  : g_nx1_store + (size_t)i * n_dim;
	}
	for (int i = 0; i < POOL_QF; i++)
		g_qf[i].used = 0;
	g_init = 1;
}

void kmalloc_init(void)
{
	qpb_compat_init(48, -1e12, 1e12);
}

static struct slot *pool_of(enum kmalloc_type type, int *cap)
{
	switch (type) {
	case NxN:
		*cap = POOL_NXN;
		return g_nxn;
	case Nx1:
		*cap = POOL_NX1;
		return g_nx1;
	case QUADRATIC_FORM:
		*cap = POOL_QF;
		return g_qf;
	default:
		*cap = 0;
		return NULL;
	}
}

void *kmalloc(enum kmalloc_type type, unsigned flags)
{
	int cap;
	struct slot *p = pool_of(type, &cap);
	if (!p || !g_init)
		return NULL; /* unknown type, or kmalloc_init() not called */
	for (int i = 0; i < cap; i++) {
		if (p[i].used)
			continue;
		p[i].used = 1;
		if (KM_ZERO & flags) {
			if (type == QUADRATIC_FORM)
				memset(&p[i].v.qf, 0, sizeof(p[i].v.qf));
			else
				memset(p[i].v.m.elements, 0,
				       sizeof(double) * (type == NxN ? g_ndim * g_ndim : g_ndim));
		}
		return &p[i].v;
	}
	return NULL; /* pool exhausted */
}

void kfree(void *me, enum kmalloc_type type)
{
	int cap;
	struct slot *p = pool_of(type, &cap);
	if (!me || !p)
		return;
	for (int i = 0; i < cap; i++)
		if ((void *)&p[i].v == me)
			p[i].used = 0;
}

/* ------------------------------------------------------------- matrices */
struct _matrix *matrix_alloc(enum kmalloc_type type)
{
	if (type != NxN && type != Nx1) {
		fprintf(stderr, "no such matrix type to allocate in matrix_alloc\n");
		return NULL;
	}
	struct _matrix *m = kmalloc(type, 0);
	if (!m) {
		fprintf(stderr, "no matrix to allocate in matrix_alloc\n");
		return NULL;
	}
	m->dimensions = 0;
	MATRIX_SET_ROW(m, g_ndim);
	MATRIX_SET_COL(m, type == NxN ? g_ndim : 1U);
	return m;
}

void matrix_free(struct _matrix *m)
{
	if (!m)
		return;
	unsigned r = MATRIX_GET_ROW(m), c = MATRIX_GET_COL(m);
	if (r == g_ndim && c == g_ndim)
		kfree(m, NxN);
	else if ((r == g_ndim && c == 1) || (r == 1 && c == g_ndim))
		kfree(m, Nx1);
	else
		fprintf(stderr, "no such matrix type in matrix_free\n");
}

static unsigned offset(struct _matrix *m, struct _matrix_entry e)
{
	return e.row * MATRIX_GET_COL(m) + e.col;
}

double matrix_get_entry(struct _matrix *m, struct _matrix_entry e)
{
	return m->elements[offset(m, e)];
}

void matrix_set_entry(struct _matrix *m, struct _matrix_entry e, double val)
{
	m->elements[offset(m, e)] = val;
}

static unsigned numel(struct _matrix *m)
{
	return MATRIX_GET_ROW(m) * MATRIX_GET_COL(m);
}

/* a_ij = s * b_ij */
static void scale_into(struct _matrix *a, struct _matrix *b, double s)
{
	unsigned k = numel(a);
	for (unsigned i = 0; i < k; i++)
		a->elements[i] = s * b->elements[i];
}

void matrix_scalar_mult(struct _matrix *m, double s) { scale_into(m, m, s); }
void matrix_copy(struct _matrix *a, struct _matrix *b) { scale_into(a, b, 1.0); }
void matrix_zero_up(struct _matrix *m) { scale_into(m, m, 0.0); }
void matrix_neg(struct _matrix *m) { scale_into(m, m, -1.0); }

void matrix_identity(struct _matrix *m)
{
	unsigned r = MATRIX_GET_ROW(m), c = MATRIX_GET_COL(m);
	memset(m->elements, 0, sizeof(double) * r * c);
	for (unsigned i = 0; i < r && i < c; i++)
		m->elements[i * c + i] = 1.0;
}

void matrix_mult(struct _matrix *prod, struct _matrix *a, struct _matrix *b)
{
	unsigned rows = MATRIX_GET_ROW(prod), cols = MATRIX_GET_COL(prod), kk = MATRIX_GET_COL(a);
	unsigned ac = MATRIX_GET_COL(a), bc = MATRIX_GET_COL(b);
	for (unsigned i = 0; i < rows; i++)
		for (unsigned j = 0; j < cols; j++) {
			double acc = 0;
			for (unsigned k = 0; k < kk; k++)
				acc += a->elements[i * ac + k] * b->elements[k * bc + j];
			prod->elements[i * cols + j] = acc;
		}
}

/* the four vector shapes the reference accepts (Nx1/1xN x Nx1/1xN) */
double matrix_scalar_prod(struct _matrix *a, struct _matrix *b)
{
	unsigned ar = MATRIX_GET_ROW(a), ac = MATRIX_GET_COL(a);
	unsigned br = MATRIX_GET_ROW(b), bc = MATRIX_GET_COL(b);
	unsigned la = (ac == 1 && ar > 1) ? ar : ((ar == 1 && ac > 1) ? ac : 0);
	unsigned lb = (bc == 1 && br > 1) ? br : ((br == 1 && bc > 1) ? bc : 0);
	if (!la || la != lb) {
		fprintf(stderr, "invalid arguments in matrix_scalar_prod: no combination of dimensions matches\n");
		return 0;
	}
	double acc = 0;
	for (unsigned k = 0; k < la; k++)
		acc += a->elements[k] * b->elements[k];
	return acc;
}

enum { OP_SUB, OP_ADD, OP_MAX, OP_MIN };

static void elementwise(struct _matrix *s, struct _matrix *a, struct _matrix *b, int op)
{
	unsigned k = numel(s);
	for (unsigned i = 0; i < k; i++) {
		double x = a->elements[i], y = b->elements[i];
		double v = op == OP_ADD ? x + y : op == OP_SUB ? x - y : op == OP_MAX ? (x > y ? x : y) : (x > y ? y : x);
		s->elements[i] = v;
	}
}

void matrix_add(struct _matrix *s, struct _matrix *a, struct _matrix *b) { elementwise(s, a, b, OP_ADD); }
void matrix_sub(struct _matrix *s, struct _matrix *a, struct _matrix *b) { elementwise(s, a, b, OP_SUB); }
void matrix_max(struct _matrix *s, struct _matrix *a, struct _matrix *b) { elementwise(s, a, b, OP_MAX); }
void matrix_min(struct _matrix *s, struct _matrix *a, struct _matrix *b) { elementwise(s, a, b, OP_MIN); }

/* in-place transpose; entries move only when both dimensions exceed 1 */
void matrix_trans(struct _matrix *m)
{
	unsigned r = MATRIX_GET_ROW(m), c = MATRIX_GET_COL(m);
	MATRIX_SET_ROW(m, c);
	MATRIX_SET_COL(m, r);
	if (r == 1 || c == 1)
		return;
	for (unsigned i = 0; i < r; i++)
		for (unsigned j = i + 1; j < c; j++) {
			double t = m->elements[i * c + j];
			m->elements[i * c + j] = m->elements[j * c + i];
			m->elements[j * c + i] = t;
		}
}

/* explicit inverse: partial-pivot LU (first strict maximum pivots, physical
 * row swaps), then one forward / back substitution per identity column */
void matrix_invert(struct _matrix *m)
{
	unsigned n = MATRIX_GET_ROW(m);
	double *a = m->elements;
	unsigned *perm = malloc(sizeof(unsigned) * n);
	double *w = malloc(sizeof(double) * n), *v = malloc(sizeof(double) * n);
	double *inv = malloc(sizeof(double) * n * n);
	if (!perm || !w || !v || !inv) {
		fprintf(stderr, "out of memory in matrix_invert\n");
		free(perm), free(w), free(v), free(inv);
		return;
	}
	for (unsigned k = 0; k < n; k++)
		perm[k] = k;
	for (unsigned k = 0; k + 1 < n; k++) {
		double piv = 0;
		unsigned pi = 0;
		for (unsigned i = k; i < n; i++) {
			double t = fabs(a[i * n + k]);
			if (t > piv) {
				piv = t;
				pi = i;
			}
		}
		if (piv == 0) {
			fprintf(stderr, "singular matrix in matrix_invert\n");
			break;
		}
		unsigned tp = perm[pi];
		perm[pi] = perm[k];
		perm[k] = tp;
		for (unsigned j = 0; j < n; j++) {
			double t = a[pi * n + j];
			a[pi * n + j] = a[k * n + j];
			a[k * n + j] = t;
		}
		for (unsigned i = k + 1; i < n; i++) {
			double l = a[i * n + k];
			l /= a[k * n + k];
			a[i * n + k] = l;
			for (unsigned j = k + 1; j < n; j++) {
				double t = a[i * n + j];
				t -= a[i * n + k] * a[k * n + j];
				a[i * n + j] = t;
			}
		}
	}
	for (unsigned i = 0; i < n; i++) {
		for (unsigned r = 0; r < n; r++) {
			double t = 0;
			for (unsigned k = 0; k < r; k++)
				t += a[r * n + k] * w[k];
			w[r] = (perm[r] == i ? 1.0 : 0.0) - t;
		}
		for (unsigned r = n; r-- > 0;) {
			double t = 0;
			for (unsigned k = r + 1; k < n; k++)
				t += a[r * n + k] * v[k];
			v[r] = (w[r] - t) / a[r * n + r];
		}
		for (unsigned r = 0; r < n; r++)
			inv[r * n + i] = v[r];
	}
	memcpy(a, inv, sizeof(double) * n * n);
	free(perm), free(w), free(v), free(inv);
}

/* 2-norm over the first N_DIM entries (the reference always sums N_DIM) */
double matrix_norm(struct _matrix *m)
{
	double acc = 0;
	for (unsigned k = 0; k < g_ndim; k++) {
		double t = m->elements[k];
		t *= t;
		acc += t;
	}
	return sqrt(acc);
}

void matrix_print(struct _matrix *m)
{
	unsigned r = MATRIX_GET_ROW(m), c = MATRIX_GET_COL(m);
	for (unsigned i = 0; i < r; i++) {
		for (unsigned j = 0; j < c; j++)
			printf("%e ", m->elements[i * c + j]);
		printf("\n");
	}
	printf("\n");
}

double random_number(double min, double max)
{
	double r = rand();
	return min + r * (max - min) / RAND_MAX;
}

void matrix_random(struct _matrix *m, double min, double max)
{
	unsigned k = numel(m);
	for (unsigned i = 0; i < k; i++)
		m->elements[i] = random_number(min, max);
}

/* P = B^T B / (max * rows), B ~ U[min, max] row-major (exactly symmetric) */
void matirx_random_pos_def(struct _matrix *m, double min, double max)
{
	unsigned n = MATRIX_GET_ROW(m);
	double *b = malloc(sizeof(double) * n * n);
	if (!b) {
		fprintf(stderr, "out of memory in matrix_random_pos_def\n");
		return;
	}
	for (unsigned i = 0; i < n * n; i++)
		b[i] = random_number(min, max);
	for (unsigned i = 0; i < n; i++)
		for (unsigned j = 0; j < n; j++) {
			double acc = 0;
			for (unsigned k = 0; k < n; k++)
				acc += b[k * n + i] * b[k * n + j];
			m->elements[i * n + j] = acc;
		}
	double s = 1 / (double)(max * n);
	for (unsigned i = 0; i < n * n; i++)
		m->elements[i] = s * m->elements[i];
	free(b);
}

/* ------------------------------------------------------- quadratic form */
struct _quadratic_form *quadratic_form_alloc(struct _matrix *p, struct _matrix *q, double r)
{
	struct _quadratic_form *qf = kmalloc(QUADRATIC_FORM, 0);
	if (!qf) {
		fprintf(stderr, "no quadratic form available to alloc\n");
		return NULL;
	}
	qf->p = p;
	qf->q = q;
	qf->r = r;
	return qf;
}

void quadratic_form_free(struct _quadratic_form *qf) { kfree(qf, QUADRATIC_FORM); }

double quadratic_form_eval(struct _quadratic_form *qf, struct _matrix *x)
{
	unsigned n = MATRIX_GET_ROW(qf->p);
	double xa = 0;
	for (unsigned i = 0; i < n; i++) {
		double acc = 0;
		for (unsigned k = 0; k < n; k++)
			acc += qf->p->elements[i * n + k] * x->elements[k];
		xa += x->elements[i] * acc;
	}
	double a = 0.5 * xa;
	double qa = 0;
	for (unsigned k = 0; k < n; k++)
		qa += qf->q->elements[k] * x->elements[k];
	a += qa;
	a += qf->r;
	return a;
}

struct _matrix *quadratic_form_eval_grad(struct _quadratic_form *qf, struct _matrix *x)
{
	struct _matrix *g = matrix_alloc(Nx1);
	if (!g) {
		fprintf(stderr, "no matrix available to alloc in quadratic_form_eval_grad\n");
		return NULL;
	}
	matrix_mult(g, qf->p, x);
	matrix_add(g, g, qf->q);
	return g;
}

/* ------------------------------------------------------------- solvers */
static struct _matrix *run_ref(int mode, struct _matrix *x0, unsigned iterations, struct _quadratic_form *qf)
{
	if (MATRIX_GET_ROW(qf->p) > QPB_REF_MAX_N) {
		fprintf(stderr,
			"%s: N_DIM = %u: the qp_solvers.h solvers of this library run on the batched GPU replicas "
			"(qpb_ref_solve), which take n <= %d (qpb.h QPB_REF_MAX_N); the matrix_ops.h routines have no "
			"such limit\n",
			mode == QPB_REF_GD ? "gradient_descent_with_line_search"
					   : mode == QPB_REF_NEWTON ? "newton_method_with_line_search" : "admm",
			(unsigned)MATRIX_GET_ROW(qf->p), QPB_REF_MAX_N);
		exit(EXIT_FAILURE); /* the reference exits on its fatal errors (qp_solvers.c:79-82) */
	}
	struct _matrix *x = matrix_alloc(Nx1);
	if (!x)
		return NULL;
	qpb_ref_desc d;
	memset(&d, 0, sizeof(d));
	d.n = (int32_t)MATRIX_GET_ROW(qf->p);
	d.mode = mode;
	d.batch = 1;
	d.iterations = (int32_t)iterations;
	d.box_min = g_box_min;
	d.box_max = g_box_max;
	/* The HIP runtime may call srand()/rand() (first-use initialisation): run
	 * the GPU call on a private generator state so the caller's rand() stream
	 * -- which drives the reference's problem generator -- is untouched, as
	 * it is by the reference's CPU solvers. */
	static char private_state[256];
	char *caller_state = initstate(1u, private_state, sizeof(private_state));
	int rc = qpb_ref_solve_host(&d, qf->p->elements, qf->q->elements, x0 ? x0->elements : qf->q->elements,
				    x->elements, NULL);
	setstate(caller_state);
	if (rc) {
		fprintf(stderr, "qpb_ref_solve failed (%d): %s\n", rc, qpb_last_error());
		exit(EXIT_FAILURE); /* the reference exits on a NULL gradient too (qp_solvers.c:79-82) */
	}
	return x;
}

struct _matrix *gradient_descent_with_line_search(struct _matrix *x0, unsigned iterations,
						  struct _quadratic_form *qf)
{
	return run_ref(QPB_REF_GD, x0, iterations, qf);
}

struct _matrix *newton_method_with_line_search(struct _matrix *x0, unsigned iterations,
					       struct _quadratic_form *qf)
{
	return run_ref(QPB_REF_NEWTON, x0, iterations, qf);
}

struct _matrix *admm(struct _matrix *x0, unsigned iterations, struct _quadratic_form *qf)
{
	return run_ref(QPB_REF_ADMM, x0, iterations, qf);
}
