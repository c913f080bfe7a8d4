/*
 * oracle/ref_driver.c -- TEST INFRASTRUCTURE ONLY (checker, never shipped).
 *
 * A thin C driver linked against the UNMODIFIED reference sources under
 * /root/reference (compiled by oracle/Makefile into oracle/_ref/, never copied
 * into this repo).  It exposes plain-pointer entry points so the Python
 * oracle / fixture generator / bench CPU baseline can call the reference's own
 * generator and solvers:
 *
 *   generator  : matirx_random_pos_def + matrix_random in the order of
 *                main.c:37-39 (P, q, x0), seeded with srand (main.c:11)
 *   solvers    : gradient_descent_with_line_search  (qp_solvers.c:65-101)
 *                newton_method_with_line_search     (qp_solvers.c:103-144)
 *                admm                               (qp_solvers.c:255-319)
 *   matrix ops : matrix_invert (matrix_ops.c:551-630), quadratic_form_eval
 *                (qp.c:9-27)
 *
 * N_DIM and the ADMM box are compile-time constants of the reference
 * (config.h:5, :29-30); oracle/Makefile builds one .so per (N_DIM, box).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
 */
#include <stdlib.h>
#include <string.h>

#include "matrix_ops.h"
#include "qp.h"
#include "qp_solvers.h"

static int g_inited;

static void ensure_init(void)
{
	if (!g_inited) {
		kmalloc_init(); /* main.c:10 -- pools are static, init exactly once */
		g_inited = 1;
	}
}

unsigned ref_ndim(void) { return N_DIM; }
double ref_box_max(void) { return ADMM_BOX_CONSTRAINT_MAX; }
double ref_box_min(void) { return ADMM_BOX_CONSTRAINT_MIN; }
void ref_srand(unsigned seed) { srand(seed); }
int ref_rand(void) { return rand(); }

static void put(struct _matrix *m, const double *src)
{
	unsigned r = MATRIX_GET_ROW(m), c = MATRIX_GET_COL(m);
	memcpy(m->elements, src, sizeof(double) * r * c);
}

static void get(double *dst, struct _matrix *m)
{
	unsigned r = MATRIX_GET_ROW(m), c = MATRIX_GET_COL(m);
	memcpy(dst, m->elements, sizeof(double) * r * c);
}

/* count QPs drawn exactly as main.c:37-39 draws them (P, then q, then x0) */
void ref_gen_qps(unsigned count, double pmin, double pmax, double qmin,
		 double qmax, double xmin, double xmax, double *P, double *q,
		 double *x0)
{
	ensure_init();
	struct _matrix *p = matrix_alloc(NxN);
	struct _matrix *qq = matrix_alloc(Nx1);
	struct _matrix *xx = matrix_alloc(Nx1);
	for (unsigned i = 0; i < count; i++) {
		matirx_random_pos_def(p, pmin, pmax);
		matrix_random(qq, qmin, qmax);
		matrix_random(xx, xmin, xmax);
		get(P + (size_t)i * N_DIM * N_DIM, p);
		get(q + (size_t)i * N_DIM, qq);
		get(x0 + (size_t)i * N_DIM, xx);
	}
	matrix_free(xx);
	matrix_free(qq);
	matrix_free(p);
}

void ref_invert(double *M)
{
	ensure_init();
	struct _matrix *m = matrix_alloc(NxN);
	put(m, M);
	matrix_invert(m);
	get(M, m);
	matrix_free(m);
}

double ref_eval(const double *P, const double *q, double r, const double *x)
{
	ensure_init();
	struct _matrix *p = matrix_alloc(NxN);
	struct _matrix *qq = matrix_alloc(Nx1);
	struct _matrix *xx = matrix_alloc(Nx1);
	put(p, P);
	put(qq, q);
	put(xx, x);
	struct _quadratic_form *qf = quadratic_form_alloc(p, qq, r);
	double v = quadratic_form_eval(qf, xx);
	quadratic_form_free(qf);
	matrix_free(xx);
	matrix_free(qq);
	matrix_free(p);
	return v;
}

typedef struct _matrix *(*solver_fn)(struct _matrix *, unsigned,
				     struct _quadratic_form *);

/* count QPs, each P n*n / q n / x0 n contiguous; writes x (count*n) */
static void run_batch(solver_fn fn, unsigned count, const double *P,
		      const double *q, const double *x0, unsigned iterations,
		      double *x)
{
	ensure_init();
	struct _matrix *p = matrix_alloc(NxN);
	struct _matrix *qq = matrix_alloc(Nx1);
	struct _matrix *xx = matrix_alloc(Nx1);
	struct _quadratic_form *qf = quadratic_form_alloc(p, qq, 0);
	for (unsigned i = 0; i < count; i++) {
		put(p, P + (size_t)i * N_DIM * N_DIM);
		put(qq, q + (size_t)i * N_DIM);
		put(xx, x0 + (size_t)i * N_DIM);
		struct _matrix *res = fn(xx, iterations, qf); /* test.c:97 */
		get(x + (size_t)i * N_DIM, res);
		matrix_free(res);
	}
	quadratic_form_free(qf);
	matrix_free(xx);
	matrix_free(qq);
	matrix_free(p);
}

void ref_newton_batch(unsigned count, const double *P, const double *q,
		      const double *x0, unsigned iterations, double *x)
{
	run_batch(newton_method_with_line_search, count, P, q, x0, iterations, x);
}

void ref_admm_batch(unsigned count, const double *P, const double *q,
		    const double *x0, unsigned iterations, double *x)
{
	run_batch(admm, count, P, q, x0, iterations, x);
}

void ref_gd_batch(unsigned count, const double *P, const double *q,
		  const double *x0, unsigned iterations, double *x)
{
	run_batch(gradient_descent_with_line_search, count, P, q, x0,
		  iterations, x);
}
