/*
 * compat_driver.c -- a C caller of the reference-compatible API
 * (include/compat: kmalloc.h, matrix_ops.h, qp.h, qp_solvers.h), written the
 * way the reference's main.c drives it (kmalloc_init, srand, P -> q -> x0 per
 * QP, optimizer through a function pointer as test/test.c does), linked with
 * -lqpb.  Built with N_DIM=16.
 *
 *   compat_driver <solver> <seed> <count> <iterations>
 *     solver: newton | admm | gd | gen
 * writes, per QP, N_DIM doubles (the returned x; for "gen": P, q, x0) to stdout.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "matrix_ops.h"
#include "qp.h"
#include "qp_solvers.h"

typedef struct _matrix *(*opt_fn)(struct _matrix *, unsigned, struct _quadratic_form *);

int main(int argc, char **argv)
{
	if (argc < 5) {
		fprintf(stderr, "usage: %s newton|admm|gd|gen seed count iterations\n", argv[0]);
		return 2;
	}
	const char *which = argv[1];
	unsigned seed = (unsigned)strtoul(argv[2], NULL, 10);
	int count = atoi(argv[3]);
	unsigned iterations = (unsigned)strtoul(argv[4], NULL, 10);
	opt_fn opt = !strcmp(which, "newton") ? newton_method_with_line_search
		     : !strcmp(which, "admm") ? admm
		     : !strcmp(which, "gd")   ? gradient_descent_with_line_search
					      : NULL;

	kmalloc_init();
	srand(seed);
	struct _matrix *p = matrix_alloc(NxN);
	struct _matrix *q = matrix_alloc(Nx1);
	struct _matrix *x0 = matrix_alloc(Nx1);
	struct _quadratic_form *qf = quadratic_form_alloc(p, q, 0);
	if (!p || !q || !x0 || !qf)
		return 1;
	for (int i = 0; i < count; i++) {
		matirx_random_pos_def(p, P_RAND_ENTRY_MIN, P_RAND_ENTRY_MAX);
		matrix_random(q, Q_RAND_ENTRY_MIN, Q_RAND_ENTRY_MAX);
		matrix_random(x0, X_RAND_ENTRY_MIN, X_RAND_ENTRY_MAX);
		if (!opt) {
			fwrite(p->elements, sizeof(double), N_DIM * N_DIM, stdout);
			fwrite(q->elements, sizeof(double), N_DIM, stdout);
			fwrite(x0->elements, sizeof(double), N_DIM, stdout);
			continue;
		}
		struct _matrix *x = opt(x0, iterations, qf);
		if (!x)
			return 1;
		fwrite(x->elements, sizeof(double), N_DIM, stdout);
		matrix_free(x);
	}
	quadratic_form_free(qf);
	matrix_free(x0);
	matrix_free(q);
	matrix_free(p);
	return 0;
}
