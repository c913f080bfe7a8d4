/* qp.h -- the reference's quadratic-form object (qpb compat layer):
 * f(x) = 1/2 x^T p x + q^T x + r.  p and q are borrowed, never freed here. */
#ifndef QP_H
#define QP_H

#include "matrix_ops.h"

#define QUADRATIC_FORM_MAX 1

struct _quadratic_form {
	struct _matrix *p;
	struct _matrix *q;
	double r;
};

struct _quadratic_form *quadratic_form_alloc(struct _matrix *p, struct _matrix *q, double r);
/* does not free p and q */
void quadratic_form_free(struct _quadratic_form *qf);
/* f(x), scalar */
double quadratic_form_eval(struct _quadratic_form *qf, struct _matrix *x);
/* grad f(x) = p x + q as a new Nx1 matrix; the caller matrix_free()s it */
struct _matrix *quadratic_form_eval_grad(struct _quadratic_form *qf, struct _matrix *x);

#endif
