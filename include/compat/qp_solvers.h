/* qp_solvers.h -- the reference's solver entry points (qpb compat layer).
 * Each call runs the reference-semantics GPU kernel (qpb_ref_solve, batch of
 * one) and returns a new Nx1 matrix the caller matrix_free()s; x0 is
 * borrowed and left unchanged (admm ignores it, as the reference does). */
#ifndef QP_SOLVERS
#define QP_SOLVERS

struct _matrix *gradient_descent_with_line_search(struct _matrix *x0, unsigned iterations,
						  struct _quadratic_form *qf);
struct _matrix *newton_method_with_line_search(struct _matrix *x0, unsigned iterations,
					       struct _quadratic_form *qf);
struct _matrix *admm(struct _matrix *x0, unsigned iterations, struct _quadratic_form *qf);

#endif
