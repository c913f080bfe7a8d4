/*
 * config.h -- compile-time configuration of the reference-compatible API
 * (qpb compat layer).  Same macro names and defaults as the reference's PC
 * configuration (YangLingyuan/Embedded-qp-solver config.h), each overridable
 * with -D.  N_DIM and the ADMM box are handed to the library at
 * kmalloc_init() (see kmalloc.h), so one libqpb.so serves every N_DIM.
 */
#ifndef CONFIG_H
#define CONFIG_H

/* matrix dimension: NxN / Nx1 objects from matrix_alloc */
#ifndef N_DIM
#define N_DIM 48U
#endif
/* pool capacities of the reference allocator (the library's pools are at
 * least this large) */
#ifndef NxN_MAX
#define NxN_MAX 5
#endif
#ifndef Nx1_MAX
#define Nx1_MAX 10
#endif

/* matrix library self-tests */
#ifndef INVERSION_TEST_PRECISION
#define INVERSION_TEST_PRECISION 1e-6
#endif
#ifndef NUM_INVERSION_TEST_RUNS
#define NUM_INVERSION_TEST_RUNS 8
#endif

/* random problem ranges (P entries, q entries, initial state) */
#ifndef P_RAND_ENTRY_MIN
#define P_RAND_ENTRY_MIN -1e3
#endif
#ifndef P_RAND_ENTRY_MAX
#define P_RAND_ENTRY_MAX 1e3
#endif
#ifndef Q_RAND_ENTRY_MIN
#define Q_RAND_ENTRY_MIN -1e3
#endif
#ifndef Q_RAND_ENTRY_MAX
#define Q_RAND_ENTRY_MAX 1e3
#endif
#ifndef X_RAND_ENTRY_MIN
#define X_RAND_ENTRY_MIN -1e3
#endif
#ifndef X_RAND_ENTRY_MAX
#define X_RAND_ENTRY_MAX 1e3
#endif

#ifndef NUM_OPT_TEST_RUNS
#define NUM_OPT_TEST_RUNS 16
#endif

/* box of admm() */
#ifndef ADMM_BOX_CONSTRAINT_MAX
#define ADMM_BOX_CONSTRAINT_MAX 1e12
#endif
#ifndef ADMM_BOX_CONSTRAINT_MIN
#define ADMM_BOX_CONSTRAINT_MIN -1e12
#endif

#ifndef PYTHON_COMMAND
#define PYTHON_COMMAND "python"
#endif

/* iteration caps handed to the optimizers by the test driver */
#ifndef GRAD_ITERATIONS
#define GRAD_ITERATIONS 1e4
#endif
#ifndef HESS_ITERATIONS
#define HESS_ITERATIONS 1e1
#endif
#ifndef ADMM_ITERATIONS
#define ADMM_ITERATIONS 1e4
#endif

/* test selection (define QPB_NO_DEFAULT_TESTS to start from none); the
 * qp_ref.py comparison needs the absent qpsolvers package: off by default */
#ifndef QPB_NO_DEFAULT_TESTS
#define INV_TEST
#define PROD_TEST
#define GRAD_TEST
#define HESS_TEST
#define ADMM_TEST
#endif

#endif
