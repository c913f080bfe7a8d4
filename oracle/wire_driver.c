/*
 * oracle/wire_driver.c -- TEST INFRASTRUCTURE ONLY (checker, never shipped).
 *
 * Captures the bytes the reference's own writer produces: test_reference()
 * (test/test.c:108-130, compiled unmodified where it lies) writes
 * "tmp_test_file" and then runs PYTHON_COMMAND " test/qp_ref.py tmp_test_file"
 * through system().  oracle/Makefile defines PYTHON_COMMAND as a copy of that
 * file to "wire_ref.bin" (no python runs), so the reference's file survives
 * its unlink().  The QP is drawn by the reference generator (main.c:37-38
 * order) after srand(seed); its P and q are also dumped raw to "pq.bin" for
 * the test to rebuild the same file through qpb_wire_write.
 *
 * usage: wire_ref_n<N> <seed>      (run in an empty directory)
 */
#include <stdio.h>
#include <stdlib.h>

#include "test.h"

int main(int argc, char **argv)
{
	unsigned seed = argc > 1 ? (unsigned)strtoul(argv[1], 0, 10) : 1U;
	kmalloc_init(); /* main.c:10 */
	srand(seed);
	struct _matrix *p = matrix_alloc(NxN);
	struct _matrix *q = matrix_alloc(Nx1);
	struct _quadratic_form *qf = quadratic_form_alloc(p, q, 0);
	if (!p || !q || !qf)
		return EXIT_FAILURE;
	matirx_random_pos_def(p, P_RAND_ENTRY_MIN, P_RAND_ENTRY_MAX);
	matrix_random(q, Q_RAND_ENTRY_MIN, Q_RAND_ENTRY_MAX);
	test_reference(qf); /* test.c:108-130 */
	FILE *fp = fopen("pq.bin", "wb");
	if (!fp)
		return EXIT_FAILURE;
	fwrite(p->elements, sizeof(double), N_DIM * N_DIM, fp);
	fwrite(q->elements, sizeof(double), N_DIM, fp);
	fclose(fp);
	return EXIT_SUCCESS;
}
