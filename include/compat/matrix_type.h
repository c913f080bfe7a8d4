/* matrix_type.h -- the reference's matrix handle, layout-compatible
 * (qpb compat layer).  struct _matrix: `dimensions` packs rows in bits 16-31
 * and columns in bits 0-15; `elements` is dense row-major fp64. */
#ifndef MATRIX_TYPE_H
#define MATRIX_TYPE_H

#include "config.h"
#include "bits.h"

/* matrix entry literal: ME(row, col) */
#define ME(i, j) ((struct _matrix_entry){(i), (j)})

#define MATRIX_GET_ROW(m) (GETM32(16, 31, (m)->dimensions) >> 16)
#define MATRIX_GET_COL(m) GETM32(0, 15, (m)->dimensions)
#define MATRIX_SET_ROW(m, n) SETM32(16, 31, (m)->dimensions, (unsigned)(n))
#define MATRIX_SET_COL(m, n) SETM32(0, 15, (m)->dimensions, (unsigned)(n))

struct _matrix {
	unsigned dimensions;
	double *elements;
};

struct _matrix_entry {
	unsigned row;
	unsigned col;
};

#endif
