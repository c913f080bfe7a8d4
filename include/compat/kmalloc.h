/* kmalloc.h -- the reference's typed object pools (qpb compat layer).
 * kmalloc_init() must be called first (as the reference's main does); in
 * code compiled against this header it also hands the caller's N_DIM and
 * ADMM box (config.h) to the library. */
#ifndef KMALLOC_H
#define KMALLOC_H

#include "bits.h"

#define KM_ZERO_BIT 31
#define KM_ZERO BIT32(KM_ZERO_BIT)

enum kmalloc_type {
	NxN,
	Nx1,
	QUADRATIC_FORM,
	KMALLOC_TYPE_END,
};

void *kmalloc(enum kmalloc_type type, unsigned flags);
void kfree(void *me, enum kmalloc_type type);
/* binary entry point: N_DIM 48, box +-1e12 (the reference's defaults) */
void kmalloc_init(void);
/* what kmalloc_init() expands to in code compiled against this header */
void qpb_compat_init(unsigned n_dim, double admm_box_min, double admm_box_max);
#define kmalloc_init() qpb_compat_init(N_DIM, ADMM_BOX_CONSTRAINT_MIN, ADMM_BOX_CONSTRAINT_MAX)

#endif
