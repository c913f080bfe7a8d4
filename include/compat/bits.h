/* bits.h -- bit-field helpers used by the matrix dimension packing
 * (qpb compat layer; same macro names as the reference's misc/bits.h). */
#ifndef BITS_H
#define BITS_H 1

#define BIT32(n) (1U << (n))
#define BIT64(n) (1ULL << (n))
/* bits n..m (inclusive) set */
#define MASK32(n, m) (((~0U) << (n)) & (~0U >> (31 - (m))))
#define MASK64(n, m) (((~0ULL) << (n)) & (~0ULL >> (63 - (m))))

#define SETB32(n, word) ((word) |= BIT32(n))
#define SETB64(n, word) ((word) |= BIT64(n))
#define CLRB32(n, word) ((word) &= ~BIT32(n))
#define CLRB64(n, word) ((word) &= ~BIT64(n))
#define CLRM32(n, m, word) ((word) &= ~MASK32(n, m))
#define CLRM64(n, m, word) ((word) &= ~MASK64(n, m))
#define SETM32(n, m, word, what) \
	do { CLRM32(n, m, word); (word) |= MASK32(n, m) & ((what) << (n)); } while (0)
#define SETM64(n, m, word, what) \
	do { CLRM64(n, m, word); (word) |= MASK64(n, m) & ((what) << (n)); } while (0)
#define GETB32(n, word) ((word) & BIT32(n))
#define GETB64(n, word) ((word) & BIT64(n))
#define GETM32(n, m, word) ((word) & MASK32(n, m))
#define GETM64(n, m, word) ((word) & MASK64(n, m))

#define ALIGN8(x) (7U & (x) ? ((x) + 8U) & ~7U : (x))

#endif
