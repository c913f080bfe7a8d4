/* qpb_wire.c -- QP wire format I/O.
 *
 * The reference exchanges one unconstrained QP with its Python checker as
 * native-endian fp64: [n][P row-major n*n][q n] (written by test/test.c:
 * 108-126, read by test/qp_ref.py:8-30).  The batched form keeps the
 * all-fp64 style: a header [n][m][B] followed by B records
 * [H n*n][f n][A m*n][b m] (AoS, the layout qpb_solve takes).  A file with
 * m = 0 and B = 1 is written in the reference's own format, so single QPs
 * move both ways between this library, test.c and qp_ref.py; readers tell the
 * two forms apart by the file size (8 (1 + n^2 + n) bytes for the reference
 * form, 8 (3 + B (n^2 + n + m n + m)) for the batched one).
 *
 * Host code only (plain C): files are read into / written from host memory.
 */
#define _DEFAULT_SOURCE
#define _FILE_OFFSET_BITS 64
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "qpb.h"

__attribute__((visibility("hidden"))) void qpb_set_error(int code, const char *msg); /* qpb_api.hip */

static int wire_fail(int code, const char *msg) {
	qpb_set_error(code, msg);
	return code;
}

static long long file_size(FILE *fp) {
	if (fseeko(fp, 0, SEEK_END) != 0) return -1;
	long long sz = (long long)ftello(fp);
	if (fseeko(fp, 0, SEEK_SET) != 0) return -1;
	return sz;
}

static int as_count(double v, long long lo, long long hi, long long *out) {
	if (!(v >= (double)lo && v <= (double)hi) || floor(v) != v) return 0;
	*out = (long long)v;
	return 1;
}

int qpb_wire_write(const char *path, int32_t n, int32_t m, int64_t batch, const double *H, const double *f,
		   const double *A, const double *b) {
	if (!path || n < 1 || m < 0 || batch < 1 || !H || !f || (m > 0 && (!A || !b)))
		return wire_fail(QPB_ERR_INVALID_ARG, "qpb_wire_write: bad arguments");
	FILE *fp = fopen(path, "wb");
	if (!fp) return wire_fail(QPB_ERR_INVALID_ARG, "qpb_wire_write: cannot open file");
	const size_t nn = (size_t)n * n, mn = (size_t)m * n;
	int ok = 1;
	if (m == 0 && batch == 1) { /* the reference's form: test/test.c:110-121 */
		const double dn = (double)n;
		ok = fwrite(&dn, sizeof dn, 1, fp) == 1 && fwrite(H, sizeof *H, nn, fp) == nn &&
		     fwrite(f, sizeof *f, (size_t)n, fp) == (size_t)n;
	} else {
		const double hdr[3] = {(double)n, (double)m, (double)batch};
		ok = fwrite(hdr, sizeof *hdr, 3, fp) == 3;
		for (int64_t k = 0; ok && k < batch; ++k) {
			ok = fwrite(H + (size_t)k * nn, sizeof *H, nn, fp) == nn &&
			     fwrite(f + (size_t)k * n, sizeof *f, (size_t)n, fp) == (size_t)n;
			if (ok && m > 0)
				ok = fwrite(A + (size_t)k * mn, sizeof *A, mn, fp) == mn &&
				     fwrite(b + (size_t)k * m, sizeof *b, (size_t)m, fp) == (size_t)m;
		}
	}
	if (fclose(fp) != 0) ok = 0;
	return ok ? 0 : wire_fail(QPB_ERR_INVALID_ARG, "qpb_wire_write: write failed");
}

/* header of either form; *is_ref = 1 for the reference's single-QP form */
static int read_header(FILE *fp, int32_t *n, int32_t *m, int64_t *batch, int *is_ref) {
	const long long sz = file_size(fp);
	double h[3] = {0, 0, 0};
	if (sz < 8 || sz % 8 != 0 || fread(h, sizeof(double), sz >= 24 ? 3 : 1, fp) < 1)
		return wire_fail(QPB_ERR_INVALID_ARG, "qpb_wire: not a QP wire file (size)");
	long long nn = 0, mm = 0, bb = 0;
	if (!as_count(h[0], 1, 65535, &nn)) return wire_fail(QPB_ERR_INVALID_ARG, "qpb_wire: bad n in header");
	if (sz == 8 * (1 + nn * nn + nn)) {
		*n = (int32_t)nn;
		*m = 0;
		*batch = 1;
		*is_ref = 1;
		return 0;
	}
	if (sz < 24 || !as_count(h[1], 0, 1 << 20, &mm) || !as_count(h[2], 1, 1LL << 40, &bb))
		return wire_fail(QPB_ERR_INVALID_ARG, "qpb_wire: bad m or batch in header");
	const long long rec = nn * nn + nn + mm * nn + mm;
	if (sz != 8 * (3 + bb * rec)) return wire_fail(QPB_ERR_INVALID_ARG, "qpb_wire: size does not match header");
	*n = (int32_t)nn;
	*m = (int32_t)mm;
	*batch = bb;
	*is_ref = 0;
	return 0;
}

int qpb_wire_read_header(const char *path, int32_t *n, int32_t *m, int64_t *batch) {
	if (!path || !n || !m || !batch) return wire_fail(QPB_ERR_INVALID_ARG, "qpb_wire_read_header: bad arguments");
	FILE *fp = fopen(path, "rb");
	if (!fp) return wire_fail(QPB_ERR_INVALID_ARG, "qpb_wire_read_header: cannot open file");
	int is_ref = 0;
	const int rc = read_header(fp, n, m, batch, &is_ref);
	fclose(fp);
	return rc;
}

int qpb_wire_read(const char *path, double *H, double *f, double *A, double *b) {
	if (!path || !H || !f) return wire_fail(QPB_ERR_INVALID_ARG, "qpb_wire_read: bad arguments");
	FILE *fp = fopen(path, "rb");
	if (!fp) return wire_fail(QPB_ERR_INVALID_ARG, "qpb_wire_read: cannot open file");
	int32_t n = 0, m = 0;
	int64_t batch = 0;
	int is_ref = 0;
	int rc = read_header(fp, &n, &m, &batch, &is_ref);
	if (rc) {
		fclose(fp);
		return rc;
	}
	if (m > 0 && (!A || !b)) {
		fclose(fp);
		return wire_fail(QPB_ERR_INVALID_ARG, "qpb_wire_read: m > 0 needs A and b");
	}
	fseeko(fp, is_ref ? 8 : 24, SEEK_SET);
	const size_t nn = (size_t)n * n, mn = (size_t)m * n;
	int ok = 1;
	for (int64_t k = 0; ok && k < batch; ++k) {
		ok = fread(H + (size_t)k * nn, sizeof *H, nn, fp) == nn &&
		     fread(f + (size_t)k * n, sizeof *f, (size_t)n, fp) == (size_t)n;
		if (ok && m > 0)
			ok = fread(A + (size_t)k * mn, sizeof *A, mn, fp) == mn &&
			     fread(b + (size_t)k * m, sizeof *b, (size_t)m, fp) == (size_t)m;
	}
	fclose(fp);
	return ok ? 0 : wire_fail(QPB_ERR_INVALID_ARG, "qpb_wire_read: short read");
}
