"""CPU tests of the reference-compatible host API in libqpb.so (include/compat):
the object pools and the single-matrix utilities, checked against the
reference's own known answers (test/test.c:37-87) and refC outputs.  The
solvers (GPU) are covered by tests/test_gpu_compat.py."""
import ctypes
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

# QPB_LIB: another build of the same library (tests/test_sanitizers.py runs
# this file against the ASan/UBSan build)
LIB = os.environ.get("QPB_LIB", os.path.join(ROOT, "embedded-qp-solver_amd", "lib", "libqpb.so"))
NxN, Nx1, QF = 0, 1, 2


class Matrix(ctypes.Structure):
    _fields_ = [("dimensions", ctypes.c_uint), ("elements", ctypes.POINTER(ctypes.c_double))]


class Entry(ctypes.Structure):
    _fields_ = [("row", ctypes.c_uint), ("col", ctypes.c_uint)]


@pytest.fixture()
def lib():
    L = ctypes.CDLL(LIB)
    MP = ctypes.POINTER(Matrix)
    L.matrix_alloc.restype = MP
    L.matrix_alloc.argtypes = [ctypes.c_int]
    L.matrix_free.argtypes = [MP]
    for f in ("matrix_invert", "matrix_trans", "matrix_neg", "matrix_zero_up", "matrix_identity"):
        getattr(L, f).argtypes = [MP]
    L.matrix_norm.argtypes = [MP]
    L.matrix_norm.restype = ctypes.c_double
    L.matrix_mult.argtypes = [MP, MP, MP]
    L.matrix_add.argtypes = [MP, MP, MP]
    L.matrix_scalar_prod.argtypes = [MP, MP]
    L.matrix_scalar_prod.restype = ctypes.c_double
    L.matrix_set_entry.argtypes = [MP, Entry, ctypes.c_double]
    L.matrix_get_entry.argtypes = [MP, Entry]
    L.matrix_get_entry.restype = ctypes.c_double
    L.qpb_compat_init.argtypes = [ctypes.c_uint, ctypes.c_double, ctypes.c_double]
    L.kmalloc.restype = ctypes.c_void_p
    L.kmalloc.argtypes = [ctypes.c_int, ctypes.c_uint]
    L.kfree.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.quadratic_form_alloc.restype = ctypes.c_void_p
    L.quadratic_form_alloc.argtypes = [MP, MP, ctypes.c_double]
    L.quadratic_form_eval.restype = ctypes.c_double
    L.quadratic_form_eval.argtypes = [ctypes.c_void_p, MP]
    L.quadratic_form_free.argtypes = [ctypes.c_void_p]
    return L


def arr(m, n_rows, n_cols):
    return np.ctypeslib.as_array(m.contents.elements, shape=(n_rows * n_cols,)).reshape(n_rows, n_cols)


def test_dimension_packing(lib):
    lib.qpb_compat_init(16, -1e12, 1e12)
    m = lib.matrix_alloc(NxN)
    v = lib.matrix_alloc(Nx1)
    assert m.contents.dimensions == (16 << 16) | 16  # rows bits 16-31, cols 0-15 (matrix_type.h:14-17)
    assert v.contents.dimensions == (16 << 16) | 1
    lib.matrix_trans(v)
    assert v.contents.dimensions == (1 << 16) | 16
    lib.matrix_trans(v)
    lib.matrix_free(m)
    lib.matrix_free(v)


def test_scalar_prod_known_answer(lib):
    """test/test.c:59-87: a (NxN, column 0 = 0..N-1) times e_0, transposed,
    dotted with d = (0..N-1): exactly sum_{i<N} i^2."""
    for N in (16, 48):
        lib.qpb_compat_init(N, -1e12, 1e12)
        a = lib.matrix_alloc(NxN)
        A = arr(a, N, N)
        A[:] = 0
        A[:, 0] = np.arange(N)
        b = lib.matrix_alloc(Nx1)
        arr(b, N, 1)[:] = 0
        lib.matrix_set_entry(b, Entry(0, 0), 1.0)
        c = lib.matrix_alloc(Nx1)
        lib.matrix_mult(c, a, b)
        d = lib.matrix_alloc(Nx1)
        arr(d, N, 1)[:, 0] = np.arange(N)
        lib.matrix_trans(c)
        lib.matrix_trans(d)
        assert lib.matrix_scalar_prod(d, c) == N * (N + 1) * (2 * N + 1) / 6 - N * N
        for x in (a, b, c, d):
            lib.matrix_trans(x) if x in (c, d) else None
            lib.matrix_free(x)


@pytest.mark.parametrize("n", [4, 16])
def test_matrix_invert_matches_reference(lib, n):
    """matrix_invert == the compiled reference's matrix_invert (fixture `inv`)."""
    g = np.load(os.path.join(GOLDEN, f"ref_n{n}.npz"))
    lib.qpb_compat_init(n, -1e12, 1e12)
    m = lib.matrix_alloc(NxN)
    M = arr(m, n, n)
    for i in range(len(g["P"])):
        M[:] = g["P"][i]
        lib.matrix_invert(m)
        assert np.array_equal(M, g["inv"][i])
    lib.matrix_free(m)


def test_pools_and_quadratic_form(lib):
    lib.qpb_compat_init(16, -1e12, 1e12)
    g = np.load(os.path.join(GOLDEN, "ref_n16.npz"))
    p = lib.matrix_alloc(NxN)
    q = lib.matrix_alloc(Nx1)
    x = lib.matrix_alloc(Nx1)
    arr(p, 16, 16)[:] = g["P"][0]
    arr(q, 16, 1)[:, 0] = g["q"][0]
    arr(x, 16, 1)[:, 0] = g["x_exact"][0]
    qf = lib.quadratic_form_alloc(p, q, 0.0)
    assert qf
    assert np.isclose(lib.quadratic_form_eval(qf, x), g["f_exact"][0], rtol=1e-12)
    lib.quadratic_form_free(qf)
    # pools hand out distinct objects and take them back
    objs = [lib.kmalloc(Nx1, 0) for _ in range(8)]
    assert len(set(objs)) == 8 and all(objs)
    for o in objs:
        lib.kfree(o, Nx1)
    assert lib.kmalloc(99, 0) is None
    for m_ in (p, q, x):
        lib.matrix_free(m_)


def test_reference_main_builds_against_compat():
    """oracle/_ref/ref_main_on_qpb: the reference's main.c + test/test.c
    compiled against include/compat and linked with libqpb.so (built here by
    `make -C oracle ref`; it runs on the GPU box: test_gpu_compat.py)."""
    path = os.path.join(ROOT, "oracle", "_ref", "ref_main_on_qpb")
    if not os.path.exists(path):
        pytest.skip("reference build not present (needs /root/reference)")
    assert os.access(path, os.X_OK)


def _child(code):
    import subprocess
    import sys
    env = dict(os.environ, QPB_LIB_UNDER_TEST=LIB)
    pre = ("import ctypes, os\n"
           "L = ctypes.CDLL(os.environ['QPB_LIB_UNDER_TEST'])\n"
           "L.qpb_compat_init.argtypes = [ctypes.c_uint, ctypes.c_double, ctypes.c_double]\n"
           "L.matrix_alloc.restype = ctypes.c_void_p\n")
    return subprocess.run([sys.executable, "-c", pre + code], env=env, capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize("n_dim,ok", [(128, True), (129, True), (300, True), (0, False), (65536, False)])
def test_compat_init_accepts_the_reference_dimension_range(n_dim, ok):
    """kmalloc_init() (qpb_compat_init) takes any N_DIM the reference's 16-bit
    dimension fields hold (matrix_type.h:14-17): the host matrix library works
    there (an n x n product at N_DIM = 300 below); 0 and 65 536 are refused with
    the reason.  A child process: the refusal exits, as the reference exits on
    its own fatal errors (qp_solvers.c:79-82).  Under tests/test_sanitizers.py
    this runs against the ASan/UBSan build."""
    r = _child(f"L.qpb_compat_init({n_dim}, -1e12, 1e12)\n"
               "a, b, c = (ctypes.c_void_p(L.matrix_alloc(0)) for _ in range(3))\n"
               "print('alloc', bool(a.value and b.value and c.value))\n"
               "L.matrix_mult(c, a, b)\n"
               "print('mult ok')\n")
    if ok:
        assert r.returncode == 0, r.stderr
        assert "alloc True" in r.stdout and "mult ok" in r.stdout
    else:
        assert r.returncode != 0
        assert f"N_DIM = {n_dim} is outside 1..65535" in r.stderr
        assert "alloc" not in r.stdout


@pytest.mark.parametrize("solver", ["admm", "newton_method_with_line_search", "gradient_descent_with_line_search"])
def test_compat_solvers_refuse_ndim_beyond_the_gpu_replicas(solver):
    """At N_DIM = 1025 the qp_solvers.h solvers (GPU replicas, n <= 1024 since
    round 6; 128 before) exit with the reason before any device call; the
    matrix routines kept working."""
    r = _child("L.qpb_compat_init(1025, -1e12, 1e12)\n"
               "L.quadratic_form_alloc.restype = ctypes.c_void_p\n"
               "L.quadratic_form_alloc.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double]\n"
               "p, q, x = (ctypes.c_void_p(L.matrix_alloc(t)) for t in (0, 1, 1))\n"
               "qf = ctypes.c_void_p(L.quadratic_form_alloc(p, q, 0.0))\n"
               f"L.{solver}.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]\n"
               f"L.{solver}(x, 1, qf)\n"
               "print('returned')\n")
    assert r.returncode != 0
    assert "returned" not in r.stdout
    assert f"{solver}: N_DIM = 1025" in r.stderr and "n <= 1024" in r.stderr
