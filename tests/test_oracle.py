"""CPU tests: the oracle pinned against the reference's own behaviour.

* glibc rand restatement == the C library's rand() (the reference draws every
  input through it: main.c:11, matrix_ops.c:677-681)
* the generator restatement reproduces the compiled reference's inputs
  bit-for-bit (fixtures from oracle/_ref, tests/golden/make_golden.py)
* test/qp_ref.py's answer (unconstrained solve) and its wire format
* the constrained oracle's answers carry a KKT certificate, and the reference's
  ADMM on the active box (qp_solvers.c:255-319) lands near them
* the reference's own known-answer / property tests (test/test.c:37-87)
"""
import ctypes
import os

import numpy as np
import pytest

from conftest import GOLDEN

import oracle as O


def load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


@pytest.mark.parametrize("seed", [0, 1, 42, 12345, 20261015, 2**31 + 7])
def test_glibc_rand_restatement(seed):
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(ctypes.c_uint(seed))
    want = [libc.rand() for _ in range(2000)]
    g = O.GlibcRand(seed)
    assert [g.rand() for _ in range(2000)] == want


@pytest.mark.parametrize("n,seed", [(4, 4001), (16, 16001), (32, 32001)])
def test_generator_matches_reference_fixtures(n, seed):
    g = load(f"ref_n{n}")
    count = g["P"].shape[0]
    P, q, x0 = O.ref_generate(seed, count, n)
    assert np.array_equal(P, g["P"]) and np.array_equal(q, g["q"]) and np.array_equal(x0, g["x0"])
    assert np.array_equal(P, np.transpose(P, (0, 2, 1)))  # B^T B is exactly symmetric


@pytest.mark.parametrize("n", [4, 16, 32])
def test_qp_ref_restatement(n, tmp_path):
    g = load(f"ref_n{n}")
    for i in range(min(4, len(g["q"]))):
        path = tmp_path / "tmp_test_file"
        O.write_wire(str(path), g["P"][i], g["q"][i])  # test.c:108-126 layout
        assert os.path.getsize(path) == 8 * (1 + n * n + n)
        nn, P, q = O.read_wire(str(path))  # qp_ref.py:8-30
        assert nn == n and np.array_equal(P, g["P"][i]) and np.array_equal(q, g["q"][i])
        x = O.qp_ref_solve(P, q)
        assert np.allclose(x, g["x_exact"][i], rtol=0, atol=1e-12 * max(1, np.abs(x).max()) * np.linalg.cond(P))
        assert np.isclose(O.eval_qp(P, q, x), g["f_exact"][i], rtol=1e-9)


def test_reference_newton_near_qp_ref():
    """refC Newton stops at ||grad|| < 0.1 (qp_solvers.c:15,125); SURVEY measured
    1e-14..4e-5 relative vs x*."""
    for n in (4, 16, 32):
        g = load(f"ref_n{n}")
        err = np.abs(g["newton_x"] - g["x_exact"]).max(1) / np.abs(g["x_exact"]).max(1)
        assert np.median(err) < 1e-4


@pytest.mark.parametrize("name", ["cond_box_n16", "cond_dense_n16_m32", "cond_box_n4", "cond_dense_n4_m8",
                                  "cond_dense_n10_m20"])
def test_constrained_oracle_certified(name):
    g = load(name)
    r = O.kkt_residuals(g["H"], g["f"], g["A"], g["b"], g["x"], g["lam"])
    for k, v in r.items():
        assert v.max() < 1e-9, k
    assert np.array_equal(g["act"], g["lam"] > 0)
    # strict complementarity margin (non-degenerate family => bit-exact masks are well defined)
    slack = g["b"] - np.einsum("bij,bj->bi", g["A"], g["x"])
    inactive = ~g["act"]
    assert (slack[inactive] > 1e-8).all()
    assert (g["lam"][g["act"]] > 1e-8).all()


def test_oracle_recomputes_fixture():
    g = load("cond_box_n4")
    for i in range(8):
        r = O.active_set_solve(g["H"][i], g["f"][i], g["A"][i], g["b"][i])
        assert r.status == 0
        assert np.allclose(r.x, g["x"][i], atol=1e-12)


def test_reference_admm_on_box_family():
    """The reference's only constrained path (admm, box 10 compiled in) on the
    conditioned box family: x within ADMM's tolerance (RELTOL 1e-2,
    qp_solvers.c:17-18) of the exact constrained optimum."""
    g = load("cond_box_n16")
    err = np.abs(g["admm_x"] - g["x"]).max(1) / np.abs(g["x"]).max(1)
    assert np.median(err) < 5e-2


@pytest.mark.parametrize("n", [4, 16])
def test_reference_inversion_test(n):
    """test/test.c:37-57: ||P * P^{-1} - I||_max <= 1e-6 (config.h:12) for the
    refC matrix_invert output, on the well-conditioned part of the family."""
    g = load(f"ref_n{n}")
    cond = np.linalg.cond(g["P"])
    ok = 0
    for i in range(len(cond)):
        E = g["P"][i] @ g["inv"][i] - np.eye(n)
        if cond[i] < 1e6:
            assert np.abs(E).max() <= 1e-6
            ok += 1
    assert ok > 0


def test_scalar_prod_known_answer():
    """test/test.c:59-87: with a = column (0..N-1) and b = e_0, c = a b and
    d = (0..N-1), d . c = N(N+1)(2N+1)/6 - N^2 (= sum_{i<N} i^2) exactly."""
    for N in (4, 16, 48):
        d = np.arange(N, dtype=np.float64)
        c = d.copy()
        assert float(d @ c) == N * (N + 1) * (2 * N + 1) / 6 - N * N


def test_device_kkt_helper_matches_oracle_certificate():
    """tests/conftest.kkt_max_residual_device (the full-batch certificate of
    the GPU tests, torch on the device) restates oracle.kkt_residuals: on CPU
    tensors both give the same worst residual, for exact and perturbed
    answers."""
    import torch
    from conftest import kkt_max_residual_device
    H, f, A, b = O.family_conditioned(77, 6, 8, m=16, box=3.0, kind="dense")
    sols = [O.active_set_solve(H[i], f[i], A[i], b[i]) for i in range(6)]
    x = np.array([s.x for s in sols])
    lam = np.array([s.lam for s in sols])
    for xx, ll in ((x, lam), (x + 1e-3, lam), (x, lam - 0.1)):
        ref = max(float(v.max()) for v in O.kkt_residuals(H, f, A, b, xx, ll).values())
        t = [torch.from_numpy(np.ascontiguousarray(v)) for v in (H, f, A, b, xx, ll)]
        got = kkt_max_residual_device(*t, chunk=4)
        assert abs(got - ref) <= 1e-12 * max(1.0, ref), (got, ref)


@pytest.mark.parametrize("name", ["cond_box_n16", "cond_dense_n16_m32", "cond_box_n4", "cond_dense_n4_m8",
                                  "cond_dense_n10_m20"])
def test_oracle_rules_reproduce_every_fixture(name):
    """The oracle with its round-6 rules (full-step flag, Bland's rule after a
    degenerate step) reproduces every committed constrained fixture: x within
    1e-9 relative and the active set bit-exact."""
    g = load(name)
    for i in range(len(g["f"])):
        r = O.active_set_solve(g["H"][i], g["f"][i], g["A"][i], g["b"][i])
        assert r.status == 0, i
        assert np.abs(r.x - g["x"][i]).max() <= 1e-9 * max(1.0, np.abs(g["x"][i]).max()), i
        assert np.array_equal(r.active, g["act"][i]), i


def _vertex_qp(n, m, seed, k):
    # one QP of tests/test_gpu_active_set.py's vertex family
    rs = np.random.default_rng(seed)
    Bm = rs.standard_normal((256, n, n))
    H = np.eye(n) + 0.1 * np.einsum("bki,bkj->bij", Bm, Bm) / n
    f = 100.0 * rs.standard_normal((256, n))
    A = rs.standard_normal((256, m, n))
    A /= np.linalg.norm(A, axis=2, keepdims=True)
    b = rs.uniform(0.1, 1.0, (256, m))
    return H[k], f[k], A[k], b[k]


@pytest.mark.parametrize("n,m,k", [(16, 32, 181), (16, 32, 182), (12, 24, 209), (32, 64, 14)])
def test_oracle_terminates_at_full_vertices(n, m, k):
    """QPs of the vertex family on whose path round 5's oracle reached a full
    working set (|W| = n) and then stepped by rounding noise until max_iter:
    now solved and KKT-certified."""
    H, f, A, b = _vertex_qp(n, m, 500 + n, k)
    r = O.active_set_solve(H, f, A, b)
    assert r.status == 0
    res = O.kkt_residuals(H[None], f[None], A[None], b[None], r.x[None], r.lam[None])
    assert max(float(v.max()) for v in res.values()) <= 1e-9


def test_oracle_degenerate_vertex_bland():
    """A degenerate start: 2n rows through the origin (more than n active
    there, so the first steps are degenerate, alpha = 0); Bland's rule ends
    them and the answer is KKT-certified."""
    n = 4
    rs = np.random.default_rng(3)
    A = np.abs(rs.standard_normal((2 * n, n))) + 0.1  # a_i > 0: x = 0 is the optimum for f < 0
    A /= np.linalg.norm(A, axis=1, keepdims=True)
    b = np.zeros(2 * n)
    H, f = np.eye(n), -np.ones(n)
    r = O.active_set_solve(H, f, A, b, x0=np.zeros(n))
    assert r.status == 0
    res = O.kkt_residuals(H[None], f[None], A[None], b[None], r.x[None], r.lam[None])
    assert max(float(v.max()) for v in res.values()) <= 1e-9
