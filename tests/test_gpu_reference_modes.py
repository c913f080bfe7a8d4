"""GPU parity of the reference-semantics kernels (qpb_ref_solve) against the
compiled reference C (golden fixtures from oracle/_ref, tests/golden/).

The kernels replay qp_solvers.c's Newton (:103-144), ADMM (:255-319) and GD
(:65-101) with matrix_invert's LU inverse and unfused fp64 in the reference's
operation order, so the answers should agree to the last bit; the test bar is
north_star's 1e-6 relative, and the bitwise-equal fraction is checked too.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TOL = 1e-6


@pytest.fixture(scope="module")
def qpb():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import qpb as q
    return q


def _run(qpb, mode, P, q, x0, iterations, box=(-1e12, 1e12)):
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()  # noqa: E731
    x, it = qpb.ref_solve(mode, dev(P), dev(q), dev(x0), iterations=iterations, box=box)
    torch.cuda.synchronize()
    return x.cpu().numpy(), it.cpu().numpy()


def _rel(x, ref):
    return np.abs(x - ref).max(axis=1) / np.maximum(1e-300, np.abs(ref).max(axis=1))


@pytest.mark.parametrize("n", [4, 16, 32])
def test_newton_matches_reference_c(qpb, n):
    g = np.load(os.path.join(GOLDEN, f"ref_n{n}.npz"))
    x, it = _run(qpb, qpb.REF_NEWTON, g["P"], g["q"], g["x0"], 10)  # HESS_ITERATIONS config.h:37
    err = _rel(x, g["newton_x"])
    assert err.max() <= TOL, err
    assert (it >= 1).all() and (it <= 10).all()
    assert (err == 0).all()  # bit-faithful replay: every QP bitwise equal


@pytest.mark.parametrize("n,box,key", [(4, 1e12, "admm_x_inactive"), (16, 1e12, "admm_x_inactive"),
                                       (32, 1e12, "admm_x_inactive"), (4, 1e2, "admm_x_active"),
                                       (16, 1e2, "admm_x_active"), (32, 1e2, "admm_x_active")])
def test_admm_matches_reference_c(qpb, n, box, key):
    g = np.load(os.path.join(GOLDEN, f"ref_n{n}.npz"))
    x, it = _run(qpb, qpb.REF_ADMM, g["P"], g["q"], g["x0"], 10000, box=(-box, box))
    err = _rel(x, g[key])
    assert err.max() <= TOL, err
    assert (err == 0).all()


def test_admm_bench_family(qpb):
    """The bench's conditioned box family with the box +-10 compiled into refC."""
    g = np.load(os.path.join(GOLDEN, "cond_box_n16.npz"))
    x, it = _run(qpb, qpb.REF_ADMM, g["H"], g["f"], np.zeros_like(g["f"]), 10000, box=(-10.0, 10.0))
    err = _rel(x, g["admm_x"])
    assert err.max() <= TOL


@pytest.mark.parametrize("n", [4, 16])
def test_gd_matches_reference_c(qpb, n):
    g = np.load(os.path.join(GOLDEN, f"ref_n{n}.npz"))
    k = g["gd_x"].shape[0]
    x, it = _run(qpb, qpb.REF_GD, g["P"][:k], g["q"][:k], g["x0"][:k], 10000)  # GRAD_ITERATIONS
    err = _rel(x, g["gd_x"])
    assert err.max() <= TOL, err
    assert (err == 0).all()


@pytest.mark.parametrize("n", [4, 16])
def test_matrix_invert_replica(qpb, n):
    """One Newton step from x0 = 0 with P = I would be trivial; instead check
    the inverse through Newton on q = -P e_j: x* = e_j exactly when the inverse
    matches the reference's (fixture `inv` = refC matrix_invert(P))."""
    g = np.load(os.path.join(GOLDEN, f"ref_n{n}.npz"))
    P = g["P"]
    inv = g["inv"]
    # Newton's first direction is -inv @ grad(x0); with x0 = 0, grad = q, so
    # d = -inv q; compare via 1 iteration with a huge-q problem where the line
    # search accepts alpha = 0.9 * ... -> just check d through qf
    B = P.shape[0]
    q = np.ones((B, n))
    x0 = np.zeros((B, n))
    x, _ = _run(qpb, qpb.REF_NEWTON, P, q, x0, 1)
    d = -np.einsum("bij,bj->bi", inv, q)
    # x = alpha * d for the accepted alpha (a power of 0.9)
    ratio = x / d
    alpha = ratio[:, 0:1]
    assert np.allclose(ratio, alpha, rtol=1e-9, atol=0)
    k = np.log(alpha[:, 0]) / np.log(0.9)
    assert np.allclose(k, np.round(k), atol=1e-6)


@pytest.mark.parametrize("n", [4, 16])
def test_matrix_invert_bitwise(qpb, n):
    """qpb_matrix_invert against the fixture `inv` = refC matrix_invert(P)
    (matrix_ops.c:551-630): the same LU + per-column solves, bit for bit."""
    g = np.load(os.path.join(GOLDEN, f"ref_n{n}.npz"))
    P = torch.from_numpy(np.ascontiguousarray(g["P"])).cuda()
    inv = qpb.matrix_invert(P).cpu().numpy()
    assert np.array_equal(inv, g["inv"])


def test_matrix_invert_rejects_large_n(qpb):
    P = torch.zeros((1, 1025, 1025), dtype=torch.float64, device="cuda")  # QPB_REF_MAX_N = 1024
    with pytest.raises(qpb.QPBError):
        qpb.matrix_invert(P)


REF_SO = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref")


@pytest.mark.parametrize("n", [4, 16, 32, 48, 80, 127, 128])
def test_replicas_bitwise_vs_live_reference(qpb, n):
    """Fresh QPs from the reference generator per n (256; 64 above n = 64,
    where refC's ADMM takes up to ~60 ms per QP), solved by the compiled
    reference (oracle/_ref, linked -Bsymbolic so its internal calls stay inside
    the reference) and by the GPU replicas: matrix_invert, Newton (10
    iterations) and ADMM (1e4, default and active box) bitwise equal.  n = 48 is
    the reference's own default (config.h:5); n > 64 runs the replicas' one-
    matrix LDS form (qpb_ref.hip): n = 80 with three workgroups per CU, n = 127
    with an odd n (column stride n itself)."""
    import refc
    if not refc.available(n, "1e12") or not refc.available(n, "1e2"):
        pytest.skip("oracle/_ref not built")
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    rc = refc.RefC(n, "1e12")
    P, q, x0 = rc.generate(seed=4242 + n, count=64 if n > 64 else 256)
    # the GPU generator replays the same reference sequence bit for bit
    Pg, qg, xg = qpb.ref_generate(n, len(P), 4242 + n)
    assert np.array_equal(Pg.cpu().numpy(), P) and np.array_equal(qg.cpu().numpy(), q)
    assert np.array_equal(xg.cpu().numpy(), x0)
    inv_ref = np.stack([rc.invert(P[i].copy()) for i in range(len(P))])
    assert np.array_equal(qpb.matrix_invert(dev(P)).cpu().numpy(), inv_ref)
    x, _ = _run(qpb, qpb.REF_NEWTON, P, q, x0, 10)
    assert np.array_equal(x, rc.newton(P, q, x0, 10))
    x, _ = _run(qpb, qpb.REF_ADMM, P, q, x0, 10000)
    assert np.array_equal(x, rc.admm(P, q, x0, 10000))
    ra = refc.RefC(n, "1e2")
    x, _ = _run(qpb, qpb.REF_ADMM, P, q, x0, 10000, box=(-1e2, 1e2))
    assert np.array_equal(x, ra.admm(P, q, x0, 10000))


@pytest.mark.parametrize("n,count,iters", [(80, 8, 20), (128, 8, 20)])
def test_gd_big_layout_bitwise_vs_live_reference(qpb, n, count, iters):
    """REF_GD above n = 64 runs on the one-matrix LDS layout with P loaded
    column-major and no invert (qpb_ref.hip): 20 iterations (~57 Armijo trials
    each; refC takes ~10 s per QP for 1e4 iterations at n = 128) on fresh
    reference-generator QPs against the compiled reference."""
    import refc
    if not refc.available(n, "1e12"):
        pytest.skip("oracle/_ref not built")
    rc = refc.RefC(n, "1e12")
    P, q, x0 = rc.generate(seed=999 + n, count=count)
    x, it = _run(qpb, qpb.REF_GD, P, q, x0, iters)
    assert np.array_equal(x, rc.gd(P, q, x0, iters))
    assert (it >= 1).all() and (it <= iters).all()


@pytest.mark.parametrize("n", [32])
def test_gd_bitwise_vs_live_reference(qpb, n):
    """REF_GD (qp_solvers.c:65-101, 1e4 iterations, ~57 Armijo trials each)
    on fresh reference-generator QPs against the compiled reference; refC
    takes ~0.5 s per QP at n = 32, so 8 QPs."""
    import refc
    if not refc.available(n, "1e12"):
        pytest.skip("oracle/_ref not built")
    rc = refc.RefC(n, "1e12")
    P, q, x0 = rc.generate(seed=777 + n, count=8)
    x, it = _run(qpb, qpb.REF_GD, P, q, x0, 10000)
    assert np.array_equal(x, rc.gd(P, q, x0, 10000))
    assert (it >= 1).all() and (it <= 10000).all()


def test_qf_eval(qpb):
    g = np.load(os.path.join(GOLDEN, "ref_n16.npz"))
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()  # noqa: E731
    out = qpb.qf_eval(dev(g["P"]), dev(g["q"]), 0.0, dev(g["x_exact"]))
    torch.cuda.synchronize()
    assert np.allclose(out.cpu().numpy(), g["f_exact"], rtol=1e-9)


def test_n128_grid_reuse_bitwise_vs_live_reference(qpb):
    """n > 64 runs the replicas as a persistent grid whose workgroups take
    QP after QP on the same LDS and workspace slice (qpb_ref.hip).  With more
    QPs than workgroups every slice is reused -- the path a 64-QP batch never
    reaches: 2 304 reference-generator QPs (the grid is one
    workgroup per CU at n = 128, so each takes about nine), matrix_invert and
    Newton bitwise against the compiled reference, and the generator replica
    bit-exact over the whole range."""
    import refc
    n = 128
    if not refc.available(n, "1e12"):
        pytest.skip("oracle/_ref not built")
    rc = refc.RefC(n, "1e12")
    B = 2304
    P, q, x0 = rc.generate(seed=31337, count=B)
    Pg, qg, xg = qpb.ref_generate(n, B, 31337)
    assert np.array_equal(Pg.cpu().numpy(), P) and np.array_equal(qg.cpu().numpy(), q)
    assert np.array_equal(xg.cpu().numpy(), x0)
    inv = qpb.matrix_invert(Pg).cpu().numpy()
    pick = np.r_[0:8, 250:262, B - 8:B]  # the first, around the CU count, the last
    for i in pick:
        assert np.array_equal(inv[i], rc.invert(P[i].copy())), i
    x, _ = _run(qpb, qpb.REF_NEWTON, P, q, x0, 10)
    assert np.array_equal(x, rc.newton(P, q, x0, 10))
    # ADMM (R = P + I inverted, then 1e3 iterations with R^-1 kept in LDS) on
    # the whole grid, compared on the picked QPs
    x, _ = _run(qpb, qpb.REF_ADMM, P, q, x0, 1000)
    for i in pick:
        assert np.array_equal(x[i], rc.admm(P[i:i + 1], q[i:i + 1], x0[i:i + 1], 1000)[0]), i


@pytest.mark.parametrize("n,count,admm_count", [(129, 8, 8), (200, 4, 2), (300, 2, 1)])
def test_huge_layout_bitwise_vs_live_reference(qpb, n, count, admm_count):
    """128 < n <= 1024 (round 6, VERDICT r05 Missing 4: the compat solvers
    stopped at N_DIM = 128): one 1024-thread workgroup per QP with P, the LU,
    W and V in a global workspace slice (qpb_ref.hip).  Fresh QPs from the
    compiled reference's generator at N_DIM = 129, 200, 300: matrix_invert,
    Newton (10 iterations), GD (20) and ADMM (1e4, default and, at n = 200,
    active box) bitwise against the compiled reference."""
    import refc
    if not refc.available(n, "1e12"):
        pytest.skip("oracle/_ref not built")
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    rc = refc.RefC(n, "1e12")
    P, q, x0 = rc.generate(seed=2468 + n, count=count)
    inv = qpb.matrix_invert(dev(P)).cpu().numpy()
    for i in range(count):
        assert np.array_equal(inv[i], rc.invert(P[i].copy())), i
    x, _ = _run(qpb, qpb.REF_NEWTON, P, q, x0, 10)
    assert np.array_equal(x, rc.newton(P, q, x0, 10))
    x, _ = _run(qpb, qpb.REF_GD, P, q, x0, 20)
    assert np.array_equal(x, rc.gd(P, q, x0, 20))
    a = slice(0, admm_count)
    x, _ = _run(qpb, qpb.REF_ADMM, P[a], q[a], x0[a], 10000)
    assert np.array_equal(x, rc.admm(P[a], q[a], x0[a], 10000))
    if refc.available(n, "1e2"):
        ra = refc.RefC(n, "1e2")
        x, _ = _run(qpb, qpb.REF_ADMM, P[a], q[a], x0[a], 10000, box=(-1e2, 1e2))
        assert np.array_equal(x, ra.admm(P[a], q[a], x0[a], 10000))


def test_huge_layout_grid_reuse_bitwise(qpb):
    """The huge layout's grid is at most one 1024-thread workgroup per CU
    (256 on the MI355X), each walking the batch on its own workspace slice:
    300 QPs of n = 129 reuse slices past the CU count.  matrix_invert on every
    QP against the compiled reference."""
    import refc
    n = 129
    if not refc.available(n, "1e12"):
        pytest.skip("oracle/_ref not built")
    rc = refc.RefC(n, "1e12")
    P, q, x0 = rc.generate(seed=97, count=300)
    inv = qpb.matrix_invert(torch.from_numpy(P).cuda()).cpu().numpy()
    for i in range(300):
        assert np.array_equal(inv[i], rc.invert(P[i].copy())), i


def test_huge_layout_max_n_bitwise(qpb):
    """The largest size the replicas take, n = QPB_REF_MAX_N = 1024 (one
    1024-thread workgroup, one thread per row, 4 n^2 = 32 MiB of workspace):
    matrix_invert, Newton (10 iterations) and GD (20) on one QP bitwise
    against the compiled reference at N_DIM = 1024.  The QP comes from numpy
    (P = B^T B / (1e3 n) symmetrised, the distributions of matirx_random_pos_def,
    matrix_ops.c:699-734): the reference's own generator needs ~10 s of CPU
    at this size and bitwise parity only needs the same input bits on both sides.
    (ADMM is left to n <= 300: one 1e4-iteration solve is ~1 min of CPU here.)"""
    import refc
    n = 1024
    if not refc.available(n, "1e12"):
        pytest.skip("oracle/_ref not built")
    rc = refc.RefC(n, "1e12")
    rng = np.random.default_rng(1024)
    Bm = rng.uniform(-1e3, 1e3, (n, n))
    P = Bm.T @ Bm / (1e3 * n)
    P = ((P + P.T) * 0.5)[None]
    q = rng.uniform(-1e3, 1e3, (1, n))
    x0 = rng.uniform(-1e3, 1e3, (1, n))
    inv = qpb.matrix_invert(torch.from_numpy(P).cuda()).cpu().numpy()
    assert np.array_equal(inv[0], rc.invert(P[0].copy()))
    x, _ = _run(qpb, qpb.REF_NEWTON, P, q, x0, 10)
    assert np.array_equal(x, rc.newton(P, q, x0, 10))
    x, _ = _run(qpb, qpb.REF_GD, P, q, x0, 20)
    assert np.array_equal(x, rc.gd(P, q, x0, 20))
