"""GPU parity of the box-constrained kernels (qpb_solve_box: qpb_gi_box.hip for
n <= 16, the BOX form of qpb_gi_wave.hip for 16 < n <= 32, the BOX form of
qpb_gi_gram.hip for 32 < n <= 128 since round 6):
lb <= x <= ub with A = [I; -I] kept implicit -- the constraint class of the
reference's admm() (qp_solvers.c:146-319).  Oracles: the KKT-certified primal
active set (oracle.active_set_solve) on the same QPs written with a dense
A = [I; -I], b = [ub; -lb] (x and lambda within 1e-6 relative, active set
bit-exact, KKT <= 1e-9 on every QP), and the dense GPU path qpb_solve on the
same dense form (same active sets; x within 1e-12).  Through the C-ABI."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402

TOL = 1e-6


@pytest.fixture(scope="module")
def qpb():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import qpb as q
    return q


def _family(seed, count, n, width=10.0, asym=True):
    """The conditioned family's H and f with bounds lb < ub around 0 (asymmetric:
    lb ~ -U(0.5, 1.5) width, ub ~ U(0.5, 1.5) width)."""
    H, f, _, _ = O.family_conditioned(seed, count, n, m=2 * n, box=width, kind="box")
    rs = np.random.default_rng(seed + 1)
    ub = rs.uniform(0.5, 1.5, size=(count, n)) * width if asym else np.full((count, n), width)
    lb = -rs.uniform(0.5, 1.5, size=(count, n)) * width if asym else np.full((count, n), -width)
    return H, f, lb, ub


def _dense(lb, ub):
    B, n = lb.shape
    A = np.concatenate([np.broadcast_to(np.eye(n), (B, n, n)), np.broadcast_to(-np.eye(n), (B, n, n))], axis=1)
    return np.ascontiguousarray(A), np.concatenate([ub, -lb], axis=1)


def _cuda(*arrs):
    return [None if a is None else torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


def _np(sol):
    torch.cuda.synchronize()
    return [t.cpu().numpy() for t in sol]


@pytest.mark.parametrize("n,count", [(16, 64), (4, 40), (7, 33), (13, 17), (1, 9), (20, 24), (32, 32), (25, 9),
                                     (17, 5), (31, 1), (33, 7), (48, 12), (100, 5), (128, 8)])
def test_box_matches_oracle(qpb, n, count):
    H, f, lb, ub = _family(100 + n, count, n)
    x, lam, act, st, it = _np(qpb.solve_box(*_cuda(H, f, lb, ub)))
    assert (st == qpb.OK).all(), st
    A, b = _dense(lb, ub)
    r = O.kkt_residuals(H, f, A, b, x, lam)
    assert max(float(v.max()) for v in r.values()) <= 1e-9, r
    mask = qpb.active_mask_to_bool(act, 2 * n)
    for i in range(count):
        ref = O.active_set_solve(H[i], f[i], A[i], b[i])
        assert ref.status == 0
        assert np.abs(x[i] - ref.x).max() / max(1.0, np.abs(ref.x).max()) <= TOL, i
        assert np.array_equal(mask[i], ref.active), i
        assert np.abs(lam[i] - ref.lam).max() / (1.0 + np.abs(ref.lam).max()) <= TOL, i


@pytest.mark.parametrize("n", [16, 9, 20, 32, 40, 128])
def test_box_matches_dense_path(qpb, n):
    """The same QPs through qpb_solve with the dense A = [I; -I]: same active
    sets and statuses, x and lambda to rounding."""
    B = 8192 + 3 if n <= 32 else 1027  # ragged last group
    H, f, lb, ub = _family(7 + n, B, n)
    A, b = _dense(lb, ub)
    xb, lb_, ab, sb, ib = _np(qpb.solve_box(*_cuda(H, f, lb, ub)))
    xd, ld, ad, sd, idd = _np(qpb.solve(*_cuda(H, f, A, b)))
    assert (sb == qpb.OK).all() and (sd == qpb.OK).all()
    assert np.array_equal(ab, ad)
    assert np.abs(xb - xd).max() <= 1e-12 * max(1.0, np.abs(xd).max())
    assert np.abs(lb_ - ld).max() <= 1e-10 * (1.0 + np.abs(ld).max())
    assert np.abs(ib.astype(int) - idd.astype(int)).max() <= 2  # selection ties may reorder steps


@pytest.mark.parametrize("n", [16, 32, 64])
def test_box_one_sided_and_absent_bounds(qpb, n):
    B = 200
    H, f, lb, ub = _family(31, B, n)
    # no bounds at all: the unconstrained minimiser
    x, lam, act, st, _ = _np(qpb.solve_box(*_cuda(H, f, None, None)))
    assert (st == qpb.OK).all() and (act == 0).all() and (lam == 0).all()
    x0 = np.linalg.solve(H, -f[..., None])[..., 0]
    assert np.abs(x - x0).max() <= 1e-9 * max(1.0, np.abs(x0).max())
    # upper bounds only (lb NULL) == lb = -inf, and both equal the dense form without the lower rows
    xa, la, aa, sa, _ = _np(qpb.solve_box(*_cuda(H, f, None, ub)))
    xi, li, ai, si, _ = _np(qpb.solve_box(*_cuda(H, f, np.full_like(lb, -np.inf), ub)))
    assert (sa == qpb.OK).all() and np.array_equal(xa, xi) and np.array_equal(aa, ai)
    assert (la[:, n:] == 0).all()
    A = np.ascontiguousarray(np.broadcast_to(np.eye(n), (B, n, n)))
    xd, ld, ad, sd, _ = _np(qpb.solve(*_cuda(H, f, A, ub)))
    assert np.abs(xa - xd).max() <= 1e-12 * max(1.0, np.abs(xd).max())
    assert np.array_equal(qpb.active_mask_to_bool(aa, 2 * n)[:, :n], qpb.active_mask_to_bool(ad, n))


@pytest.mark.parametrize("n", [16, 32, 80])
def test_box_statuses(qpb, n):
    H, f, lb, ub = _family(5, 8, n)
    lb[3, 2] = ub[3, 2] + 1.0  # empty box -> INFEASIBLE
    H[5] = -H[5]  # not SPD
    x, lam, act, st, _ = _np(qpb.solve_box(*_cuda(H, f, lb, ub)))
    assert st[3] == qpb.INFEASIBLE and st[5] == qpb.NOT_SPD
    others = [i for i in range(8) if i not in (3, 5)]
    assert (st[others] == qpb.OK).all()
    # a bad QP never disturbs its neighbours: the others equal a solve without them
    x2, *_ = _np(qpb.solve_box(*_cuda(H[others], f[others], lb[others], ub[others])))
    assert np.array_equal(x[others], x2)


def test_box_metric_batch_kkt(qpb):
    """The bench's box QPs (|x| <= 10) at the metric's batch: KKT on every QP."""
    B, n = 1 << 20, 16
    H, f, A, b = qpb.generate(n, B, 20261015, family="box", device=torch.device("cuda", 0))
    lb = torch.full((B, n), -10.0, dtype=torch.float64, device=f.device)
    ub = -lb
    sol = qpb.solve_box(H, f, lb, ub)
    dense = qpb.solve(H, f, A, b)
    torch.cuda.synchronize()
    assert bool((sol.status == qpb.OK).all())
    assert torch.equal(sol.active, dense.active)
    assert float((sol.x - dense.x).abs().max()) <= 1e-10
    # KKT of the box answer on a sample of 4096 QPs (oracle residuals on the host)
    idx = torch.arange(0, B, B // 4096, device=f.device)
    Hs, fs, As, bs = (t[idx].cpu().numpy() for t in (H, f, A, b))
    r = O.kkt_residuals(Hs, fs, As, bs, sol.x[idx].cpu().numpy(), sol.lam[idx].cpu().numpy())
    assert max(float(v.max()) for v in r.values()) <= 1e-9


@pytest.mark.parametrize("n", [16, 5, 32, 24])
def test_box_tiny_hessian_only_first_bound_violated(qpb, n):
    """ADVICE r03 on the box kernel: H = 1e-40 I and f scaled with it, only
    x_0's upper bound violated at the unconstrained minimiser.  The selection
    key of that single violated bound must not round to the "none violated"
    key: x* = (1, -f0[1:]), one active bound."""
    B = 8
    rs = np.random.default_rng(n)
    f0 = rs.uniform(-0.5, 0.5, size=(B, n))
    f0[:, 0] = -3.0
    H = np.broadcast_to(np.eye(n), (B, n, n)) * 1e-40
    lb, ub = -np.ones((B, n)), np.ones((B, n))
    sol = qpb.solve_box(*_cuda(np.ascontiguousarray(H), f0 * 1e-40, lb, ub))
    x, lam, act, st, it = _np(sol)
    assert (st == qpb.OK).all(), st
    x_ref = -f0.copy()
    x_ref[:, 0] = 1.0
    assert np.abs(x - x_ref).max() <= 1e-9
    mask = qpb.active_mask_to_bool(act, 2 * n)
    assert mask[:, 0].all() and mask.sum(axis=1).tolist() == [1] * B


def test_box_config4_shape_batch(qpb):
    """n = 32 (the configs[4] size class) at B = 262,144: the implicit-A box
    kernel and the dense path on A = [I; -I] choose the same active set for
    every QP, x to rounding, KKT on a sample of 2048 QPs."""
    B, n = 262144, 32
    H, f, A, b = qpb.generate(n, B, 20261015, family="box", device=torch.device("cuda", 0))
    ub = b[:, :n].contiguous()
    lb = (-b[:, n:]).contiguous()
    sol = qpb.solve_box(H, f, lb, ub)
    dense = qpb.solve(H, f, A, b)
    torch.cuda.synchronize()
    assert bool((sol.status == qpb.OK).all()) and bool((dense.status == qpb.OK).all())
    assert torch.equal(sol.active, dense.active)
    assert float((sol.x - dense.x).abs().max() / dense.x.abs().max().clamp(min=1.0)) <= 1e-10
    idx = torch.arange(0, B, B // 2048, device=f.device)
    Hs, fs, As, bs = (t[idx].cpu().numpy() for t in (H, f, A, b))
    r = O.kkt_residuals(Hs, fs, As, bs, sol.x[idx].cpu().numpy(), sol.lam[idx].cpu().numpy())
    assert max(float(v.max()) for v in r.values()) <= 1e-9


def test_box_config3_shape_batch(qpb):
    """n = 128 (BASELINE configs[3]'s size) at its batch B = 16 384 through
    the box entry point (the BOX form of the n <= 128 kernel, A implicit)
    against the dense path on A = [I; -I]: the same active set on every QP, x
    to rounding, KKT on a sample of 1024 QPs, the oracle on 16."""
    B, n = 16384, 128
    H, f, A, b = qpb.generate(n, B, 20261015, family="box", device=torch.device("cuda", 0))
    ub = b[:, :n].contiguous()
    lb = (-b[:, n:]).contiguous()
    sol = qpb.solve_box(H, f, lb, ub)
    dense = qpb.solve(H, f, A, b)
    torch.cuda.synchronize()
    assert bool((sol.status == qpb.OK).all()) and bool((dense.status == qpb.OK).all())
    assert torch.equal(sol.active, dense.active)
    assert float((sol.x - dense.x).abs().max() / dense.x.abs().max().clamp(min=1.0)) <= 1e-10
    idx = torch.arange(0, B, B // 1024, device=f.device)
    Hs, fs, As, bs = (t[idx].cpu().numpy() for t in (H, f, A, b))
    xs, ls = sol.x[idx].cpu().numpy(), sol.lam[idx].cpu().numpy()
    r = O.kkt_residuals(Hs, fs, As, bs, xs, ls)
    assert max(float(v.max()) for v in r.values()) <= 1e-9
    mask = qpb.active_mask_to_bool(sol.active[idx].cpu().numpy(), 2 * n)
    for k in range(0, len(idx), 64):
        ref = O.active_set_solve(Hs[k], fs[k], As[k], bs[k])
        assert ref.status == 0
        assert np.abs(xs[k] - ref.x).max() / max(1.0, np.abs(ref.x).max()) <= TOL, k
        assert np.array_equal(mask[k], ref.active), k


def test_box_beyond_128_is_unsupported(qpb):
    H, f, lb, ub = _family(3, 2, 129)
    with pytest.raises(qpb.QPBError):
        qpb.solve_box(*_cuda(H, f, lb, ub))
