"""GPU parity of the one-QP-per-wavefront active-set kernel (qpb_gi_wave.hip):
every size beyond the 16-lane kernel (16 < n <= 32 or 32 < m <= 64), with the
BASELINE config-5 shape n=32, m=64.  Oracle: the KKT-certified primal
active-set solver (oracle.active_set_solve) on each QP; x within 1e-6
relative, active set bit-exact, multipliers within 1e-6, and the KKT
certificate on the GPU's own answer.  All calls go through the C-ABI."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402

X_TOL = 1e-6


@pytest.fixture(scope="module")
def qpb():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import qpb as q
    return q


def _solve(qpb, H, f, A=None, b=None):
    dev = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in ((H, f) if A is None else (H, f, A, b))]
    sol = qpb.solve(*dev)
    torch.cuda.synchronize()
    return [t.cpu().numpy() for t in sol]


def _relerr(x, ref):
    return np.abs(x - ref).max(axis=1) / np.maximum(1.0, np.abs(ref).max(axis=1))


@pytest.mark.parametrize("n,m,kind", [(32, 64, "box"), (32, 64, "dense"), (20, 40, "box"), (24, 48, "dense"),
                                      (17, 34, "dense"), (16, 48, "dense"), (8, 64, "dense"), (32, 40, "dense")])
def test_wave_kernel_matches_oracle(qpb, n, m, kind):
    H, f, A, b = O.family_conditioned(1000 + n * m, 24, n, m=m, box=10.0, kind=kind)
    x, lam, act, st, it = _solve(qpb, H, f, A, b)
    assert (st == qpb.OK).all(), st
    r = O.kkt_residuals(H, f, A, b, x, lam)
    assert max(float(v.max()) for v in r.values()) <= 1e-9
    mask = qpb.active_mask_to_bool(act, m)
    for i in range(len(f)):
        ref = O.active_set_solve(H[i], f[i], A[i], b[i])
        assert ref.status == 0
        assert _relerr(x[i:i + 1], ref.x[None]).max() <= X_TOL, i
        assert np.array_equal(mask[i], ref.active), i
        assert np.abs(lam[i] - ref.lam).max() / (1 + np.abs(ref.lam).max()) <= X_TOL


def test_wave_kernel_unconstrained_and_ragged(qpb):
    H, f, A, b = O.family_conditioned(5, 37, 32, m=64, box=10.0, kind="dense")
    x, *_ = _solve(qpb, H, f)  # m = 0
    assert _relerr(x, np.linalg.solve(H, -f[..., None])[..., 0]).max() <= 1e-9
    full = _solve(qpb, H, f, A, b)
    part = _solve(qpb, H[5:18], f[5:18], A[5:18], b[5:18])
    for a, p in zip(full, part):
        assert np.array_equal(a[5:18], p)


def test_wave_kernel_config5_batch(qpb):
    """BASELINE config 5 shape (n=32, m=64) at a large batch from the on-device
    generator: every QP certified, a sample against the oracle."""
    B = 32768
    H, f, A, b = qpb.generate(32, B, 20261015, family="dense")
    sol = qpb.solve(H, f, A, b)
    torch.cuda.synchronize()
    st = sol.status.cpu().numpy()
    assert (st == qpb.OK).all(), np.bincount(st)
    Hn, fn, An, bn = (t.cpu().numpy() for t in (H, f, A, b))
    x, lam = sol.x.cpu().numpy(), sol.lam.cpu().numpy()
    r = O.kkt_residuals(Hn, fn, An, bn, x, lam)
    assert max(float(v.max()) for v in r.values()) <= 1e-9
    mask = qpb.active_mask_to_bool(sol.active.cpu().numpy(), 64)
    for i in np.random.default_rng(1).choice(B, 12, replace=False):
        ref = O.active_set_solve(Hn[i], fn[i], An[i], bn[i])
        assert _relerr(x[i:i + 1], ref.x[None]).max() <= X_TOL
        assert np.array_equal(mask[i], ref.active)
