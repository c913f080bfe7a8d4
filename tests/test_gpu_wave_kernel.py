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


@pytest.mark.parametrize("family", ["dense", "box"])
def test_wave_kernel_config5_full_batch(qpb, family):
    """BASELINE configs[4]'s shape at its full batch (n = 32, m = 64,
    B = 262 144, fp64 default path) from the on-device generator: the KKT
    certificate on every QP (evaluated on the device), and 48 QPs spread over
    the whole batch -- the first, the last and random ones -- against the
    oracle (x, lambda within 1e-6, active set bit-exact)."""
    from conftest import kkt_max_residual_device
    B = 262144
    H, f, A, b = qpb.generate(32, B, 20261015, family=family)
    sol = qpb.solve(H, f, A, b)
    torch.cuda.synchronize()
    st = sol.status.cpu().numpy()
    assert (st == qpb.OK).all(), np.bincount(st)
    assert kkt_max_residual_device(H, f, A, b, sol.x, sol.lam) <= 1e-9
    mask = qpb.active_mask_to_bool(sol.active.cpu().numpy(), 64)
    pick = np.r_[0, 1, B - 2, B - 1, np.random.default_rng(5).choice(B, 44, replace=False)]
    x, lam = sol.x[pick].cpu().numpy(), sol.lam[pick].cpu().numpy()
    Hn, fn, An, bn = (t[pick].cpu().numpy() for t in (H, f, A, b))
    for k, i in enumerate(pick):
        ref = O.active_set_solve(Hn[k], fn[k], An[k], bn[k])
        assert ref.status == 0
        assert _relerr(x[k:k + 1], ref.x[None]).max() <= X_TOL, i
        assert np.array_equal(mask[i], ref.active), i
        assert np.abs(lam[k] - ref.lam).max() / (1 + np.abs(ref.lam).max()) <= X_TOL, i


@pytest.mark.parametrize("n,m,kind", [(1, 2, "box"), (7, 14, "dense"), (13, 20, "dense"), (13, 26, "box"),
                                      (16, 32, "box"), (5, 31, "dense")])
def test_diag_wave_flag_small_and_odd_sizes(qpb, n, m, kind):
    """QPB_FLAG_DIAG_WAVE routes n <= 16, m <= 32 to the one-QP-per-wavefront
    kernel (the group-size-1 endpoint of DESIGN.md §2.1), which otherwise only
    runs with n > 16 or m > 32: at small and odd shapes its answer
    matches the oracle (x, lambda within 1e-6, active set bit-exact) and the
    four-QPs-per-wavefront kernel's active sets on the same QPs."""
    H, f, A, b = O.family_conditioned(77 + 3 * n + m, 21, n, m=m, box=10.0, kind=kind)
    dev = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (H, f, A, b)]
    wave = qpb.solve(*dev, flags=qpb.FLAG_DIAG_WAVE)
    dense = qpb.solve(*dev)
    torch.cuda.synchronize()
    st = wave.status.cpu().numpy()
    assert (st == qpb.OK).all(), st
    x, lam = wave.x.cpu().numpy(), wave.lam.cpu().numpy()
    mask = qpb.active_mask_to_bool(wave.active.cpu().numpy(), m)
    assert np.array_equal(mask, qpb.active_mask_to_bool(dense.active.cpu().numpy(), m))
    r = O.kkt_residuals(H, f, A, b, x, lam)
    assert max(float(v.max()) for v in r.values()) <= 1e-9
    for i in range(len(f)):
        ref = O.active_set_solve(H[i], f[i], A[i], b[i])
        assert ref.status == 0
        assert _relerr(x[i:i + 1], ref.x[None]).max() <= X_TOL, i
        assert np.array_equal(mask[i], ref.active), i
        assert np.abs(lam[i] - ref.lam).max() / (1 + np.abs(ref.lam).max()) <= X_TOL, i
