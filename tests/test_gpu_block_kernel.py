"""GPU parity of the one-QP-per-workgroup active-set kernel for the n <= 128
class (qpb_gi_gram.hip): 32 < n <= 128, m <= 256, including BASELINE configs[3]'s
shape n=128, m=256.
Oracle: oracle.active_set_solve (KKT-certified primal active set) per QP;
x within 1e-6 relative, active set bit-exact, multipliers within 1e-6, and the
KKT certificate on every GPU answer.  Calls go through the C-ABI."""
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


def _solve(qpb, H, f, A=None, b=None, flags=0):
    dev = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in ((H, f) if A is None else (H, f, A, b))]
    sol = qpb.solve(*dev, flags=flags)
    torch.cuda.synchronize()
    return [t.cpu().numpy() for t in sol]


def _relerr(x, ref):
    return np.abs(x - ref).max(axis=1) / np.maximum(1.0, np.abs(ref).max(axis=1))


@pytest.mark.parametrize("n,m,kind,count", [(48, 96, "box", 6), (64, 128, "dense", 6), (33, 200, "dense", 4),
                                            (128, 256, "box", 3), (128, 256, "dense", 2), (100, 40, "dense", 3)])
def test_block_kernel_matches_oracle(qpb, n, m, kind, count):
    H, f, A, b = O.family_conditioned(2000 + n + m, count, n, m=m, box=10.0, kind=kind)
    x, lam, act, st, it = _solve(qpb, H, f, A, b)
    assert (st == qpb.OK).all(), st
    r = O.kkt_residuals(H, f, A, b, x, lam)
    assert max(float(v.max()) for v in r.values()) <= 1e-9, {k: float(v.max()) for k, v in r.items()}
    mask = qpb.active_mask_to_bool(act, m)
    for i in range(count):
        ref = O.active_set_solve(H[i], f[i], A[i], b[i])
        assert ref.status == 0
        assert _relerr(x[i:i + 1], ref.x[None]).max() <= X_TOL, i
        assert np.array_equal(mask[i], ref.active), i
        assert np.abs(lam[i] - ref.lam).max() / (1 + np.abs(ref.lam).max()) <= X_TOL


def test_block_kernel_unconstrained(qpb):
    H, f, _, _ = O.family_conditioned(77, 5, 128, box=10.0)
    x, lam, act, st, it = _solve(qpb, H, f)
    assert (st == qpb.OK).all()
    assert _relerr(x, np.linalg.solve(H, -f[..., None])[..., 0]).max() <= 1e-9


@pytest.mark.parametrize("kind", ["box", "dense"])
def test_config3_full_batch(qpb, kind):
    """BASELINE configs[3] as specified (n=128, m=256, B=16384) from the
    on-device generator: every QP KKT-certified, 128 QPs spread over the batch
    against the oracle (x, mask)."""
    B = 16384
    H, f, A, b = qpb.generate(128, B, 20261015, family=kind)
    sol = qpb.solve(H, f, A, b)
    torch.cuda.synchronize()
    st = sol.status.cpu().numpy()
    assert (st == qpb.OK).all(), np.bincount(st)
    x, lam = sol.x.cpu().numpy(), sol.lam.cpu().numpy()
    mask = qpb.active_mask_to_bool(sol.active.cpu().numpy(), 256)
    for k0 in range(0, B, 2048):  # KKT on every QP, in host-memory-sized chunks
        sl = slice(k0, k0 + 2048)
        Hn, fn, An, bn = (t[sl].cpu().numpy() for t in (H, f, A, b))
        r = O.kkt_residuals(Hn, fn, An, bn, x[sl], lam[sl])
        assert max(float(v.max()) for v in r.values()) <= 1e-9, (k0, {k: float(v.max()) for k, v in r.items()})
    idx = np.linspace(0, B - 1, 128).astype(int)
    Hn, fn, An, bn = (t[idx].cpu().numpy() for t in (H, f, A, b))
    for j, i in enumerate(idx):
        ref = O.active_set_solve(Hn[j], fn[j], An[j], bn[j])
        assert ref.status == 0
        assert _relerr(x[i:i + 1], ref.x[None]).max() <= X_TOL, i
        assert np.array_equal(mask[i], ref.active), i
