"""The metric's batch (BASELINE.json configs[2]: 1,048,576 QPs, n=16, m=32) on
one GPU, and ragged batches around it.

* B = 1,048,576, box and dense families generated on the GPU (qpb_generate):
  the KKT certificate of oracle.kkt_residuals (same formulas, evaluated on the
  GPU in fp64 with torch -- test infrastructure) on EVERY QP, statuses all OK,
  plus the independent primal active-set oracle on a sample.
* B = 65,537 / 65,538 / 65,539 (1, 2, 3 QPs in the last 4-QP wavefront of the
  n <= 16 kernel): every QP equals the same QP solved inside a full batch, bit
  for bit, and the ragged tail needs DROP steps (dense family).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

KKT_TOL = 1e-9
X_TOL = 1e-6


@pytest.fixture(scope="module")
def qpb():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import qpb as q
    return q


def kkt_torch(H, f, A, b, x, lam):
    """oracle.kkt_residuals (oracle/oracle.py) on device tensors: worst
    stationarity / primal / dual / complementarity residual over the batch."""
    r = torch.bmm(H, x[:, :, None])[:, :, 0] + f + torch.bmm(A.transpose(1, 2), lam[:, :, None])[:, :, 0]
    xn = x.abs().amax(1)
    Hn = H.abs().sum(2).amax(1)
    stat = r.abs().amax(1) / (1.0 + f.abs().amax(1) + Hn * xn)
    An = A.abs().sum(2).amax(1)
    sc = 1.0 + b.abs().amax(1) + An * xn
    slack = b - torch.bmm(A, x[:, :, None])[:, :, 0]
    prim = torch.clamp(-slack.amin(1), min=0.0) / sc
    ln = 1.0 + lam.abs().amax(1)
    dual = torch.clamp(-lam.amin(1), min=0.0) / ln
    comp = (lam * slack).abs().amax(1) / (ln * sc)
    return {k: float(v.max()) for k, v in (("stat", stat), ("prim", prim), ("dual", dual), ("comp", comp))}


@pytest.mark.parametrize("family", ["box", "dense"])
def test_metric_batch_1m(qpb, family):
    import oracle as O
    B = 1 << 20
    H, f, A, b = qpb.generate(16, B, 20261015, family=family, shift=1.0, box=10.0)
    sol = qpb.solve(H, f, A, b)
    torch.cuda.synchronize()
    st = sol.status
    assert bool((st == qpb.OK).all()), torch.bincount(st.long()).tolist()
    worst = kkt_torch(H, f, A, b, sol.x, sol.lam)
    assert all(v <= KKT_TOL for v in worst.values()), worst
    # active mask == positive multipliers
    bits = ((sol.active.long() & 0xFFFFFFFF)[:, :, None] >> torch.arange(32, device=st.device)) & 1
    mask = bits.reshape(B, -1)[:, :32].bool()
    assert float((mask == (sol.lam > 0)).double().mean()) > 0.9999
    # independent primal oracle on a sample spread over the batch
    idx = np.random.default_rng(1).choice(B, size=1022, replace=False)
    idx = np.concatenate([idx, [0, B - 1]])
    Hs, fs, As, bs = (t[idx].cpu().numpy() for t in (H, f, A, b))
    xs, ms = sol.x[idx].cpu().numpy(), mask[idx].cpu().numpy()
    for k in range(len(idx)):
        ref = O.active_set_solve(Hs[k], fs[k], As[k], bs[k])
        assert ref.status == 0
        err = np.abs(xs[k] - ref.x).max() / max(1.0, np.abs(ref.x).max())
        assert err <= X_TOL, (idx[k], err)
        assert np.array_equal(ms[k], ref.active), idx[k]


@pytest.mark.parametrize("B", [65537, 65538, 65539])
def test_ragged_last_wavefront(qpb, B):
    Bf = 65540  # whole wavefronts
    H, f, A, b = qpb.generate(16, Bf, 4242, family="dense", shift=1.0, box=10.0)
    full = qpb.solve(H, f, A, b)
    part = qpb.solve(H[:B].contiguous(), f[:B].contiguous(), A[:B].contiguous(), b[:B].contiguous())
    torch.cuda.synchronize()
    for k in ("x", "lam", "active", "status", "iters"):
        assert torch.equal(getattr(part, k), getattr(full, k)[:B]), k
    assert bool((part.status == qpb.OK).all())
    # the dense family drops constraints: some QPs of the run need DROP steps
    # (iterations beyond the final active-set size + 1)
    nact = torch.tensor([bin(int(w) & 0xFFFFFFFF).count("1") for w in part.active[:, 0].cpu()])
    assert bool((part.iters.cpu() > nact + 1).any())
    # and the tail QPs alone, each as a batch of its own
    for g in range(B - (B % 4 or 4), B):
        one = qpb.solve(H[g:g + 1].contiguous(), f[g:g + 1].contiguous(), A[g:g + 1].contiguous(),
                        b[g:g + 1].contiguous())
        torch.cuda.synchronize()
        assert torch.equal(one.x[0], full.x[g]) and torch.equal(one.lam[0], full.lam[g])
