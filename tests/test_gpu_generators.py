"""GPU parity of the on-device generators (csrc/qpb_gen.hip).

qpb_ref_generate must reproduce the reference generator bit for bit: the
golden fixtures hold P, q, x0 drawn by the compiled reference C itself
(oracle/ref_driver.c, srand(seed) then main.c:37-39 order), and far-away QPs
are checked against the jump-ahead restatement.  qpb_generate is checked
against the numpy Philox restatement: bit-exact where no floating-point sum
is involved (f, box A/b, dense b), H to 1e-13 relative (the matrix cores
sum in their own order), dense A to 1e-13 (device libm log/cos).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle  # noqa: E402


@pytest.fixture(scope="module")
def qpb():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import qpb as q
    return q


@pytest.mark.parametrize("n,seed,count", [(4, 4001, 32), (16, 16001, 32), (32, 32001, 12)])
def test_ref_generate_bitexact_vs_reference_c(qpb, n, seed, count):
    g = np.load(os.path.join(GOLDEN, f"ref_n{n}.npz"))
    P, q, x0 = qpb.ref_generate(n, count, seed)
    torch.cuda.synchronize()
    assert np.array_equal(P.cpu().numpy(), g["P"][:count])
    assert np.array_equal(q.cpu().numpy(), g["q"][:count])
    assert np.array_equal(x0.cpu().numpy(), g["x0"][:count])


def test_ref_generate_shards_and_far_qps(qpb):
    n, seed = 16, 20261015
    P, q, x0 = qpb.ref_generate(n, 65536, seed)
    Ps, qs, xs = qpb.ref_generate(n, 7, seed, first=40000)
    torch.cuda.synchronize()
    assert torch.equal(Ps, P[40000:40007]) and torch.equal(qs, q[40000:40007]) and torch.equal(xs, x0[40000:40007])
    for k in (0, 1, 4095, 65535):
        Pk, qk, xk = oracle.ref_generate_at(seed, k, n)
        assert np.array_equal(P[k].cpu().numpy(), Pk)
        assert np.array_equal(q[k].cpu().numpy(), qk) and np.array_equal(x0[k].cpu().numpy(), xk)


@pytest.mark.parametrize("n,family", [(16, "box"), (16, "dense"), (4, "box"), (10, "dense"), (32, "box"),
                                      (128, "dense")])
def test_generate_matches_restatement(qpb, n, family):
    batch, seed = (8 if n > 32 else 64), 777
    H, f, A, b = qpb.generate(n, batch, seed, family=family, first=3)
    torch.cuda.synchronize()
    Hr, fr, Ar, br = oracle.family_generate(n, batch, seed, family, first=3)
    H, f, A, b = (t.cpu().numpy() for t in (H, f, A, b))
    assert np.array_equal(H, np.transpose(H, (0, 2, 1)))  # stored symmetric
    assert np.max(np.abs(H - Hr) / np.abs(Hr).max(axis=(1, 2), keepdims=True)) <= 1e-13
    assert np.array_equal(f, fr)
    if family == "box":
        assert np.array_equal(A, Ar) and np.array_equal(b, br)
    else:
        assert np.max(np.abs(A - Ar)) <= 1e-13 and np.array_equal(b, br)


def test_generate_shard_identity_and_solvable(qpb):
    H, f, A, b = qpb.generate(16, 4096, 5)
    Hs, fs, As, bs = qpb.generate(16, 100, 5, first=1000)
    torch.cuda.synchronize()
    for full, part in ((H, Hs), (f, fs), (A, As), (b, bs)):
        assert torch.equal(full[1000:1100], part)
    sol = qpb.solve(H, f, A, b)
    torch.cuda.synchronize()
    assert int((sol.status != 0).sum()) == 0


def test_generator_argument_errors(qpb):
    with pytest.raises(qpb.QPBError):
        qpb.generate(16, 4, 1, m=20)  # box family needs m = 2n
    with pytest.raises(qpb.QPBError):
        qpb.ref_generate(129, 1, 1)  # n <= 128 (QPB_MAX_N)
