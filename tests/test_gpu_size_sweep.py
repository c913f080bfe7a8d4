"""GPU parity across the size classes at odd shapes: the padded n < 16 rows and
masked m < 32 rows of the 16-lane kernel (qpb_gi.hip, MR = 1 and 2), the
one-QP-per-wavefront kernel past either bound (qpb_gi_wave.hip), and the
n <= 128 Gram kernel (qpb_gi_gram.hip) at n = 33 (one padded 16-column tile).
Oracle: the KKT-certified primal active set (oracle.active_set_solve) on every
QP -- x and lambda within 1e-6 relative, the active set bit-exact -- and the
KKT certificate (<= 1e-9) on the GPU's own answer.  Through the C-ABI."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402

TOL = 1e-6

SHAPES = [
    # 16-lane kernel, one D row per lane (m <= 16) and two (16 < m <= 32)
    (1, 1, "dense"), (1, 2, "box"), (2, 3, "dense"), (3, 5, "dense"), (3, 6, "box"), (5, 1, "dense"),
    (7, 9, "dense"), (7, 14, "box"), (9, 16, "dense"), (13, 17, "dense"), (13, 26, "box"), (15, 31, "dense"),
    (16, 1, "dense"), (16, 17, "dense"), (11, 32, "dense"),
    # one QP per wavefront: n past 16 or m past 32
    (17, 1, "dense"), (19, 33, "dense"), (21, 42, "box"), (31, 63, "dense"), (6, 50, "dense"), (32, 33, "dense"),
    # Gram kernel (n > 32 or m > 64)
    (33, 7, "dense"), (12, 65, "dense"), (40, 80, "box"),
]


@pytest.fixture(scope="module")
def qpb():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import qpb as q
    return q


@pytest.mark.parametrize("n,m,kind", SHAPES)
def test_size_sweep(qpb, n, m, kind):
    count = 4 if n > 32 or m > 64 else 9  # 9: a ragged last group of the 4-QP kernel
    H, f, A, b = O.family_conditioned(7919 * n + 31 * m, count, n, m=m, box=10.0, kind=kind)
    dev = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (H, f, A, b)]
    sol = qpb.solve(*dev)
    torch.cuda.synchronize()
    x, lam, act, st = (t.cpu().numpy() for t in (sol.x, sol.lam, sol.active, sol.status))
    assert (st == qpb.OK).all(), st
    r = O.kkt_residuals(H, f, A, b, x, lam)
    assert max(float(v.max()) for v in r.values()) <= 1e-9, r
    mask = qpb.active_mask_to_bool(act, m)
    for i in range(count):
        ref = O.active_set_solve(H[i], f[i], A[i], b[i])
        assert ref.status == 0
        assert np.abs(x[i] - ref.x).max() / max(1.0, np.abs(ref.x).max()) <= TOL, (i, x[i], ref.x)
        assert np.array_equal(mask[i], ref.active), i
        assert np.abs(lam[i] - ref.lam).max() / (1.0 + np.abs(ref.lam).max()) <= TOL, i
