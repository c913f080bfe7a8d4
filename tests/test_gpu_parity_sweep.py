"""A parity sweep larger than the per-feature tests' samples: qpb_solve (and
qpb_solve_box for the box family) against the primal active-set oracle
(oracle/oracle.py: N&W 16.3 with the round-6 stall and Bland rules) on K QPs
drawn from a B-QP batch per (n, family): every checked QP's active set bit
for bit, x within the 1e-6 relative tolerance north_star states, every GPU
status OK, and the box entry point's active sets equal to the dense path's
on the whole batch.

The default samples keep the test to a few seconds; QPB_PARITY_SCALE=8
checks every QP of configs[1]'s 65 536-QP batch at n = 16 (8 192 of 16 384
at n = 32, 256 of 1 024 at n = 128), and QPB_PARITY_OUT=<file> writes the
per-row results as JSON (profiles/r06/parity/).
"""
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

X_TOL = 1e-6
SCALE = int(os.environ.get("QPB_PARITY_SCALE", "1"))
ROWS = [(16, "box", 65536, 8192), (16, "dense", 65536, 8192), (32, "box", 16384, 1024),
        (32, "dense", 16384, 1024), (128, "box", 1024, 32), (128, "dense", 1024, 32)]
RESULTS = []


@pytest.fixture(scope="module")
def qpb():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import qpb as q
    yield q
    out = os.environ.get("QPB_PARITY_OUT")
    if out and RESULTS:
        with open(out, "w") as fh:
            json.dump({"library": q.version(), "scale": SCALE, "rows": RESULTS}, fh, indent=1)


def _mask_bits(active, m):
    a = active.cpu().numpy().astype(np.uint32)
    bits = (a[:, :, None] >> np.arange(32, dtype=np.uint32)) & 1
    return bits.reshape(a.shape[0], -1)[:, :m].astype(bool)


@pytest.mark.parametrize("n,fam,B,K", ROWS)
def test_parity_sweep(qpb, n, fam, B, K):
    import oracle as O
    dev = torch.device("cuda", 0)
    K = min(B, K * SCALE)
    H, f, A, b = qpb.generate(n, B, 4242, family=fam, shift=1.0, box=10.0, device=dev)
    m = A.shape[1]
    sol = qpb.solve(H, f, A, b)
    torch.cuda.synchronize()
    assert bool((sol.status == qpb.OK).all())
    row = {"n": n, "m": m, "family": fam, "batch": B, "sample": K}
    if fam == "box":
        bsol = qpb.solve_box(H, f, (-b[:, n:]).contiguous(), b[:, :n].contiguous())
        torch.cuda.synchronize()
        assert bool((bsol.status == qpb.OK).all())
        assert torch.equal(bsol.active, sol.active)
        row["box_max_abs_x_diff_vs_dense"] = float((bsol.x - sol.x).abs().max())
        assert row["box_max_abs_x_diff_vs_dense"] <= X_TOL * max(1.0, float(sol.x.abs().max()))
    idx = np.sort(np.random.default_rng(4242 + n).choice(B, size=K, replace=False))
    ti = torch.from_numpy(idx).to(dev)
    Hs, fs, As, bs = (t.index_select(0, ti).cpu().numpy() for t in (H, f, A, b))
    xs = sol.x.index_select(0, ti).cpu().numpy()
    ms = _mask_bits(sol.active.index_select(0, ti), m)
    worst, bad = 0.0, []
    for k in range(K):
        ref = O.active_set_solve(Hs[k], fs[k], As[k], bs[k])
        assert ref.status == 0, idx[k]
        worst = max(worst, float(np.abs(xs[k] - ref.x).max() / max(1.0, np.abs(ref.x).max())))
        if not np.array_equal(ms[k], ref.active):
            bad.append(int(idx[k]))
    row.update({"checked": K, "max_rel_x_err": worst, "mask_mismatches": len(bad), "x_tol": X_TOL})
    RESULTS.append(row)
    assert not bad, bad[:10]
    assert worst <= X_TOL, worst
