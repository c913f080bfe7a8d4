"""The ctypes stub INTEGRATION.md §3 hands to a maintainer of test/qp_ref.py
(the replacement of qpsolvers.solve_qp, qp_ref.py:35), run as written: its
text is taken from INTEGRATION.md, so the document cannot drift from a
working binding.  Round 3's stub allocated one active-set word for any m (a
heap overflow at m > 32); the m = 64 case below would write past it."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _stub():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    head = text.index("**Python (`test/qp_ref.py`, ctypes).**")
    block = re.search(r"```python\n(.*?)```", text[head:], re.S).group(1)
    block = block.replace('"embedded-qp-solver_amd/lib/libqpb.so"',
                          repr(os.path.join(ROOT, "embedded-qp-solver_amd", "lib", "libqpb.so")))
    env = {}
    exec(compile(block, "INTEGRATION.md", "exec"), env)  # noqa: S102 (our own document)
    return env["solve_qp"]


@pytest.fixture(scope="module")
def solve_qp():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return _stub()


def _oracle():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    return oracle


def test_stub_unconstrained_is_qp_ref(solve_qp):
    O = _oracle()
    P, q, _ = O.ref_generate(5, 3, 16)
    for k in range(3):
        x = solve_qp(P[k], q[k])
        ref = np.linalg.solve(P[k], -q[k])
        tol = max(1e-6, 1e-14 * np.linalg.cond(P[k]))  # the reference generator's heavy-tailed cond
        assert np.abs(x - ref).max() <= tol * max(1.0, np.abs(ref).max())


@pytest.mark.parametrize("n,m", [(16, 32), (32, 64), (20, 40)])
def test_stub_constrained_matches_oracle(solve_qp, n, m):
    O = _oracle()
    rng = np.random.default_rng(n * 1000 + m)
    B = rng.standard_normal((n, n))
    P = B.T @ B / n + np.eye(n)
    q = rng.uniform(-10, 10, n)
    G = rng.standard_normal((m, n))
    G /= np.linalg.norm(G, axis=1, keepdims=True)
    h = rng.uniform(0.1, 1.0, m)
    x = solve_qp(P, q, G, h)
    r = O.active_set_solve(P, q, G, h)
    assert r.status == 0
    assert np.abs(x - r.x).max() <= 1e-6 * max(1.0, np.abs(r.x).max())
