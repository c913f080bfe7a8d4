"""CPU test of tools/config_sweep.py's measurement order (VERDICT r05 Weak 6):
the success fraction and iteration counts come from the full solve, before the
max_iter = 1 ablation reuses (and overwrites) the output buffers."""
import os
import sys
import types

import pytest

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def sweep():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    sys.path.insert(0, ROOT)
    import config_sweep
    return config_sweep


def test_ok_frac_is_read_before_the_ablation(sweep):
    OK, MAX_ITER, B = 0, 1, 64
    calls = []

    def run(mi=0, out=None):
        calls.append(mi)
        sol = out or types.SimpleNamespace(status=torch.zeros(B, dtype=torch.int32),
                                           iters=torch.zeros(B, dtype=torch.int32))
        # the full solve: every QP OK in 5 iterations; max_iter = 1: MAX_ITER, 1
        sol.status.fill_(OK if mi == 0 else MAX_ITER)
        sol.iters.fill_(5 if mi == 0 else 1)
        return sol

    def timer(fn, reps):
        for _ in range(reps):
            fn()
        return 1.0

    res = sweep.measure(run, 3, OK, lambda: None, timer)
    assert res["ok_frac"] == 1.0 and res["iters_mean"] == 5.0 and res["iters_max"] == 5
    assert calls[0] == 0 and calls[-1] == 1  # the ablation ran last and did not change the record
    assert res["kernel_ms"] == 1.0 and res["maxit1_ms"] == 1.0
