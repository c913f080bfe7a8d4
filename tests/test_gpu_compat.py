"""GPU: the reference-compatible C API end to end.

* tests/compat/compat_driver (a C program using kmalloc/matrix_ops/qp/
  qp_solvers exactly like the reference's main.c) reproduces the compiled
  reference's Newton / ADMM / GD answers for the same srand seed;
* the reference's own main.c + test/test.c linked against libqpb.so
  (oracle/_ref/ref_main_on_qpb) runs to completion.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu
DRIVER = os.path.join(ROOT, "tests", "compat", "compat_driver")


def run_driver(which, seed, count, iters):
    if not os.path.exists(DRIVER):
        pytest.skip("compat_driver not built (make -C embedded-qp-solver_amd)")
    out = subprocess.run([DRIVER, which, str(seed), str(count), str(iters)], capture_output=True, timeout=600)
    assert out.returncode == 0, out.stderr.decode()
    return np.frombuffer(out.stdout, dtype=np.float64).reshape(count, -1)


@pytest.mark.parametrize("which,key,iters,count", [("newton", "newton_x", 10, 32), ("admm", "admm_x_inactive", 10000, 32),
                                                   ("gd", "gd_x", 10000, 8)])
def test_compat_solvers_reproduce_reference(which, key, iters, count):
    g = np.load(os.path.join(GOLDEN, "ref_n16.npz"))
    x = run_driver(which, 16001, count, iters)
    ref = g[key][:count]
    err = np.abs(x - ref).max(1) / np.abs(ref).max(1)
    assert err.max() <= 1e-6, err


def test_reference_main_runs_on_compat():
    path = os.path.join(ROOT, "oracle", "_ref", "ref_main_on_qpb")
    if not os.path.exists(path):
        pytest.skip("reference build not present")
    out = subprocess.run([path], capture_output=True, timeout=900, cwd=os.path.join(ROOT, "tests"))
    assert out.returncode == 0, out.stderr.decode()[-2000:]
    text = out.stdout.decode()
    assert "inversion tests completed" in text and "scalar_prod test completed" in text
    for name in ("gradient_descent_with_line_search gave:", "newton_method_with_line_search gave:", "admm gave:"):
        assert text.count(name) == 16, name
    assert "error in mult test" not in out.stderr.decode()
