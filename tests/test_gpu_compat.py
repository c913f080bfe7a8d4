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


@pytest.mark.parametrize("which,iters,count", [("newton", 10, 2), ("admm", 10000, 1), ("gd", 20, 2)])
def test_compat_solvers_at_ndim_200(which, iters, count):
    """The compat API at N_DIM = 200 (round 6: the solvers used to refuse
    N_DIM > 128): tests/compat/compat_driver_n200, a C caller built with
    -DN_DIM=200U, against the compiled reference at N_DIM = 200 on the same
    srand sequence -- bitwise (the replicas' global layout, qpb_ref.hip)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import refc
    drv = DRIVER + "_n200"
    if not os.path.exists(drv) or not refc.available(200, "1e12"):
        pytest.skip("compat_driver_n200 or oracle/_ref not built")
    out = subprocess.run([drv, which, "7", str(count), str(iters)], capture_output=True, timeout=600)
    assert out.returncode == 0, out.stderr.decode()
    x = np.frombuffer(out.stdout, dtype=np.float64).reshape(count, -1)
    rc = refc.RefC(200, "1e12")
    P, q, x0 = rc.generate(seed=7, count=count)
    ref = getattr(rc, which)(P, q, x0, iters)
    assert np.array_equal(x, ref)
