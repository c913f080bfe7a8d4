"""CPU tests of the boundary: libqpb.so loads without a GPU, exports every
function declared in include/qpb.h and include/compat/*.h, and its entry
points fail cleanly (no compute, no crash) when no HIP device is present."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

# QPB_LIB: another build of the same library (tests/test_sanitizers.py runs
# this file against the ASan/UBSan build)
LIB = os.environ.get("QPB_LIB", os.path.join(ROOT, "embedded-qp-solver_amd", "lib", "libqpb.so"))
HEADERS = [os.path.join(ROOT, "include", "qpb.h")] + [
    os.path.join(ROOT, "include", "compat", h) for h in ("kmalloc.h", "matrix_ops.h", "qp.h", "qp_solvers.h")]


def declared_functions(path):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"^\s*#.*$", "", src, flags=re.M)
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{}]*\)\s*;", src)
    return {n for n in names if n not in ("sizeof", "defined")}


def exported():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_library_loads_and_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build with make -C embedded-qp-solver_amd"
    ctypes.CDLL(LIB)
    syms = exported()
    for h in HEADERS:
        missing = declared_functions(h) - syms
        assert not missing, (os.path.basename(h), missing)


def test_reference_api_symbols_present():
    # the reference's public prototypes (matrix_ops.h:8-36, qp.h:15-24,
    # qp_solvers.h:4-16, kmalloc.h:16-18) -- spelling included (matirx_...)
    want = {"matrix_trans", "matrix_neg", "matrix_invert", "matrix_norm", "matrix_add", "matrix_sub", "matrix_max",
            "matrix_min", "matrix_scalar_mult", "matrix_mult", "matrix_scalar_prod", "matrix_print",
            "matrix_zero_up", "matrix_identity", "matrix_copy", "matrix_get_entry", "matrix_set_entry",
            "matrix_random", "matirx_random_pos_def", "matrix_alloc", "matrix_free", "random_number",
            "quadratic_form_alloc", "quadratic_form_free", "quadratic_form_eval", "quadratic_form_eval_grad",
            "gradient_descent_with_line_search", "newton_method_with_line_search", "admm", "kmalloc", "kfree",
            "kmalloc_init"}
    assert want <= exported()


class Desc(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("m", ctypes.c_int32), ("batch", ctypes.c_int64),
                ("max_iter", ctypes.c_int32), ("flags", ctypes.c_int32), ("feas_tol", ctypes.c_double)]


def test_desc_layout_matches_header():
    assert ctypes.sizeof(Desc) == 32
    assert Desc.batch.offset == 8 and Desc.feas_tol.offset == 24


def test_argument_errors_without_gpu():
    lib = ctypes.CDLL(LIB)
    lib.qpb_last_error.restype = ctypes.c_char_p
    vp = ctypes.c_void_p
    lib.qpb_solve.argtypes = [ctypes.POINTER(Desc)] + [vp] * 10
    # invalid sizes are rejected before any device work
    d = Desc(129, 32, 10, 0, 0, 0.0)
    assert lib.qpb_solve(ctypes.byref(d), *([None] * 10)) == -2  # QPB_ERR_UNSUPPORTED
    d = Desc(0, 0, 10, 0, 0, 0.0)
    assert lib.qpb_solve(ctypes.byref(d), *([None] * 10)) == -1  # QPB_ERR_INVALID_ARG
    assert lib.qpb_solve(None, *([None] * 10)) == -1
    # batch 0 is a no-op
    d = Desc(16, 32, 0, 0, 0, 0.0)
    assert lib.qpb_solve(ctypes.byref(d), *([None] * 10)) == 0
    # a real call with no device fails loudly (never a CPU fallback)
    if not _device_present():
        d = Desc(16, 32, 4, 0, 0, 0.0)
        buf = ctypes.create_string_buffer(64)
        p = ctypes.cast(buf, vp)
        assert lib.qpb_solve(ctypes.byref(d), *([p] * 9), None) == -4  # QPB_ERR_NO_DEVICE
        assert b"no HIP device" in lib.qpb_last_error()


def test_box_argument_errors_without_gpu():
    lib = ctypes.CDLL(LIB)
    lib.qpb_last_error.restype = ctypes.c_char_p
    vp = ctypes.c_void_p
    lib.qpb_solve_box.argtypes = [ctypes.POINTER(Desc)] + [vp] * 10
    d = Desc(16, 30, 4, 0, 0, 0.0)  # m must be 2n
    assert lib.qpb_solve_box(ctypes.byref(d), *([None] * 10)) == -1
    d = Desc(129, 258, 4, 0, 0, 0.0)  # the box kernels cover n <= 128 (round 6; n <= 32 before)
    assert lib.qpb_solve_box(ctypes.byref(d), *([None] * 10)) == -2
    assert b"outside this build" in lib.qpb_last_error()
    for n in (20, 100):  # supported; NULL outputs are refused
        d = Desc(n, 2 * n, 4, 0, 0, 0.0)
        assert lib.qpb_solve_box(ctypes.byref(d), *([None] * 10)) == -1
    d = Desc(16, 32, 0, 0, 0, 0.0)
    assert lib.qpb_solve_box(ctypes.byref(d), *([None] * 10)) == 0
    if not _device_present():
        d = Desc(16, 32, 4, 0, 0, 0.0)
        buf = ctypes.create_string_buffer(64)
        p = ctypes.cast(buf, vp)
        # lb / ub may be NULL (absent bounds); no device -> QPB_ERR_NO_DEVICE
        assert lib.qpb_solve_box(ctypes.byref(d), p, p, None, None, p, p, p, p, None, None) == -4


def _device_present():
    # under the sanitizer run torch stays out of the process (it is not
    # instrumented and only answers this question); that run is CPU-only
    if os.environ.get("QPB_SANITIZED"):
        return False
    import torch
    return torch.cuda.is_available()


@pytest.mark.skipif(bool(os.environ.get("QPB_SANITIZED")), reason="imports torch")
def test_python_binding_imports():
    import qpb
    assert qpb.version().startswith("qpb")


def test_version_macros_match_library():
    """include/qpb.h's QPB_VERSION_MAJOR / _MINOR name the library they ship
    with: qpb_version() reports "qpb MAJOR.MINOR (...)"."""
    src = open(HEADERS[0]).read()
    major = int(re.search(r"#define QPB_VERSION_MAJOR (\d+)", src).group(1))
    minor = int(re.search(r"#define QPB_VERSION_MINOR (\d+)", src).group(1))
    lib = ctypes.CDLL(LIB)
    lib.qpb_version.restype = ctypes.c_char_p
    m = re.match(r"qpb (\d+)\.(\d+) \(", lib.qpb_version().decode())
    assert m, lib.qpb_version()
    assert (int(m.group(1)), int(m.group(2))) == (major, minor)
