"""The host code of libqpb.so under AddressSanitizer + UndefinedBehaviorSanitizer.

`make asan` (embedded-qp-solver_amd/Makefile) builds the whole library with
every host instruction instrumented: the C-ABI's validation and dispatch in the
.hip files (-Xarch_host; the device code is the normal build's), compat.c and
qpb_wire.c.  This test runs tests/test_compat.py, test_wire.py and test_abi.py
against that build in a child process with the sanitizer runtime preloaded
(halt on the first report), and first checks that the harness is live: an
access one element past a pool matrix through matrix_get_entry must be reported
as a heap-buffer-overflow.  CPU only; the sanitized library never runs a
kernel."""
import glob
import os
import subprocess
import sys

import pytest

from conftest import ROOT

PKG = os.path.join(ROOT, "embedded-qp-solver_amd")
ASAN_LIB = os.path.join(PKG, "build", "asan", "libqpb.so")
RUNTIME = sorted(glob.glob("/opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))

CANARY = r"""
import ctypes, os
L = ctypes.CDLL(os.environ["QPB_LIB"])
class M(ctypes.Structure):
    _fields_ = [("dimensions", ctypes.c_uint), ("elements", ctypes.POINTER(ctypes.c_double))]
class E(ctypes.Structure):
    _fields_ = [("row", ctypes.c_uint), ("col", ctypes.c_uint)]
L.qpb_compat_init.argtypes = [ctypes.c_uint, ctypes.c_double, ctypes.c_double]
L.matrix_alloc.restype = ctypes.POINTER(M)
L.matrix_get_entry.argtypes = [ctypes.POINTER(M), E]
L.matrix_get_entry.restype = ctypes.c_double
L.qpb_compat_init(4, -1.0, 1.0)
m = L.matrix_alloc(0)
print(L.matrix_get_entry(m, E(3, 3)), flush=True)
print(L.matrix_get_entry(m, E(4, 0)))   # one past the 4 x 4 elements
"""


def _env():
    env = dict(os.environ)
    env.update(QPB_LIB=ASAN_LIB, QPB_SANITIZED="1", LD_PRELOAD=RUNTIME[-1],
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    return env


@pytest.fixture(scope="module")
def asan_build():
    if not RUNTIME or not os.path.exists("/opt/rocm/llvm/bin/clang"):
        pytest.skip("no clang sanitizer runtime in this image")
    r = subprocess.run(["make", "-s", "-j8", "-C", PKG, "ARCH=gfx950", "asan"], capture_output=True, text=True,
                       timeout=1800)
    assert r.returncode == 0, r.stderr[-4000:]
    assert os.path.exists(ASAN_LIB)
    return ASAN_LIB


def test_sanitizer_harness_is_live(asan_build):
    r = subprocess.run([sys.executable, "-c", CANARY], env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "AddressSanitizer: heap-buffer-overflow" in r.stderr
    assert "matrix_get_entry" in r.stderr
    assert r.stdout.splitlines()[0] == "0.0"  # the in-bounds read before it ran clean


def test_host_suites_clean_under_asan_ubsan(asan_build):
    tests = [os.path.join(ROOT, "tests", f) for f in ("test_compat.py", "test_wire.py", "test_abi.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", "-m", "not gpu", *tests],
                       env=_env(), cwd=ROOT, capture_output=True, text=True, timeout=1200)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error:" not in out, out[-6000:]
    assert r.returncode == 0, out[-6000:]
    assert " passed" in r.stdout
