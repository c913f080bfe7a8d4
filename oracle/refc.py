"""oracle/refc.py -- TEST INFRASTRUCTURE ONLY.

ctypes wrapper around oracle/_ref/libqpref_n<N>_<box>.so: the unmodified
reference C sources (matrix_ops.c, qp.c, qp_solvers.c, kmalloc.c, klist.c)
compiled by oracle/Makefile together with oracle/ref_driver.c.  Used to make
golden fixtures (tests/golden/make_golden.py) and as bench.py's CPU baseline
("kind": "reference").  Each .so holds static pools and the global rand()
state of the reference (kmalloc.c:37-42), so it is single-threaded; the
bench forks one process per core.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(HERE, "_ref")

_dp = ctypes.POINTER(ctypes.c_double)


def lib_path(n: int, box: str = "1e12") -> str:
    return os.path.join(REF_DIR, f"libqpref_n{n}_{box}.so")


def available(n: int, box: str = "1e12") -> bool:
    return os.path.exists(lib_path(n, box))


class RefC:
    def __init__(self, n: int, box: str = "1e12"):
        path = lib_path(n, box)
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle ref` where /root/reference exists")
        # RTLD_LOCAL + a private copy per (n, box): every variant keeps its own static pools
        self.lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        L = self.lib
        L.ref_ndim.restype = ctypes.c_uint
        L.ref_box_max.restype = ctypes.c_double
        L.ref_box_min.restype = ctypes.c_double
        L.ref_eval.restype = ctypes.c_double
        L.ref_eval.argtypes = [_dp, _dp, ctypes.c_double, _dp]
        self.n = int(L.ref_ndim())
        assert self.n == n
        self.box_max = L.ref_box_max()
        self.box_min = L.ref_box_min()

    @staticmethod
    def _p(a: np.ndarray):
        return a.ctypes.data_as(_dp)

    def generate(self, seed: int, count: int, prange=(-1e3, 1e3), qrange=(-1e3, 1e3), xrange=(-1e3, 1e3)):
        n = self.n
        P = np.zeros((count, n, n))
        q = np.zeros((count, n))
        x0 = np.zeros((count, n))
        self.lib.ref_srand(ctypes.c_uint(seed))
        self.lib.ref_gen_qps(ctypes.c_uint(count), *[ctypes.c_double(v) for v in (*prange, *qrange, *xrange)],
                             self._p(P), self._p(q), self._p(x0))
        return P, q, x0

    def _batch(self, fn, P, q, x0, iters):
        P = np.ascontiguousarray(P, dtype=np.float64)
        q = np.ascontiguousarray(q, dtype=np.float64)
        x0 = np.ascontiguousarray(x0, dtype=np.float64)
        x = np.zeros_like(q)
        fn(ctypes.c_uint(len(q)), self._p(P), self._p(q), self._p(x0), ctypes.c_uint(int(iters)), self._p(x))
        return x

    def newton(self, P, q, x0, iters=10):
        return self._batch(self.lib.ref_newton_batch, P, q, x0, iters)

    def admm(self, P, q, x0, iters=10000):
        return self._batch(self.lib.ref_admm_batch, P, q, x0, iters)

    def gd(self, P, q, x0, iters=10000):
        return self._batch(self.lib.ref_gd_batch, P, q, x0, iters)

    def invert(self, M):
        M = np.array(M, dtype=np.float64, order="C")
        self.lib.ref_invert(self._p(M))
        return M

    def eval(self, P, q, r, x):
        P = np.ascontiguousarray(P, dtype=np.float64)
        q = np.ascontiguousarray(q, dtype=np.float64)
        x = np.ascontiguousarray(x, dtype=np.float64)
        return self.lib.ref_eval(self._p(P), self._p(q), ctypes.c_double(r), self._p(x))
