"""qpb -- Python host binding of the batched MI355X QP solver (include/qpb.h).

Thin ctypes layer over ``lib/libqpb.so`` (built by ``make -C
embedded-qp-solver_amd``).  Device memory and streams are PyTorch-ROCm tensors
and streams; every solve runs in the HIP kernels of the library.  There is no
CPU fallback: importing this module fails loudly when the library is missing,
and solving fails when no HIP device is present.

The reference's single-QP C API (qp.h / qp_solvers.h) is the C
compat layer in include/compat/; this module mirrors the batched C-ABI:

    solve(H, f, A, b)          -> qpb_solve       (active set, m > 0)
    solve(H, f)                -> qpb_solve, m=0  (test/qp_ref.py:35 semantics)
    ref_solve(mode, P, q, x0)  -> qpb_ref_solve   (qp_solvers.c replicas)
    qf_eval(P, q, r, x)        -> qpb_qf_eval     (qp.c:9-27)
    ref_generate(n, B, seed)   -> qpb_ref_generate (the reference generator, bit for bit)
    generate(n, B, seed)       -> qpb_generate     (Philox benchmark families)
"""
from __future__ import annotations

import ctypes
import os
from typing import NamedTuple

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
LIB_PATH = os.environ.get("QPB_LIB", os.path.join(PKG_ROOT, "lib", "libqpb.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(f"qpb: {LIB_PATH} not found -- build it with `make -C {PKG_ROOT}` "
                      "(there is no CPU fallback)")

_lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)

# status codes (qpb_status)
OK, MAX_ITER, NOT_SPD, INFEASIBLE, NUMERICAL = 0, 1, 2, 3, 4
STATUS_NAMES = {OK: "OK", MAX_ITER: "MAX_ITER", NOT_SPD: "NOT_SPD", INFEASIBLE: "INFEASIBLE", NUMERICAL: "NUMERICAL"}
# error codes (qpb_error)
ERR_INVALID_ARG, ERR_UNSUPPORTED, ERR_HIP, ERR_NO_DEVICE = -1, -2, -3, -4
# reference modes (qpb_ref_mode)
REF_NEWTON, REF_ADMM, REF_GD = 1, 2, 3
MAX_N, MAX_M = 128, 256
REF_MAX_N = 1024  # qpb_ref_solve / qpb_matrix_invert (QPB_REF_MAX_N)
# qpb_desc.flags (include/qpb.h)
FLAG_DIAG_L2, FLAG_DIAG_MALL = 1, 16
FLAG_MIXED, FLAG_DIAG_NO_REDO = 32, 64
FLAG_DIAG_WAVE = 256  # n <= 16 solved by the one-QP-per-wavefront kernel (lockstep endpoint; measurement only)
STATUS_REDO = 100  # internal: a QP the mixed kernel leaves to the fp64 re-solve (FLAG_DIAG_NO_REDO only)


class Desc(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("m", ctypes.c_int32), ("batch", ctypes.c_int64),
                ("max_iter", ctypes.c_int32), ("flags", ctypes.c_int32), ("feas_tol", ctypes.c_double)]


class RefDesc(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("mode", ctypes.c_int32), ("batch", ctypes.c_int64),
                ("iterations", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("box_min", ctypes.c_double), ("box_max", ctypes.c_double)]


_vp = ctypes.c_void_p
_lib.qpb_solve.argtypes = [ctypes.POINTER(Desc)] + [_vp] * 10
_lib.qpb_solve.restype = ctypes.c_int
_lib.qpb_solve_host.argtypes = [ctypes.POINTER(Desc)] + [_vp] * 9
_lib.qpb_solve_host.restype = ctypes.c_int
_lib.qpb_solve_box.argtypes = [ctypes.POINTER(Desc)] + [_vp] * 10
_lib.qpb_solve_box.restype = ctypes.c_int
_lib.qpb_ref_solve.argtypes = [ctypes.POINTER(RefDesc)] + [_vp] * 6
_lib.qpb_ref_solve.restype = ctypes.c_int
_lib.qpb_ref_solve_host.argtypes = [ctypes.POINTER(RefDesc)] + [_vp] * 5
_lib.qpb_ref_solve_host.restype = ctypes.c_int
_lib.qpb_qf_eval.argtypes = [ctypes.c_int32, ctypes.c_int64, _vp, _vp, ctypes.c_double, _vp, _vp, _vp]
_lib.qpb_qf_eval.restype = ctypes.c_int
_lib.qpb_matrix_invert.argtypes = [ctypes.c_int32, ctypes.c_int64, _vp, _vp, _vp]
_lib.qpb_matrix_invert.restype = ctypes.c_int
_lib.qpb_last_error.restype = ctypes.c_char_p
_lib.qpb_version.restype = ctypes.c_char_p
_lib.qpb_device_count.restype = ctypes.c_int
_lib.qpb_set_device.argtypes = [ctypes.c_int]
_lib.qpb_synchronize.argtypes = [_vp]


class QPBError(RuntimeError):
    def __init__(self, code: int, where: str):
        msg = _lib.qpb_last_error().decode(errors="replace")
        super().__init__(f"{where} failed with {code}: {msg}")
        self.code = code


def _check(rc: int, where: str) -> None:
    if rc != 0:
        raise QPBError(rc, where)


def lib() -> ctypes.CDLL:
    return _lib


def version() -> str:
    return _lib.qpb_version().decode()


def device_count() -> int:
    return int(_lib.qpb_device_count())


class Solution(NamedTuple):
    x: object       # (B, n) float64
    lam: object     # (B, m) float64
    active: object  # (B, ceil(m/32)) int32 (uint32 bit pattern)
    status: object  # (B,) int32
    iters: object   # (B,) int32


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None and t.numel() > 0 else ctypes.c_void_p(0)


def _stream_ptr(stream):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def solve(H, f, A=None, b=None, *, max_iter: int = 0, feas_tol: float = 0.0, out: Solution | None = None,
          stream=None, flags: int = 0) -> Solution:
    """Batched min 1/2 x^T H x + f^T x s.t. A x <= b on the GPU (torch CUDA float64 tensors).

    H (B,n,n), f (B,n), A (B,m,n), b (B,m).  Asynchronous on ``stream``
    (default: torch's current stream; the n > 32 class caches a scratch buffer per
    stream: call ``release_stream_workspace(stream)`` before destroying a stream
    passed here).  A/b omitted -> unconstrained solve.
    ``flags``: QPB_FLAG_DIAG_* kernel variants (measurement only, qpb.h).
    """
    import torch
    if not (H.is_cuda and f.is_cuda):
        raise ValueError("qpb.solve expects CUDA (HIP) tensors; use solve_host for numpy")
    B, n = f.shape
    m = 0 if A is None else A.shape[1]
    for t in (H, f) + ((A, b) if m else ()):
        if t.dtype != torch.float64 or not t.is_contiguous():
            raise ValueError("inputs must be contiguous float64")
    if H.shape != (B, n, n) or (m and (A.shape != (B, m, n) or b.shape != (B, m))):
        raise ValueError("shape mismatch")
    dev = f.device
    w = (m + 31) // 32
    if out is None:
        out = Solution(torch.empty((B, n), dtype=torch.float64, device=dev),
                       torch.empty((B, m), dtype=torch.float64, device=dev),
                       torch.empty((B, w), dtype=torch.int32, device=dev),
                       torch.empty((B,), dtype=torch.int32, device=dev),
                       torch.empty((B,), dtype=torch.int32, device=dev))
    d = Desc(n, m, B, max_iter, flags, feas_tol)
    rc = _lib.qpb_solve(ctypes.byref(d), _ptr(H), _ptr(f), _ptr(A) if m else None, _ptr(b) if m else None,
                        _ptr(out.x), _ptr(out.lam), _ptr(out.active), _ptr(out.status), _ptr(out.iters),
                        _stream_ptr(stream))
    _check(rc, "qpb_solve")
    return out


def solve_box(H, f, lb=None, ub=None, *, max_iter: int = 0, feas_tol: float = 0.0, out: Solution | None = None,
              stream=None) -> Solution:
    """Batched min 1/2 x^T H x + f^T x s.t. lb <= x <= ub on the GPU (qpb_solve_box,
    n <= 128): the reference admm()'s box QP (qp_solvers.c:146-319), solved exactly.

    H (B,n,n), f (B,n), lb / ub (B,n) CUDA float64 tensors or None (absent
    bounds; +-inf entries likewise).  The Solution has m = 2n: lam[:, :n] and
    active bits 0..n-1 belong to the upper bounds, lam[:, n:] and bits n..2n-1
    to the lower bounds (the row order of A = [I; -I], b = [ub; -lb]).
    """
    import torch
    if not (H.is_cuda and f.is_cuda):
        raise ValueError("qpb.solve_box expects CUDA (HIP) tensors")
    B, n = f.shape
    for t in (H, f, lb, ub):
        if t is not None and (t.dtype != torch.float64 or not t.is_contiguous()):
            raise ValueError("inputs must be contiguous float64")
        if t is not None and t.device != f.device:
            raise ValueError("H, f, lb and ub must live on the same CUDA device")
    if H.shape != (B, n, n) or any(t is not None and t.shape != (B, n) for t in (lb, ub)):
        raise ValueError("shape mismatch")
    dev = f.device
    m = 2 * n
    if out is None:
        out = Solution(torch.empty((B, n), dtype=torch.float64, device=dev),
                       torch.empty((B, m), dtype=torch.float64, device=dev),
                       torch.empty((B, (m + 31) // 32), dtype=torch.int32, device=dev),
                       torch.empty((B,), dtype=torch.int32, device=dev),
                       torch.empty((B,), dtype=torch.int32, device=dev))
    d = Desc(n, m, B, max_iter, 0, feas_tol)
    rc = _lib.qpb_solve_box(ctypes.byref(d), _ptr(H), _ptr(f), _ptr(lb), _ptr(ub), _ptr(out.x), _ptr(out.lam),
                            _ptr(out.active), _ptr(out.status), _ptr(out.iters), _stream_ptr(stream))
    _check(rc, "qpb_solve_box")
    return out


def solve_raw(desc: Desc, ptrs, stream_ptr) -> int:
    """Direct C-ABI call with raw device pointers (H, f, A, b, x, lam, active, status, iters)."""
    return _lib.qpb_solve(ctypes.byref(desc), *[ctypes.c_void_p(p) for p in ptrs], ctypes.c_void_p(stream_ptr))


def solve_host(H, f, A=None, b=None, *, max_iter: int = 0, feas_tol: float = 0.0) -> Solution:
    """numpy in / numpy out (qpb_solve_host: H2D, solve, D2H)."""
    import numpy as np
    H = np.ascontiguousarray(H, dtype=np.float64)
    f = np.ascontiguousarray(f, dtype=np.float64)
    B, n = f.shape
    m = 0 if A is None else A.shape[1]
    if m:
        A = np.ascontiguousarray(A, dtype=np.float64)
        b = np.ascontiguousarray(b, dtype=np.float64)
    w = (m + 31) // 32
    x = np.zeros((B, n))
    lam = np.zeros((B, m))
    act = np.zeros((B, w), dtype=np.uint32)
    st = np.zeros(B, dtype=np.int32)
    it = np.zeros(B, dtype=np.int32)
    d = Desc(n, m, B, max_iter, 0, feas_tol)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p) if a is not None and a.size else None  # noqa: E731
    rc = _lib.qpb_solve_host(ctypes.byref(d), p(H), p(f), p(A), p(b), p(x), p(lam), p(act), p(st), p(it))
    _check(rc, "qpb_solve_host")
    return Solution(x, lam, act, st, it)


def active_mask_to_bool(active, m: int):
    """(B, words) uint32/int32 bit words -> (B, m) bool (numpy)."""
    import numpy as np
    a = np.asarray(active).astype(np.uint32)
    bits = ((a[:, :, None] >> np.arange(32, dtype=np.uint32)) & 1).astype(bool)
    return bits.reshape(a.shape[0], -1)[:, :m]


def _require_f64_cuda(name: str, t, shape: tuple):
    """A contiguous float64 CUDA tensor of exactly `shape`: the C-ABI reads
    the pointer as device memory of that layout, so a CPU tensor, another
    dtype or a strided view must be refused here, not dereferenced there."""
    import torch
    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float64 and t.is_contiguous()
            and tuple(t.shape) == tuple(shape)):
        got = (tuple(t.shape), str(t.dtype), str(t.device), t.is_contiguous()) if isinstance(t, torch.Tensor) \
            else type(t).__name__
        raise ValueError(f"{name}: expected a contiguous float64 CUDA tensor of shape {tuple(shape)}, got {got}")


def ref_solve(mode: int, P, q, x0=None, *, iterations: int, box=(-1e12, 1e12), stream=None):
    """Reference-semantics batched solvers (qp_solvers.c replicas) on CUDA tensors:
    P (B, n, n), q (B, n), x0 (B, n) or None: zeros for GD and Newton, unused
    by ADMM (qp_solvers.c:256 ignores its x0)."""
    import torch
    if not (isinstance(q, torch.Tensor) and q.dim() == 2):
        raise ValueError("qpb.ref_solve: q must be a (B, n) tensor")
    B, n = q.shape
    _require_f64_cuda("qpb.ref_solve: q", q, (B, n))
    _require_f64_cuda("qpb.ref_solve: P", P, (B, n, n))
    if x0 is not None:
        _require_f64_cuda("qpb.ref_solve: x0", x0, (B, n))
        if x0.device != q.device or P.device != q.device:
            raise ValueError("qpb.ref_solve: P, q and x0 must be on one device")
    elif P.device != q.device:
        raise ValueError("qpb.ref_solve: P and q must be on one device")
    elif mode != REF_ADMM:
        # GD and Newton start from x0 (qpb_ref_solve requires it); ADMM ignores
        # it, as the reference does (qp_solvers.c:256)
        x0 = torch.zeros_like(q)
    x = torch.empty((B, n), dtype=torch.float64, device=q.device)
    it = torch.empty((B,), dtype=torch.int32, device=q.device)
    d = RefDesc(n, mode, B, iterations, 0, float(box[0]), float(box[1]))
    rc = _lib.qpb_ref_solve(ctypes.byref(d), _ptr(P), _ptr(q), _ptr(x0) if x0 is not None else None,
                            _ptr(x), _ptr(it), _stream_ptr(stream))
    _check(rc, "qpb_ref_solve")
    return x, it


_lib.qpb_release_stream_workspace.argtypes = [_vp]
_lib.qpb_release_stream_workspace.restype = ctypes.c_int
_lib.qpb_release_workspaces.argtypes = []
_lib.qpb_release_workspaces.restype = ctypes.c_int


def release_stream_workspace(stream=None) -> None:
    """qpb_release_stream_workspace: free the scratch buffer cached for
    `stream` (a torch.cuda.Stream or ExternalStream; None = the current
    stream).  The n <= 128 kernels and the reference replicas above n = 64
    cache one buffer per (device, stream) and free it stream-ordered on that
    stream, so call this before destroying a stream passed as ``stream=``."""
    _check(_lib.qpb_release_stream_workspace(_stream_ptr(stream)), "qpb_release_stream_workspace")


def release_workspaces() -> None:
    """qpb_release_workspaces: synchronise every cached stream and free all the scratch buffers."""
    _check(_lib.qpb_release_workspaces(), "qpb_release_workspaces")


def matrix_invert(P, stream=None):
    """Batched reference matrix_invert (matrix_ops.c:551-630) of (B, n, n) CUDA tensors."""
    import torch
    if not (P.is_cuda and P.dtype == torch.float64 and P.is_contiguous() and P.dim() == 3
            and P.shape[1] == P.shape[2]):
        raise ValueError("qpb.matrix_invert expects a contiguous float64 CUDA tensor of shape (B, n, n)")
    B, n, _ = P.shape
    out = torch.empty_like(P)
    _check(_lib.qpb_matrix_invert(n, B, _ptr(P), _ptr(out), _stream_ptr(stream)), "qpb_matrix_invert")
    return out


def qf_eval(P, q, r: float, x, stream=None):
    """Batched quadratic_form_eval (qp.c:9-27): 1/2 x'Px + q'x + r per QP;
    P (B, n, n), q (B, n), x (B, n) float64 CUDA tensors."""
    import torch
    if not (isinstance(q, torch.Tensor) and q.dim() == 2):
        raise ValueError("qpb.qf_eval: q must be a (B, n) tensor")
    B, n = q.shape
    _require_f64_cuda("qpb.qf_eval: q", q, (B, n))
    _require_f64_cuda("qpb.qf_eval: P", P, (B, n, n))
    _require_f64_cuda("qpb.qf_eval: x", x, (B, n))
    if not (P.device == q.device == x.device):
        raise ValueError("qpb.qf_eval: P, q and x must be on one device")
    out = torch.empty((B,), dtype=torch.float64, device=q.device)
    rc = _lib.qpb_qf_eval(n, B, _ptr(P), _ptr(q), float(r), _ptr(x), _ptr(out), _stream_ptr(stream))
    _check(rc, "qpb_qf_eval")
    return out


_lib.qpb_solve_sections.argtypes = [ctypes.POINTER(Desc)] + [_vp] * 10 + [ctypes.c_int64, _vp]
_lib.qpb_solve_sections.restype = ctypes.c_int
SECTION_NAMES = ["load", "cholesky", "substitution", "init", "select", "exchange", "back_solve", "step",
                 "add", "drop", "loop_exit", "output"]
N_SECTIONS = 20  # kSections (csrc/qpb_common.h): every stamped kernel adds all of them into the buffer
SECTION_SLOTS = 256  # kSectionSlots: rows of the device buffer (one per blockIdx mod 256)
WAVE_SECTION_NAMES = ["load", "sweep", "init", "select", "exchange", "back_solve", "step", "add", "drop",
                      "loop_exit", "x", "stores"]


def solve_sections(H, f, A, b, sections, *, max_iter: int = 0, out: Solution | None = None, stream=None):
    """Diagnostic builds of the n=16 (16<m<=32) and 16<n<=32 (m<=64) kernels:
    accumulate per-section wave ticks (100 MHz) into the int64 CUDA tensor
    ``sections`` (N_SECTIONS = 20 int64 entries; the first 12 are named by
    SECTION_NAMES / WAVE_SECTION_NAMES)."""
    import torch
    if not (sections.is_cuda and sections.dtype == torch.int64 and sections.is_contiguous()
            and sections.numel() >= N_SECTIONS):
        raise ValueError(f"sections must be a contiguous int64 CUDA tensor of >= {N_SECTIONS} entries")
    B, n = f.shape
    m = A.shape[1]
    if out is None:
        out = solve(H, f, A, b, max_iter=max_iter, stream=stream)
    d = Desc(n, m, B, max_iter, 0, 0.0)
    rows = torch.zeros((SECTION_SLOTS, N_SECTIONS), dtype=torch.int64, device=sections.device)
    rc = _lib.qpb_solve_sections(ctypes.byref(d), _ptr(H), _ptr(f), _ptr(A), _ptr(b), _ptr(out.x), _ptr(out.lam),
                                 _ptr(out.active), _ptr(out.status), _ptr(out.iters), _ptr(rows), rows.numel(),
                                 _stream_ptr(stream))
    _check(rc, "qpb_solve_sections")
    sections[:N_SECTIONS] += rows.sum(0)
    return out


# ------------------------------------------------------------------ generators
class RefGenDesc(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("seed", ctypes.c_uint32), ("batch", ctypes.c_int64),
                ("first", ctypes.c_uint64), ("p_min", ctypes.c_double), ("p_max", ctypes.c_double),
                ("q_min", ctypes.c_double), ("q_max", ctypes.c_double),
                ("x_min", ctypes.c_double), ("x_max", ctypes.c_double)]


class GenDesc(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("m", ctypes.c_int32), ("batch", ctypes.c_int64),
                ("first", ctypes.c_uint64), ("seed", ctypes.c_uint64), ("family", ctypes.c_int32),
                ("flags", ctypes.c_int32), ("shift", ctypes.c_double), ("box", ctypes.c_double)]


FAMILY_BOX, FAMILY_DENSE = 0, 1
FAMILIES = {"box": FAMILY_BOX, "dense": FAMILY_DENSE}
_lib.qpb_ref_generate.argtypes = [ctypes.POINTER(RefGenDesc), _vp, _vp, _vp, _vp]
_lib.qpb_ref_generate.restype = ctypes.c_int
_lib.qpb_generate.argtypes = [ctypes.POINTER(GenDesc), _vp, _vp, _vp, _vp, _vp]
_lib.qpb_generate.restype = ctypes.c_int


def ref_generate(n: int, batch: int, seed: int, *, first: int = 0, p_range=(-1e3, 1e3), q_range=(-1e3, 1e3),
                 x_range=(-1e3, 1e3), device=None, stream=None):
    """The reference generator (srand(seed); main.c:37-39 order) on the GPU,
    QPs [first, first + batch): (P (B,n,n), q (B,n), x0 (B,n)) CUDA tensors."""
    import torch
    dev = device or torch.device("cuda", torch.cuda.current_device())
    P = torch.empty((batch, n, n), dtype=torch.float64, device=dev)
    q = torch.empty((batch, n), dtype=torch.float64, device=dev)
    x0 = torch.empty((batch, n), dtype=torch.float64, device=dev)
    d = RefGenDesc(n, seed & 0xFFFFFFFF, batch, first, *p_range, *q_range, *x_range)
    _check(_lib.qpb_ref_generate(ctypes.byref(d), _ptr(P), _ptr(q), _ptr(x0), _stream_ptr(stream)),
           "qpb_ref_generate")
    return P, q, x0


def generate(n: int, batch: int, seed: int, *, family: str = "box", m: int | None = None, first: int = 0,
             shift: float = 1.0, box: float = 10.0, device=None, stream=None):
    """Benchmark-family QPs from the counter-based generator (qpb_generate):
    (H, f, A, b) CUDA tensors; QP first + k is the same for any launch."""
    import torch
    dev = device or torch.device("cuda", torch.cuda.current_device())
    m = 2 * n if m is None else m
    H = torch.empty((batch, n, n), dtype=torch.float64, device=dev)
    f = torch.empty((batch, n), dtype=torch.float64, device=dev)
    A = torch.empty((batch, m, n), dtype=torch.float64, device=dev)
    b = torch.empty((batch, m), dtype=torch.float64, device=dev)
    d = GenDesc(n, m, batch, first, seed, FAMILIES[family], 0, shift, box)
    _check(_lib.qpb_generate(ctypes.byref(d), _ptr(H), _ptr(f), _ptr(A), _ptr(b), _stream_ptr(stream)),
           "qpb_generate")
    return H, f, A, b


# ------------------------------------------------------------------ wire format
_lib.qpb_wire_write.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64] + [_vp] * 4
_lib.qpb_wire_write.restype = ctypes.c_int
_lib.qpb_wire_read_header.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int32),
                                      ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64)]
_lib.qpb_wire_read_header.restype = ctypes.c_int
_lib.qpb_wire_read.argtypes = [ctypes.c_char_p] + [_vp] * 4
_lib.qpb_wire_read.restype = ctypes.c_int


def wire_write(path: str, H, f, A=None, b=None) -> None:
    """numpy (B,n,n), (B,n)[, (B,m,n), (B,m)] -> wire file (qpb_wire_write);
    a single unconstrained QP is written in the reference's own format."""
    import numpy as np
    H = np.ascontiguousarray(H, dtype=np.float64)
    f = np.ascontiguousarray(f, dtype=np.float64)
    B, n = f.shape
    m = 0 if A is None else A.shape[1]
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p) if a is not None else None  # noqa: E731
    if m:
        A = np.ascontiguousarray(A, dtype=np.float64)
        b = np.ascontiguousarray(b, dtype=np.float64)
    _check(_lib.qpb_wire_write(os.fsencode(path), n, m, B, p(H), p(f), p(A), p(b)), "qpb_wire_write")


def wire_read(path: str):
    """wire file -> numpy (H, f, A, b) (A, b have m = 0 columns for an unconstrained file)."""
    import numpy as np
    n, m, B = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
    _check(_lib.qpb_wire_read_header(os.fsencode(path), ctypes.byref(n), ctypes.byref(m), ctypes.byref(B)),
           "qpb_wire_read_header")
    n, m, B = n.value, m.value, B.value
    H, f = np.empty((B, n, n)), np.empty((B, n))
    A, b = np.empty((B, m, n)), np.empty((B, m))
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p) if a.size else None  # noqa: E731
    _check(_lib.qpb_wire_read(os.fsencode(path), p(H), p(f), p(A), p(b)), "qpb_wire_read")
    return H, f, A, b
