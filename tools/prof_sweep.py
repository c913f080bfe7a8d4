#!/usr/bin/env python3
"""Kernel-time breakdown of qpb_solve at n=16, m=32 (B=65,536) by ablation:
setup only (m=0), then max_iter = 1, 2, 4, 8, default; box and dense families.
HIP-event timing on the launch stream, median of R launches."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import qpb  # noqa: E402


def settle(fn, seconds=0.05):
    """fn back to back for about `seconds` (groups of 5, a sync between): the
    GPU's clocks ramp for its first launches after idle"""
    import time
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(5):
            fn()
        torch.cuda.synchronize()


def t_kernel(fn, reps=15):
    s = torch.cuda.current_stream()
    settle(fn)
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        fn()
        b.record(s)
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def _diag_args(H, f, A, b, sol, flags=1):
    import ctypes
    B, n = f.shape
    d = qpb.Desc(n, A.shape[1], B, 0, flags, 0.0)  # 1 = QPB_FLAG_DIAG_L2, 16 = QPB_FLAG_DIAG_MALL
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    return (ctypes.byref(d), p(H), p(f), p(A), p(b), p(sol.x), p(sol.lam), p(sol.active), p(sol.status),
            p(sol.iters), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))


def main():
    dev = torch.device("cuda", 0)
    B = int(os.environ.get("B", 65536))
    out = {}
    for fam in ("box", "dense"):
        H, f, A, b = bench.make_batch(torch, B, 16, fam, 1, dev)
        sol = qpb.solve(H, f, A, b)
        torch.cuda.synchronize()
        out[f"{fam}_iters_mean"] = float(sol.iters.double().mean())
        out[f"{fam}_m0_setup_ms"] = t_kernel(lambda: qpb.solve(H, f))
        sol2 = qpb.solve(H, f, A, b)
        out[f"{fam}_l2diag_ms"] = t_kernel(lambda: qpb.lib().qpb_solve(*_diag_args(H, f, A, b, sol2)))
        out[f"{fam}_occ2_ms"] = t_kernel(lambda: qpb.lib().qpb_solve(*_diag_args(H, f, A, b, sol2, 4)))
        out[f"{fam}_occ2_l2diag_ms"] = t_kernel(lambda: qpb.lib().qpb_solve(*_diag_args(H, f, A, b, sol2, 5)))
        out[f"{fam}_persist_ms"] = t_kernel(lambda: qpb.lib().qpb_solve(*_diag_args(H, f, A, b, sol2, 8)))
        torch.cuda.synchronize()
        out[f"{fam}_persist_match"] = bool(torch.equal(sol2.x, sol.x) and torch.equal(sol2.active, sol.active))
        its = sol.iters.view(-1, 4).max(dim=1).values.double()
        out[f"{fam}_wave_trips_mean"] = float(its.mean())
        for mi in (1, 2, 4, 8, 0):
            out[f"{fam}_maxit{mi or 'def'}_ms"] = t_kernel(lambda: qpb.solve(H, f, A, b, max_iter=mi, out=sol))
    # batch scaling (box)
    for Bs in (4096, 16384, 65536, 262144):
        H, f, A, b = bench.make_batch(torch, Bs, 16, "box", 2, dev)
        sol = qpb.solve(H, f, A, b)
        ms = t_kernel(lambda: qpb.solve(H, f, A, b, out=sol))
        out[f"box_B{Bs}_ms"] = ms
        out[f"box_B{Bs}_GBs"] = Bs * bench.bytes_per_qp(16, 32) / ms / 1e6
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
