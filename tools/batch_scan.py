#!/usr/bin/env python3
"""Kernel time of qpb_solve at n=16, m=32 (box family) against the batch size,
plus the cache diagnostics: where does a launch's time go -- steady-state
throughput, ramp/tail, or HBM?

  T(B) for B = k * 12288 (12288 = 3072 resident waves x 4 QPs: one "round")
  DIAG_MALL: inputs of QP g mod 16384 (Infinity-Cache resident), same compute
HIP-event timing on the launch stream, median of R launches, each waited for
(B{B}_us), and the per-launch time of K launches queued back to back between
two events (B{B}_b2b_us: the GPU never idles between them, as in bench.py's
timed steps -- the chip's clock under a stream of short launches differs from
its clock for one launch after an idle gap)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import bench  # noqa: E402
import qpb  # noqa: E402
from prof_sweep import _diag_args, t_kernel  # noqa: E402


def t_back_to_back(fn, launches=None):
    """ms per launch of K launches queued without a wait between them
    (K sized to ~50 ms of work), median of 3"""
    s = torch.cuda.current_stream()
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    fn()
    b.record(s)
    b.synchronize()
    one = max(a.elapsed_time(b), 1e-3)
    k = launches or max(20, min(2000, int(50.0 / one)))
    ts = []
    for _ in range(3):
        a.record(s)
        for _ in range(k):
            fn()
        b.record(s)
        b.synchronize()
        ts.append(a.elapsed_time(b) / k)
    return sorted(ts)[1]


def main():
    dev = torch.device("cuda", 0)
    fam = os.environ.get("FAM", "box")
    out = {}
    bs = os.environ.get("BS")
    sizes = [int(x) for x in bs.split(",")] if bs else [4096, 8192, 16384, 32768, 65536, 131072, 262144,
                                                         524288, 1048576]
    Bmax = max(sizes + [262144])
    H, f, A, b = qpb.generate(16, Bmax, 1, family=fam, shift=1.0, box=10.0, device=dev)
    for B in sizes:
        h, ff, a, bb = H[:B], f[:B], A[:B], b[:B]
        sol = qpb.solve(h, ff, a, bb)
        ms = t_kernel(lambda: qpb.solve(h, ff, a, bb, out=sol))
        out[f"B{B}_us"] = round(ms * 1e3, 1)
        out[f"B{B}_QPs_per_s"] = B / ms * 1e3
        out[f"B{B}_b2b_us"] = round(t_back_to_back(lambda: qpb.solve(h, ff, a, bb, out=sol)) * 1e3, 1)
    for B in ([] if os.environ.get("NO_MALL") else [65536, 262144]):
        h, ff, a, bb = H[:B], f[:B], A[:B], b[:B]
        sol = qpb.solve(h, ff, a, bb)
        ms = t_kernel(lambda: qpb.lib().qpb_solve(*_diag_args(h, ff, a, bb, sol, 16)))
        out[f"mall_B{B}_us"] = round(ms * 1e3, 1)
    # the revision of the kernel scanned (bench.py's shard-time prediction reads it)
    out["revision"] = sorted(r for r in bench.kernel_revisions(qpb.version()) if r.startswith("gi_dense"))[0]
    big = sorted(B for B in sizes if B >= 131072)
    if len(big) >= 2:
        # T(B) = a + c B over the large batches: a = the per-launch fixed cost
        import numpy as np
        t = np.array([out[f"B{B}_us"] for B in big])
        c, a = np.polyfit(np.array(big, dtype=float), t, 1)
        out["fit_intercept_us"], out["fit_ns_per_qp"] = float(a), float(c * 1e3)
    if "B131072_us" in out and "B1048576_us" in out:
        out["T1M_over_T131072"] = out["B1048576_us"] / out["B131072_us"]
        out["T1M_over_T131072_b2b"] = out["B1048576_b2b_us"] / out["B131072_b2b_us"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
