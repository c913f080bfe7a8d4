#!/usr/bin/env python3
"""Kernel time of qpb_solve at n=16, m=32 (box family) against the batch size,
plus the cache diagnostics: where does a launch's time go -- steady-state
throughput, ramp/tail, or HBM?

  T(B) for B = k * 12288 (12288 = 3072 resident waves x 4 QPs: one "round")
  DIAG_MALL: inputs of QP g mod 16384 (Infinity-Cache resident), same compute
HIP-event timing on the launch stream, median of R launches."""
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


def main():
    dev = torch.device("cuda", 0)
    fam = os.environ.get("FAM", "box")
    out = {}
    bs = os.environ.get("BS")
    sizes = [int(x) for x in bs.split(",")] if bs else [4096, 12288, 24576, 36864, 49152, 61440, 65536, 73728,
                                                         98304, 131072, 196608, 262144]
    Bmax = max(sizes + [262144])
    H, f, A, b = qpb.generate(16, Bmax, 1, family=fam, shift=1.0, box=10.0, device=dev)
    for B in sizes:
        h, ff, a, bb = H[:B], f[:B], A[:B], b[:B]
        sol = qpb.solve(h, ff, a, bb)
        ms = t_kernel(lambda: qpb.solve(h, ff, a, bb, out=sol))
        out[f"B{B}_us"] = round(ms * 1e3, 1)
        out[f"B{B}_QPs_per_s"] = B / ms * 1e3
    for B in ([] if os.environ.get("NO_MALL") else [65536, 262144]):
        h, ff, a, bb = H[:B], f[:B], A[:B], b[:B]
        sol = qpb.solve(h, ff, a, bb)
        ms = t_kernel(lambda: qpb.lib().qpb_solve(*_diag_args(h, ff, a, bb, sol, 16)))
        out[f"mall_B{B}_us"] = round(ms * 1e3, 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
