#!/usr/bin/env python3
"""Tail-trimmed n<=16 solve (two launches: K trips for every QP, then the
unfinished ones from scratch) against the single launch (QPB_FLAG_NO_TAIL_TRIM)
on the bench's box and dense families: per-batch kernel time, interleaved A/B
medians, and the outputs compared bit for bit."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
import torch  # noqa: E402

import qpb  # noqa: E402

NO_TRIM = 256
dev = torch.device("cuda", 0)
sizes = [int(v) for v in os.environ.get("SIZES", "16384,65536,131072,262144,524288,1048576").split(",")]
s = torch.cuda.current_stream()
p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
out = {}
for fam in ("box", "dense"):
    H, f, A, b = qpb.generate(16, sizes[-1], 1, family=fam, shift=1.0, box=10.0, device=dev)
    m = A.shape[1]
    for B in sizes:
        sols = {}
        times = {0: [], NO_TRIM: []}
        descs = {fl: qpb.Desc(16, m, B, 0, fl, 0.0) for fl in times}
        for fl in times:
            sols[fl] = qpb.solve(H[:B], f[:B], A[:B], b[:B])

        def call(fl):
            sol = sols[fl]
            rc = qpb.lib().qpb_solve(ctypes.byref(descs[fl]), p(H), p(f), p(A), p(b), p(sol.x), p(sol.lam),
                                     p(sol.active), p(sol.status), p(sol.iters), ctypes.c_void_p(s.cuda_stream))
            assert rc == 0, rc
        for fl in times:
            call(fl)
        torch.cuda.synchronize()
        same = all(torch.equal(getattr(sols[0], k), getattr(sols[NO_TRIM], k))
                   for k in ("x", "lam", "active", "status", "iters"))
        for _ in range(11):
            for fl in times:
                a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                call(fl)
                e.record(s)
                e.synchronize()
                times[fl].append(a.elapsed_time(e) * 1e3)
        it = sols[NO_TRIM].iters[:B].to(torch.int64)
        t0, t1 = sorted(times[0])[5], sorted(times[NO_TRIM])[5]
        out[f"{fam}_B{B}"] = {"trim_us": round(t0, 1), "single_us": round(t1, 1), "ratio": round(t0 / t1, 4),
                              "bitwise_equal": bool(same), "max_iters": int(it.max()),
                              "frac_over_K": float((it > qpb.TAIL_TRIM_TRIPS).double().mean())}
        print(fam, B, out[f"{fam}_B{B}"], flush=True)
print(json.dumps(out, indent=1))
