#!/usr/bin/env python3
"""Where does the fixed per-launch cost of the n=16 kernel come from?  Kernel
time at several batch sizes with the default iteration cap and with
max_iter = 1 (load, setup, one trip, outputs: no iteration tail), and with
the inputs of QP g mod 16384 (QPB_FLAG_DIAG_MALL: no HBM ramp).  The fixed
part is the intercept of T(B) = a + c B over the two largest batches."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
import torch  # noqa: E402

import qpb  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [65536, 131072, 524288, 1048576]
H, f, A, b = qpb.generate(16, sizes[-1], 1, family="box", shift=1.0, box=10.0, device=dev)
s = torch.cuda.current_stream()
p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
out = {}
for maxit, flags, tag in ((0, 0, "full"), (1, 0, "maxit1"), (0, 16, "mall"), (1, 16, "maxit1_mall")):
    for B in sizes:
        sol = qpb.solve(H[:B], f[:B], A[:B], b[:B])
        d = qpb.Desc(16, 32, B, maxit, flags, 0.0)

        def call():
            rc = qpb.lib().qpb_solve(ctypes.byref(d), p(H), p(f), p(A), p(b), p(sol.x), p(sol.lam), p(sol.active),
                                     p(sol.status), p(sol.iters), ctypes.c_void_p(s.cuda_stream))
            assert rc == 0, rc
        call()
        ts = []
        for _ in range(9):
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            call()
            e.record(s)
            e.synchronize()
            ts.append(a.elapsed_time(e) * 1e3)
        out[f"{tag}_B{B}_us"] = round(sorted(ts)[4], 1)
    c = (out[f"{tag}_B{sizes[-1]}_us"] - out[f"{tag}_B{sizes[-2]}_us"]) / (sizes[-1] - sizes[-2])
    out[f"{tag}_intercept_us"] = round(out[f"{tag}_B{sizes[-1]}_us"] - c * sizes[-1], 1)
    out[f"{tag}_ns_per_qp"] = round(c * 1e3, 4)
print(json.dumps(out, indent=1))
