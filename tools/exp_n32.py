#!/usr/bin/env python3
"""configs[4] shape (n=32, m=64, B=262,144): kernel time of the fp64 wave
kernel and of the mixed-precision path (QPB_FLAG_MIXED, with and without the
fp64 re-solve launch), the re-solve fraction, and iterations.  HIP events on
the launch stream, median of REPS.  usage: exp_n32.py [B] [family]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
import torch  # noqa: E402

import qpb  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
fam = sys.argv[2] if len(sys.argv) > 2 else "dense"
H, f, A, b = qpb.generate(32, B, 20261015, family=fam)
sol = qpb.solve(H, f, A, b)
torch.cuda.synchronize()


def t(flags, reps=7):
    s = torch.cuda.current_stream()
    qpb.solve(H, f, A, b, out=sol, flags=flags)
    ts = []
    for _ in range(reps):
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        qpb.solve(H, f, A, b, out=sol, flags=flags)
        e.record(s)
        e.synchronize()
        ts.append(a.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


out = {"B": B, "family": fam, "library": qpb.version()}
out["fp64_ms"] = t(0)
it64 = sol.iters.double().mean().item()
out["mixed_ms"] = t(qpb.FLAG_MIXED)
out["mixed_no_redo_ms"] = t(qpb.FLAG_MIXED | qpb.FLAG_DIAG_NO_REDO)
out["redo_fraction"] = float((sol.status == qpb.STATUS_REDO).double().mean())
out["iters_mean_fp64"] = it64
out["iters_mean_fp32"] = sol.iters.double().mean().item()
bpq = 8 * (32 * 32 + 32 + 64 * 32 + 64) + 8 * (32 + 64) + 4 * 2 + 4
for k in ("fp64_ms", "mixed_ms"):
    out[k.replace("_ms", "_qps")] = B / (out[k] * 1e-3)
    out[k.replace("_ms", "_frac")] = B * bpq / (out[k] * 1e-3) / 8e12
print(json.dumps(out, indent=1))
