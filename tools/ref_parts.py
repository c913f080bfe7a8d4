#!/usr/bin/env python3
"""Time the parts of the reference replicas at n (128), B (16384): the batched
matrix_invert alone, Newton with 0 / 1 / 10 iterations (0: the invert and
the setup only), GD and ADMM with a few iterations.  Prints one JSON object."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
import torch  # noqa: E402

import qpb  # noqa: E402


def t_ms(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        e.record()
        e.synchronize()
        out.append(a.elapsed_time(e))
    return sorted(out)[len(out) // 2]


n, B = int(os.environ.get("N", 128)), int(os.environ.get("B", 16384))
P, q, x0 = qpb.ref_generate(n, B, 1)
res = {"n": n, "B": B, "library": qpb.version()[:60]}
res["invert_ms"] = t_ms(lambda: qpb.matrix_invert(P))
for it in (0, 1, 10):
    res[f"newton_{it}_ms"] = t_ms(lambda: qpb.ref_solve(qpb.REF_NEWTON, P, q, x0, iterations=it))
for it in (1, 2):
    res[f"gd_{it}_ms"] = t_ms(lambda: qpb.ref_solve(qpb.REF_GD, P, q, x0, iterations=it))
for it in (1, 100):
    res[f"admm_{it}_ms"] = t_ms(lambda: qpb.ref_solve(qpb.REF_ADMM, P, q, x0, iterations=it))
sol_x, sol_it = qpb.ref_solve(qpb.REF_NEWTON, P, q, x0, iterations=10)
res["newton_10_iters_mean"] = float(sol_it.double().mean())
print(json.dumps(res, indent=1))
