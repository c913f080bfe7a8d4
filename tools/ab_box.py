#!/usr/bin/env python3
"""Kernel time of the box fast path (qpb_solve_box) against the dense path
(qpb_solve with A = [I; -I]) on the same QPs, rounds interleaved.
env: B (1048576), N (16), ROUNDS (5), REPS (6)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
import torch  # noqa: E402

import qpb  # noqa: E402

B, n = int(os.environ.get("B", 1 << 20)), int(os.environ.get("N", 16))
rounds, reps = int(os.environ.get("ROUNDS", 5)), int(os.environ.get("REPS", 6))
H, f, A, b = qpb.generate(n, B, 20261015, family="box", shift=1.0, box=10.0, device=torch.device("cuda", 0))
ub = b[:, :n].contiguous()
lb = (-b[:, n:]).contiguous()
s = torch.cuda.current_stream()
sd = qpb.solve(H, f, A, b)
sb = qpb.solve_box(H, f, lb, ub)
calls = {"dense": lambda: qpb.solve(H, f, A, b, out=sd), "box": lambda: qpb.solve_box(H, f, lb, ub, out=sb)}
times = {k: [] for k in calls}
for k in calls:
    calls[k]()
for _ in range(rounds):
    for k, c in calls.items():
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            c()
            e1.record(s)
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) * 1e3)
torch.cuda.synchronize()
out = {"B": B, "n": n, "same_active": bool(torch.equal(sd.active, sb.active)),
       "x_maxdiff": float((sd.x - sb.x).abs().max())}
for k, t in times.items():
    t = sorted(t)
    out[k] = {"median_us": round(t[len(t) // 2], 1), "min_us": round(t[0], 1)}
bpq_box = 8 * (n * n + 3 * n) + 8 * (n + 2 * n) + 4 + 4
out["box"]["bytes_per_qp"] = bpq_box
out["box"]["hbm_frac"] = B * bpq_box / (out["box"]["median_us"] * 1e-6) / 8e12
print(json.dumps(out, indent=1))
