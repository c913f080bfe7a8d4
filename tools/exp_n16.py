#!/usr/bin/env python3
"""Where the n=16, m=32 kernel's time goes at the metric's batch (1M QPs):
kernel time (HIP events, median), with the inputs read from L2 only
(QPB_FLAG_DIAG_L2), with max_iter = 1 / 2 / 4, the iteration histogram and
the 4-QP lockstep trip count, and the per-section wave ticks of the stamped
build.  usage: exp_n16.py [B] [family]; N=32 runs the n=32, m=64 wave kernel
(configs[4] shape, one QP per wave, default generator scales)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
import torch  # noqa: E402

import qpb  # noqa: E402

N = int(os.environ.get("N", 16))
B = int(sys.argv[1]) if len(sys.argv) > 1 else (1 << 20 if N <= 16 else 262144)
fam = sys.argv[2] if len(sys.argv) > 2 else ("box" if N <= 16 else "dense")
dev = torch.device("cuda", 0)
if N <= 16:
    H, f, A, b = qpb.generate(N, B, 20261015, family=fam, shift=1.0, box=10.0)
else:
    H, f, A, b = qpb.generate(N, B, 20261015, family=fam)
sol = qpb.solve(H, f, A, b)
torch.cuda.synchronize()


def t(fn, reps=9):
    s = torch.cuda.current_stream()
    fn()
    ts = []
    for _ in range(reps):
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        fn()
        e.record(s)
        e.synchronize()
        ts.append(a.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


out = {"B": B, "family": fam, "library": qpb.version()}
out["kernel_ms"] = t(lambda: qpb.solve(H, f, A, b, out=sol))
out["kernel_ms_l2_inputs"] = t(lambda: qpb.solve(H, f, A, b, out=sol, flags=1))
for mi in (1, 2, 4):
    out[f"kernel_ms_max_iter_{mi}"] = t(lambda: qpb.solve(H, f, A, b, out=sol, max_iter=mi))
sol = qpb.solve(H, f, A, b, out=sol)
torch.cuda.synchronize()
it = sol.iters.cpu().long()
out["iters_mean"] = float(it.double().mean())
out["iters_hist"] = torch.bincount(it).tolist()
for w in (2, 4):
    mx = it[: (B // w) * w].view(-1, w).max(1).values.double()
    out[f"lockstep_trips_mean_{w}qp"] = float(mx.mean())
sec = torch.zeros(qpb.N_SECTIONS, dtype=torch.int64, device=dev)
qpb.solve_sections(H, f, A, b, sec, out=sol)
sec.zero_()
a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
qpb.solve_sections(H, f, A, b, sec, out=sol)
e.record()
torch.cuda.synchronize()
v = sec.cpu().tolist()
waves = B // 4 if N <= 16 else B
names = qpb.SECTION_NAMES if N <= 16 else qpb.WAVE_SECTION_NAMES
out["sections_us_per_wave"] = {nm: round(x / waves / 100.0, 3) for nm, x in zip(names, v)}
out["stamped_kernel_ms"] = a.elapsed_time(e)
out["mean_resident_waves"] = round(sum(v) / 100.0 / (a.elapsed_time(e) * 1e3), 1)
print(json.dumps(out, indent=1))
