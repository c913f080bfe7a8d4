#!/usr/bin/env python3
"""Lockstep group-size endpoints at the metric's shape (n = 16, m = 32, B = 1 M):
the shipped four-QPs-per-wavefront kernel (gi_dense) against the
one-QP-per-wavefront kernel of the n <= 32 class (gi_wave, QPB_FLAG_DIAG_WAVE),
on the box (bench) and dense families.  Per kernel: median kernel time over
interleaved repetitions (HIP events on the launch stream), the max_iter = 1
launch (load, setup, one trip, outputs), iterations per QP and the trips a
four-QP lockstep group runs; both kernels' answers are compared (mask equal,
x within 1e-9 relative).  Prints one JSON object.  usage: group_probe.py [B]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
import torch  # noqa: E402

import qpb  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
REPS = 7


def timed(fn):
    s = torch.cuda.current_stream()
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    fn()
    e.record(s)
    e.synchronize()
    return a.elapsed_time(e)


out = {"B": B, "n": 16, "m": 32}
for fam in ("box", "dense"):
    H, f, A, b = qpb.generate(16, B, 20261015, family=fam, shift=1.0, box=10.0)
    sols = {}
    for name, fl in (("gi_dense", 0), ("gi_wave", qpb.FLAG_DIAG_WAVE)):
        sols[name] = qpb.solve(H, f, A, b, flags=fl)
    torch.cuda.synchronize()
    res = {}
    runs = {k: [] for k in ("gi_dense", "gi_wave", "gi_dense_maxit1", "gi_wave_maxit1")}
    for _ in range(REPS):
        for name, fl in (("gi_dense", 0), ("gi_wave", qpb.FLAG_DIAG_WAVE)):
            runs[name].append(timed(lambda: qpb.solve(H, f, A, b, flags=fl, out=sols[name])))
            runs[name + "_maxit1"].append(timed(lambda: qpb.solve(H, f, A, b, flags=fl, max_iter=1)))
    # the answers of the last full solves
    for name, fl in (("gi_dense", 0), ("gi_wave", qpb.FLAG_DIAG_WAVE)):
        sols[name] = qpb.solve(H, f, A, b, flags=fl)
    torch.cuda.synchronize()
    d, w = sols["gi_dense"], sols["gi_wave"]
    it = d.iters.to(torch.float64)
    B4 = B // 4 * 4
    res["kernel_ms"] = {k: sorted(v)[len(v) // 2] for k, v in runs.items()}
    res["iters_mean"] = float(it.mean())
    res["iters_max"] = int(d.iters.max())
    res["lockstep4_trips"] = float(it[:B4].view(-1, 4).amax(1).mean())
    res["lockstep2_trips"] = float(it[: B // 2 * 2].view(-1, 2).amax(1).mean())
    res["same_mask"] = bool(torch.equal(d.active, w.active))
    res["same_iters"] = bool(torch.equal(d.iters, w.iters))
    xs = d.x.abs().amax(1).clamp(min=1.0)
    res["x_max_rel_diff"] = float(((d.x - w.x).abs().amax(1) / xs).max())
    res["status_ok"] = {k: int((s.status == qpb.OK).sum()) for k, s in sols.items()}
    out[fam] = res
    del H, f, A, b, sols
    torch.cuda.empty_cache()
print(json.dumps(out, indent=1))
