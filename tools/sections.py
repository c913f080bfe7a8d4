#!/usr/bin/env python3
"""Per-section wave wall time of the n=16, m=32 kernel (diagnostic
s_memrealtime build, 100 MHz ticks): microseconds per wave and share."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import qpb  # noqa: E402

dev = torch.device("cuda", 0)
out = {}
for fam in ("box", "dense"):
    H, f, A, b = bench.make_batch(torch, 65536, 16, fam, 1, dev)
    sol = qpb.solve(H, f, A, b)
    sec = torch.zeros(12, dtype=torch.int64, device=dev)
    qpb.solve_sections(H, f, A, b, sec, out=sol)
    sec.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    qpb.solve_sections(H, f, A, b, sec, out=sol)
    e1.record()
    torch.cuda.synchronize()
    v = sec.cpu().tolist()
    tot = sum(v)
    waves = 65536 // 4
    out[fam] = {name: round(x / waves / 100.0, 3) for name, x in zip(qpb.SECTION_NAMES, v)}  # us per wave
    out[fam]["wave_lifetime_us"] = round(tot / waves / 100.0, 3)
    out[fam]["kernel_ms"] = e0.elapsed_time(e1)
    out[fam]["mean_resident_waves"] = round(tot / 100.0 / (e0.elapsed_time(e1) * 1e3), 1)
print(json.dumps(out, indent=1))
