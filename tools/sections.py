#!/usr/bin/env python3
"""Per-section wave wall time of the diagnostic s_memrealtime builds (100 MHz
ticks): microseconds per wave and mean resident waves.

  python tools/sections.py          n=16, m=32, B=65,536 (box and dense)
  python tools/sections.py n32      n=32, m=64, B=262,144 dense (configs[4] shape)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
import torch  # noqa: E402

import qpb  # noqa: E402

dev = torch.device("cuda", 0)
n32 = len(sys.argv) > 1 and sys.argv[1] == "n32"
cases = [("dense", 32, 262144)] if n32 else [("box", 16, 65536), ("dense", 16, 65536)]
names = qpb.WAVE_SECTION_NAMES if n32 else qpb.SECTION_NAMES
qps_per_wave = 1 if n32 else 4
out = {}
for fam, n, B in cases:
    H, f, A, b = qpb.generate(n, B, 20261015, family=fam)
    sol = qpb.solve(H, f, A, b)
    sec = torch.zeros(20, dtype=torch.int64, device=dev)
    qpb.solve_sections(H, f, A, b, sec, out=sol)
    sec.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    qpb.solve_sections(H, f, A, b, sec, out=sol)
    e1.record()
    torch.cuda.synchronize()
    v = sec.cpu().tolist()
    tot = sum(v)
    waves = B // qps_per_wave
    key = f"{fam}_n{n}"
    out[key] = {name: round(x / waves / 100.0, 3) for name, x in zip(names, v)}  # us per wave
    out[key]["wave_lifetime_us"] = round(tot / waves / 100.0, 3)
    out[key]["kernel_ms"] = e0.elapsed_time(e1)
    out[key]["mean_resident_waves"] = round(tot / 100.0 / (e0.elapsed_time(e1) * 1e3), 1)
print(json.dumps(out, indent=1))
