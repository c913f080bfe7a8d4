#!/usr/bin/env python3
"""How long the n = 16 kernel takes to reach its steady rate after the GPU
has been idle (bench.py's timed steps follow a ~10 s CPU-only baseline leg).

After IDLE seconds without GPU work, PRE seconds of back-to-back solves of
the same batch, then 5 warmup launches and 20 launches with an event pair
around each (the bench's timed loop); reported per PRE in the PRES list,
twice over, on one box.  env: PRES ("0,0.05,0.15,0.5,1.5"), IDLE (10), B (1048576)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
import torch  # noqa: E402

import qpb  # noqa: E402


def main():
    B = int(os.environ.get("B", 1 << 20))
    pres = [float(x) for x in os.environ.get("PRES", "0,0.05,0.15,0.5,1.5").split(",")]
    idle = float(os.environ.get("IDLE", 10))
    dev = torch.device("cuda", 0)
    H, f, A, b = qpb.generate(16, B, 20261015, family="box", shift=1.0, box=10.0, device=dev)
    s = torch.cuda.current_stream()
    sol = qpb.solve(H, f, A, b, stream=s)
    torch.cuda.synchronize()
    rows = []
    for rep in range(2):
        for pre in pres:
            time.sleep(idle)
            t0 = time.perf_counter()
            npre = 0
            while time.perf_counter() - t0 < pre:
                for _ in range(5):
                    qpb.solve(H, f, A, b, out=sol, stream=s)
                npre += 5
                torch.cuda.synchronize()
            for _ in range(5):
                qpb.solve(H, f, A, b, out=sol, stream=s)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for e0, e1 in evs:
                e0.record(s)
                qpb.solve(H, f, A, b, out=sol, stream=s)
                e1.record(s)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t1) / 20 * 1e3
            ev = [a.elapsed_time(e) for a, e in evs]
            rows.append({"rep": rep, "pre_s": pre, "pre_launches": npre, "wall_ms": round(wall, 4),
                         "kernel_ms": round(sum(ev) / 20, 4), "first5_ms": round(sum(ev[:5]) / 5, 4),
                         "last5_ms": round(sum(ev[-5:]) / 5, 4)})
            print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    print(json.dumps({"B": B, "idle_s": idle, "rows": rows}, indent=1))


if __name__ == "__main__":
    main()
