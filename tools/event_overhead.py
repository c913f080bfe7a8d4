#!/usr/bin/env python3
"""Does recording HIP events between the bench's launches change the launches?

The bench line's timed loop records an event pair around every qpb_solve; its
sustained leg launches back to back.  Interleaved here, on the metric's batch
(1 M QPs, n = 16, box family): K launches with an event pair around each, K
launches with one pair around the K, and K launches with no event at all
(host wall clock after a synchronize), ROUNDS times each.  Prints one JSON
object: per mode the median ms per launch (wall and, where recorded, events).
env: B (1048576), K (20), ROUNDS (8)
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
    B, K, R = int(os.environ.get("B", 1 << 20)), int(os.environ.get("K", 20)), int(os.environ.get("ROUNDS", 8))
    dev = torch.device("cuda", 0)
    H, f, A, b = qpb.generate(16, B, 20261015, family="box", shift=1.0, box=10.0, device=dev)
    s = torch.cuda.current_stream()
    sol = qpb.solve(H, f, A, b, stream=s)
    for _ in range(200):  # the clock settles
        qpb.solve(H, f, A, b, out=sol, stream=s)
    torch.cuda.synchronize()
    res = {"per_launch_events": {"wall": [], "events": []}, "outer_events": {"wall": [], "events": []},
           "no_events": {"wall": []}}
    for _ in range(R):
        # an event pair around every launch (bench.py's timed loop)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for e0, e1 in evs:
            e0.record(s)
            qpb.solve(H, f, A, b, out=sol, stream=s)
            e1.record(s)
        torch.cuda.synchronize()
        res["per_launch_events"]["wall"].append((time.perf_counter() - t0) / K * 1e3)
        res["per_launch_events"]["events"].append(sum(a.elapsed_time(e) for a, e in evs) / K)
        # one pair around the K launches
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(s)
        for _ in range(K):
            qpb.solve(H, f, A, b, out=sol, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        res["outer_events"]["wall"].append((time.perf_counter() - t0) / K * 1e3)
        res["outer_events"]["events"].append(e0.elapsed_time(e1) / K)
        # none
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            qpb.solve(H, f, A, b, out=sol, stream=s)
        torch.cuda.synchronize()
        res["no_events"]["wall"].append((time.perf_counter() - t0) / K * 1e3)
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    out = {"B": B, "K": K, "rounds": R,
           "ms_per_launch_median": {m: {k: round(med(v), 4) for k, v in d.items()} for m, d in res.items()},
           "raw": res}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
