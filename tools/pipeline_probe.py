#!/usr/bin/env python3
"""How much of a launch's fixed cost (ramp-up: every wave slot loading at once;
drain: the last round of waves finishing one by one) does a serving loop hide
when consecutive batches alternate between two HIP streams, so one batch's
drain overlaps the next one's ramp-up?  K solves of the same B-QP batch
(separate outputs per stream) on one stream vs alternating two streams; the
answers are checked equal.  Not the bench: bench.py times one stream."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
import torch  # noqa: E402

import qpb  # noqa: E402

dev = torch.device("cuda", 0)
K = int(os.environ.get("K", 40))
out = {}
for B in (131072, 262144, 1048576):
    H, f, A, b = qpb.generate(16, B, 20261015, family="box", shift=1.0, box=10.0, device=dev)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    sols = [qpb.solve(H, f, A, b, stream=s) for s in streams]
    torch.cuda.synchronize()

    def run(ns):
        torch.cuda.synchronize()
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(torch.cuda.current_stream())
        for s in streams[:ns]:
            s.wait_event(a)
        for k in range(K):
            i = k % ns
            qpb.solve(H, f, A, b, stream=streams[i], out=sols[i])
        for s in streams[:ns]:
            ev = torch.cuda.Event()
            ev.record(s)
            torch.cuda.current_stream().wait_event(ev)
        e.record(torch.cuda.current_stream())
        e.synchronize()
        return a.elapsed_time(e) * 1e3 / K

    res = {}
    for ns in (1, 2, 1, 2, 1, 2):
        res.setdefault(ns, []).append(run(ns))
    same = all(torch.equal(getattr(sols[0], k), getattr(sols[1], k)) for k in ("x", "lam", "active", "status", "iters"))
    one, two = sorted(res[1])[1], sorted(res[2])[1]
    out[f"B{B}"] = {"one_stream_us_per_batch": round(one, 1), "two_streams_us_per_batch": round(two, 1),
                    "gain": round(one / two - 1, 4), "qps_per_s_two_streams": round(B / (two * 1e-6)),
                    "answers_equal": bool(same)}
    print(B, out[f"B{B}"], flush=True)
print(json.dumps(out, indent=1))
