#!/usr/bin/env python3
"""qpb_solve_box kernel time across library variants (lib/libqpb_<name>.so,
'head' = lib/libqpb.so) on the same 1M box QPs, rounds interleaved."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
import torch  # noqa: E402

import qpb  # noqa: E402

names = sys.argv[1:]
B, n = int(os.environ.get("B", 1 << 20)), 16
H, f, A, b = qpb.generate(n, B, 20261015, family="box", shift=1.0, box=10.0, device=torch.device("cuda", 0))
ub, lb = b[:, :n].contiguous(), (-b[:, n:]).contiguous()
s = torch.cuda.current_stream()
p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
libs, sols = {}, {}
for nm in names:
    path = os.path.join(ROOT, "embedded-qp-solver_amd", "lib", "libqpb.so" if nm == "head" else f"libqpb_{nm}.so")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    lib.qpb_solve_box.argtypes = [ctypes.POINTER(qpb.Desc)] + [ctypes.c_void_p] * 10
    libs[nm] = lib
    sols[nm] = qpb.solve_box(H, f, lb, ub)


def call(nm):
    o = sols[nm]
    d = qpb.Desc(n, 2 * n, B, 0, 0, 0.0)
    rc = libs[nm].qpb_solve_box(ctypes.byref(d), p(H), p(f), p(lb), p(ub), p(o.x), p(o.lam), p(o.active),
                                p(o.status), p(o.iters), ctypes.c_void_p(s.cuda_stream))
    assert rc == 0, rc


times = {nm: [] for nm in names}
for nm in names:
    call(nm)
for _ in range(int(os.environ.get("ROUNDS", 5))):
    for nm in names:
        for _ in range(int(os.environ.get("REPS", 6))):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            call(nm)
            e1.record(s)
            e1.synchronize()
            times[nm].append(e0.elapsed_time(e1) * 1e3)
out = {}
for nm in names:
    t = sorted(times[nm])
    out[nm] = {"median_us": round(t[len(t) // 2], 1), "same_as_first": bool(torch.equal(sols[nm].x, sols[names[0]].x)),
               "ok": bool((sols[nm].status == 0).all())}
print(json.dumps(out, indent=1))
