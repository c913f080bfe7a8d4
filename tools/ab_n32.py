#!/usr/bin/env python3
"""A/B timing of libqpb variants on the n=32, m=64 path (configs[4] shape),
rounds interleaved.  usage: python tools/ab_n32.py name[@flags] ...
('head' = lib/libqpb.so; flags = qpb_desc.flags, e.g. head@32 = mixed,
head@96 = mixed without the fp64 re-solve).  env: B (262144), FAM (dense),
ROUNDS (4), REPS (4), N (32), M (64): any size class (e.g. N=128 M=256 B=16384 FAM=box)"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
import torch  # noqa: E402

import qpb  # noqa: E402


def main(names):
    n, m = int(os.environ.get("N", 32)), int(os.environ.get("M", 64))
    B = int(os.environ.get("B", 262144))
    fam = os.environ.get("FAM", "dense")
    rounds, reps = int(os.environ.get("ROUNDS", 4)), int(os.environ.get("REPS", 4))
    H, f, A, b = qpb.generate(n, B, 20261015, family=fam, m=m)
    libs, fl = {}, {}
    for nm in names:
        base, _, fs = nm.partition("@")
        fl[nm] = int(fs or 0)
        path = os.path.join(ROOT, "embedded-qp-solver_amd", "lib",
                            "libqpb.so" if base in ("", "head") else f"libqpb_{base}.so")
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        lib.qpb_solve.argtypes = [ctypes.POINTER(qpb.Desc)] + [ctypes.c_void_p] * 10
        libs[nm] = lib
    s = torch.cuda.current_stream()
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    sols = {nm: qpb.solve(H, f, A, b) for nm in names}

    def call(nm):
        o = sols[nm]
        d = qpb.Desc(n, m, B, 0, fl[nm], 0.0)
        rc = libs[nm].qpb_solve(ctypes.byref(d), p(H), p(f), p(A), p(b), p(o.x), p(o.lam), p(o.active), p(o.status),
                                p(o.iters), ctypes.c_void_p(s.cuda_stream))
        assert rc == 0, rc

    times = {nm: [] for nm in names}
    for nm in names:
        call(nm)
    for _ in range(rounds):
        for nm in names:
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                call(nm)
                e1.record(s)
                e1.synchronize()
                times[nm].append(e0.elapsed_time(e1) * 1e3)
    torch.cuda.synchronize()
    out = {}
    for nm in names:
        t = sorted(times[nm])
        st = sols[nm].status
        out[nm] = {"median_us": round(t[len(t) // 2], 1), "min_us": round(t[0], 1),
                   "redo_frac": float((st == qpb.STATUS_REDO).double().mean()),
                   "ok_frac": float((st == qpb.OK).double().mean()),
                   "iters_mean": float(sols[nm].iters.double().mean()),
                   "x_maxdiff_vs_first": float((sols[nm].x - sols[names[0]].x).abs().max())}
    print(json.dumps({"B": B, "family": fam, "variants": out}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
