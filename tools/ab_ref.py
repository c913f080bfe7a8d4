#!/usr/bin/env python3
"""A/B timing of libqpb variants on the reference-semantics replicas
(qpb_ref_solve), rounds interleaved, bitwise agreement checked.
usage: python tools/ab_ref.py name ...  ('head' = lib/libqpb.so)
env: N (128), B (16384), MODE (newton|admm|gd), ITERS (10), ROUNDS (3)"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
import torch  # noqa: E402

import qpb  # noqa: E402


def main(names):
    n, B = int(os.environ.get("N", 128)), int(os.environ.get("B", 16384))
    mode = {"newton": qpb.REF_NEWTON, "admm": qpb.REF_ADMM, "gd": qpb.REF_GD}[os.environ.get("MODE", "newton")]
    iters, rounds = int(os.environ.get("ITERS", 10)), int(os.environ.get("ROUNDS", 3))
    P, q, x0 = qpb.ref_generate(n, B, 1)
    s = torch.cuda.current_stream()
    libs = {}
    for nm in names:
        path = os.path.join(ROOT, "embedded-qp-solver_amd", "lib", "libqpb.so" if nm == "head" else f"libqpb_{nm}.so")
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        lib.qpb_ref_solve.argtypes = [ctypes.POINTER(qpb.RefDesc)] + [ctypes.c_void_p] * 6
        libs[nm] = lib
    outs = {nm: (torch.empty_like(q), torch.empty((B,), dtype=torch.int32, device=q.device)) for nm in names}
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def call(nm):
        x, it = outs[nm]
        d = qpb.RefDesc(n, mode, B, iters, 0, -1e12, 1e12)
        rc = libs[nm].qpb_ref_solve(ctypes.byref(d), p(P), p(q), p(x0), p(x), p(it), ctypes.c_void_p(s.cuda_stream))
        assert rc == 0, rc

    times = {nm: [] for nm in names}
    for nm in names:
        call(nm)
    for _ in range(rounds):
        for nm in names:
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            call(nm)
            e.record(s)
            e.synchronize()
            times[nm].append(a.elapsed_time(e))
    ref = names[0]
    print(json.dumps({"n": n, "B": B, "iterations": iters, "variants": {
        nm: {"median_ms": sorted(t)[len(t) // 2], "bitwise_as_first": bool(torch.equal(outs[nm][0].view(torch.int64), outs[ref][0].view(torch.int64)))}
        for nm, t in times.items()}}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
