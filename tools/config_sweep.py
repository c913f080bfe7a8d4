#!/usr/bin/env python3
"""Kernel times of the BASELINE configs beyond the headline one (HIP events,
median of R launches) with the max_iter ablation (setup + one iteration vs
the full solve): configs[3] n=128 m=256 B=16,384, configs[4] shape n=32
m=64 B=262,144 (fp64), and the headline n=16 m=32 B=65,536 for reference."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import qpb  # noqa: E402


def t_kernel(fn, reps=5):
    s = torch.cuda.current_stream()
    fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        fn()
        b.record(s)
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    # argv: [config names ...] [--flags F]
    args = sys.argv[1:]
    flags = 0
    if "--flags" in args:
        i = args.index("--flags")
        flags = int(args[i + 1])
        del args[i:i + 2]
    out = {}
    for name, n, B, fam, reps in (("c1_n16_m32", 16, 65536, "box", 9), ("c4_n32_m64", 32, 262144, "dense", 5),
                                  ("c3_n128_m256", 128, 16384, "box", 3)):
        if args and name not in args:
            continue
        H, f, A, b = qpb.generate(n, B, 20261015, family=fam)
        sol = qpb.solve(H, f, A, b, flags=flags)
        torch.cuda.synchronize()
        it = sol.iters.double()
        ms = t_kernel(lambda: qpb.solve(H, f, A, b, out=sol, flags=flags), reps)
        ms1 = t_kernel(lambda: qpb.solve(H, f, A, b, max_iter=1, out=sol, flags=flags), reps)
        bpq = bench.bytes_per_qp(n, 2 * n)
        out[name] = {"n": n, "m": 2 * n, "batch": B, "family": fam, "kernel_ms": ms, "maxit1_ms": ms1,
                     "qps_per_s": B / (ms * 1e-3), "achieved_GBs": B * bpq / (ms * 1e-3) / 1e9,
                     "frac_of_8TBs": B * bpq / (ms * 1e-3) / 8e12, "iters_mean": float(it.mean()),
                     "iters_max": int(it.max()), "flags": flags}
        print(name, json.dumps(out[name]), file=sys.stderr, flush=True)
    if not args or "c3_ref_newton" in args:
        out["c3_ref_newton"] = ref_newton_n128()
        print("c3_ref_newton", json.dumps(out["c3_ref_newton"]), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


def ref_newton_n128(B=16384, cpu_qps=512, seconds=10.0):
    """Like-for-like at configs[3]'s n = 128: the reference's own Newton
    (qp_solvers.c:103-144, 10 iterations, x0 = 0 on both sides) on the
    reference generator's P and q (qpb_ref_generate, srand 1), as the bitwise
    GPU replica (qpb_ref_solve,
    B QPs) and as the compiled reference (oracle/_ref/libqpref_n128_1e12.so,
    one process per CPU of this job's share, on the first cpu_qps of them)."""
    n = 128
    P, q, _ = qpb.ref_generate(n, B, seed=1)
    x0 = torch.zeros_like(q)
    sol = qpb.ref_solve(qpb.REF_NEWTON, P, q, x0, iterations=10)
    torch.cuda.synchronize()
    ms = t_kernel(lambda: qpb.ref_solve(qpb.REF_NEWTON, P, q, x0, iterations=10), 3)
    row = {"n": n, "batch": B, "iterations": 10, "gpu_kernel_ms": ms, "gpu_qps_per_s": B / (ms * 1e-3)}
    procs = bench.cpu_share()
    Pc, qc = P[:cpu_qps].cpu().numpy(), q[:cpu_qps].cpu().numpy()
    cpu = bench.cpu_run("ref_newton_batch", 10, Pc, qc, seconds, procs, lib_name="libqpref_n128_1e12.so")
    row.update({"cpu_reference_qps_per_s": cpu, "cpu_cores": procs, "cpu_sample_qps": cpu_qps,
                "ratio": (B / (ms * 1e-3)) / cpu if cpu else None,
                "bitwise_vs_reference": "tests/test_gpu_reference_modes.py (n = 128, 64 QPs)"})
    return row


if __name__ == "__main__":
    main()
