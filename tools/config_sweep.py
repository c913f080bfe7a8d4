#!/usr/bin/env python3
"""Kernel times of the BASELINE configs beyond the headline one (HIP events,
median of R launches) with the max_iter ablation (setup + one iteration vs
the full solve): configs[3] n=128 m=256 B=16,384, configs[4] shape n=32
m=64 B=262,144 (fp64 and mixed precision), the n = 32 and n = 128 box
families through the dense path and the implicit-A box path, and the headline
n=16 m=32 B=65,536 (configs[1])."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402

qpb = None  # imported in main(), after the forked CPU leg (nothing before it touches the GPU)


def settle(fn, seconds=0.05):
    """fn back to back for about `seconds` (groups of 5, a sync between): the
    GPU's clocks ramp for its first launches after idle (the
    CPU leg before the first row leaves the GPU idle for ~10 s)"""
    import time
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(5):
            fn()
        torch.cuda.synchronize()


def t_kernel(fn, reps=5):
    s = torch.cuda.current_stream()
    settle(fn)  # the clocks out of their idle state first
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


def measure(run, reps, ok, sync, timer):
    """Solve once and record the full solve's outcome (status, iterations)
    BEFORE the timed launches reuse the output buffers: the max_iter = 1
    ablation overwrites status with MAX_ITER on every QP that needs more than
    one iteration (round 5 read ok_frac after it, VERDICT r05 Weak 6).  Then
    the kernel time of the full solve and of the ablation."""
    sol = run()
    sync()
    it = sol.iters.double()
    res = {"ok_frac": float((sol.status == ok).double().mean()), "iters_mean": float(it.mean()),
           "iters_max": int(it.max())}
    res["kernel_ms"] = timer(lambda: run(out=sol), reps)
    res["maxit1_ms"] = timer(lambda: run(mi=1, out=sol), reps)
    return res


def main():
    # argv: [config names ...] [--flags F]
    global qpb
    args = sys.argv[1:]
    flags = 0
    if "--flags" in args:
        i = args.index("--flags")
        flags = int(args[i + 1])
        del args[i:i + 2]
    # The CPU leg first: bench.cpu_run forks one worker per CPU, which is only
    # safe before this process initialises the GPU (round 3's sweep forked
    # after GPU kernels had run, and the pool's workers died with SIGSEGV in
    # the inherited HIP / profiler state).  cpu_run now refuses to fork then.
    cpu_row = ref_newton_n128_cpu() if (not args or "c3_ref_newton" in args) else None
    import qpb as _qpb
    qpb = _qpb
    out = {}
    # name, n, B, family, repetitions, extra flags, path ("dense": qpb_solve on
    # A = [I; -I] for the box family; "box": qpb_solve_box, A implicit)
    rows = (("c1_n16_m32", 16, 65536, "box", 9, 0, "dense"), ("c4_n32_m64", 32, 262144, "dense", 5, 0, "dense"),
            ("c4_n32_m64_mixed", 32, 262144, "dense", 5, qpb.FLAG_MIXED, "dense"),
            ("c4_n32_box_dense_path", 32, 262144, "box", 5, 0, "dense"),
            ("c4_n32_box_fast_path", 32, 262144, "box", 5, 0, "box"),
            ("c3_n128_m256", 128, 16384, "box", 3, 0, "dense"),
            ("c3_n128_box_fast_path", 128, 16384, "box", 3, 0, "box"))
    for name, n, B, fam, reps, fl, path in rows:
        if args and name not in args:
            continue
        fl |= flags
        H, f, A, b = qpb.generate(n, B, 20261015, family=fam)
        if path == "box":
            ub, lb = b[:, :n].contiguous(), (-b[:, n:]).contiguous()
            run = lambda mi=0, out=None: qpb.solve_box(H, f, lb, ub, max_iter=mi, out=out)  # noqa: E731
            bpq = 8 * (n * n + 3 * n + n + 2 * n) + 4 * ((2 * n + 31) // 32) + 4  # H f lb ub | x lam mask status
        else:
            run = lambda mi=0, out=None: qpb.solve(H, f, A, b, max_iter=mi, out=out, flags=fl)  # noqa: E731
            bpq = bench.bytes_per_qp(n, 2 * n)
        st = measure(run, reps, qpb.OK, torch.cuda.synchronize, t_kernel)
        ms = st["kernel_ms"]
        out[name] = {"n": n, "m": 2 * n, "batch": B, "family": fam, "path": path, "kernel_ms": ms,
                     "maxit1_ms": st["maxit1_ms"], "qps_per_s": B / (ms * 1e-3), "bytes_per_qp": bpq,
                     "achieved_GBs": B * bpq / (ms * 1e-3) / 1e9, "frac_of_8TBs": B * bpq / (ms * 1e-3) / 8e12,
                     "iters_mean": st["iters_mean"], "iters_max": st["iters_max"], "ok_frac": st["ok_frac"],
                     "flags": fl}
        sol = None
        print(name, json.dumps(out[name]), file=sys.stderr, flush=True)
        del H, f, A, b, sol
        torch.cuda.empty_cache()
    if cpu_row is not None:
        out["c3_ref_newton"] = ref_newton_n128(cpu_row)
        print("c3_ref_newton", json.dumps(out["c3_ref_newton"]), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))
    bad = [k for k, v in out.items() if "ok_frac" in v and v["ok_frac"] != 1.0]
    if bad:  # every QP of every config must solve; the JSON above shows which did not
        sys.exit(f"ok_frac below 1.0: {bad}")


def ref_newton_n128_cpu(cpu_qps=512, seconds=10.0, seed=1):
    """CPU half of the like-for-like row: the compiled reference's Newton
    (oracle/_ref/libqpref_n128_1e12.so, one forked process per CPU of this
    job's share) on the first cpu_qps QPs of the reference generator
    (srand(seed), generated by the compiled reference itself -- bit-exact with
    qpb_ref_generate, tests/test_gpu_generators.py).  Runs before any GPU call."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import refc
    procs = bench.cpu_share()
    if not refc.available(128):
        return {"cpu_reference_qps_per_s": None, "cpu_cores": procs, "cpu_sample_qps": 0,
                "note": "oracle/_ref/libqpref_n128_1e12.so missing"}
    P, q, _ = refc.RefC(128).generate(seed, cpu_qps)
    cpu = bench.cpu_run("ref_newton_batch", 10, P, q, seconds, procs, lib_name="libqpref_n128_1e12.so")
    return {"cpu_reference_qps_per_s": cpu, "cpu_cores": procs, "cpu_sample_qps": cpu_qps, "seed": seed}


def ref_newton_n128(cpu_row, B=16384, seed=1):
    """Like-for-like at configs[3]'s n = 128: the reference's own Newton
    (qp_solvers.c:103-144, 10 iterations, x0 = 0 on both sides) on the
    reference generator's P and q (srand(seed)): the bitwise GPU replica
    (qpb_ref_solve, B QPs from qpb_ref_generate) against the compiled
    reference's rate from ref_newton_n128_cpu (the first QPs of the same
    sequence)."""
    n = 128
    P, q, _ = qpb.ref_generate(n, B, seed=seed)
    x0 = torch.zeros_like(q)
    sol = qpb.ref_solve(qpb.REF_NEWTON, P, q, x0, iterations=10)
    torch.cuda.synchronize()
    ms = t_kernel(lambda: qpb.ref_solve(qpb.REF_NEWTON, P, q, x0, iterations=10), 3)
    row = {"n": n, "batch": B, "iterations": 10, "gpu_kernel_ms": ms, "gpu_qps_per_s": B / (ms * 1e-3)}
    cpu = cpu_row.get("cpu_reference_qps_per_s")
    row.update(cpu_row)
    row.update({"ratio": (B / (ms * 1e-3)) / cpu if cpu else None,
                "bitwise_vs_reference": "tests/test_gpu_reference_modes.py (n = 128)"})
    del sol
    return row


if __name__ == "__main__":
    main()
