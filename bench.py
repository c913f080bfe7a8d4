#!/usr/bin/env python3
"""bench.py -- QPs/sec of the batched MI355X QP solver (BASELINE.json metric).

Metric (BASELINE.json): "QPs/sec (whole node) at n=16,m=32 batch=1M".  The
default workload is that config: a GLOBAL batch of 1,048,576 dense QPs, n=16,
m=32, fp64, sharded by QP index over the ranks (configs[2]; on one GPU it is
the whole 1 M batch -- 7.26 GB, it fits one MI355X), solved by the active-set
kernel (qpb_solve) through the C-ABI.  Synthetic "conditioned box" family
(SURVEY.md §8d): H = B^T B/(1e3 n) + I (the reference generator's P,
matrix_ops.c:699-734, shifted), f ~ U[-1e3,1e3], box |x_i| <= 10 written as a
dense A = [I; -I], b = 10 (so the solver reads the full dense (H, f, A, b)).
Inputs are generated on the GPU and resident in HBM before the timed region.
This replaces the reference's serial per-QP loop (main.c:36-59).

One step = one qpb_solve call over the rank's shard.  Multi-GPU: one process
per GPU.  `--gpus N` without a torchrun environment relaunches this script
under torch.distributed.run (a child process, started before anything here
touches the GPU); every rank solves its contiguous shard with no collective in
the data path; timings are max-reduced over ranks.  Scaling is "strong": the
1 M batch is fixed as N grows (`--batch B` gives weak scaling at B per GPU).

Also reported:
  roofline     -- algorithmic HBM bytes per launch / mean kernel time (HIP
                  events on the launch stream) vs 8 TB/s
  cpu_baseline -- the reference's own qp_solvers.c admm() (compiled from
                  /root/reference by oracle/Makefile, box +-10 compiled in) on
                  a sample of the same QPs, one forked process per core of
                  this process's CPU share, rank 0, N=1
  like_for_like -- the reference's Newton and ADMM: the GPU replicas
                  (qpb_ref_solve) against the compiled reference on the
                  same QPs (extra keys; N=1 only)
"""
from __future__ import annotations

import argparse
import json
import os
import re
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))

BASELINE_METRIC = "QPs/sec (whole node) at n=16,m=32 batch=1M; % HBM roofline at 1/2/4/8 GPUs"  # BASELINE.json
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); 6.29 TB/s measured copy
METRIC_BATCH = 1 << 20


def bytes_per_qp(n: int, m: int) -> int:
    """Algorithmic HBM bytes per QP: inputs H n*n, f n, A m*n,
    b m; outputs x n, lam m, active ceil(m/32) words, status 1 word (fp64 = 8 B)."""
    return 8 * (n * n + n + m * n + m) + 8 * (n + m) + 4 * ((m + 31) // 32) + 4


def baseline_config(n: int, total: int, world: int) -> str:
    """Which BASELINE.json config a run measures."""
    if n == 16 and total == METRIC_BATCH:
        return "BASELINE configs[2] (the metric's 1M batch)"
    if n == 16 and total == 65536 and world == 1:
        return "BASELINE configs[1]"
    if n == 32 and total == 262144:
        return "BASELINE configs[4] shape"
    if n == 128 and total == 16384:
        return "BASELINE configs[3]"
    return "not a BASELINE config"


def kernel_revisions(library: str) -> set:
    """The per-kernel revision tokens of qpb_version(): "qpb X (gfx950; gi_dense
    v10: ...; gi_box v1: ...)" -> {"gi_dense v10", "gi_box v1", ...}."""
    inner = library.split("(", 1)[1].rsplit(")", 1)[0] if "(" in library else library
    return {part.split(":", 1)[0].strip() for part in inner.split(";") if ":" in part}


def pmc_traffic(n: int, m: int, B: int, family: str, library: str):
    """HBM bytes per launch measured by rocprofv3 PMC passes (FETCH_SIZE,
    WRITE_SIZE; gfx950-corrected, tools/summarize_profile.py) and the VALU
    instruction classes per wave, for this exact kernel configuration and
    revision, from the committed profiles/pmc_traffic.json, or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        t = json.load(open(path))
    except (OSError, ValueError):
        return None
    c = t.get("config", {})
    if (c.get("n"), c.get("m"), c.get("batch_per_gpu"), c.get("family")) != (n, m, B, family):
        return None
    rev = t.get("kernel_rev")
    if not rev or rev not in kernel_revisions(library):  # measured on another revision of the hot kernel
        return None
    return {"bytes": t["hbm_bytes_per_launch"], "source": t.get("source", path),
            "valu_classes": t.get("valu_classes"), "valu_source": t.get("valu_source")}


# Issue cost of one wave64 instruction per SIMD, by class (cycles at 2.4 GHz,
# many waves per SIMD: tools/probe/valu_probe.hip, profiles/r03/valu_probe_r03.jsonl).
# fp64 add has no probe of its own and is charged as mul; the 32-bit classes
# (integer, conversions, selects, DPP moves, the rest of SQ_INSTS_VALU) at the
# v_fma_f32 rate.
VALU_COST = {"FMA_F64": 5.24, "MUL_F64": 5.47, "ADD_F64": 5.47, "TRANS_F64": 17.23, "B32": 3.07}
SIMDS, CLOCK_GHZ = 1024, 2.4  # MI355X: 256 CUs x 4 SIMDs, peak engine clock


def shard_time_prediction(n: int, m: int, family: str, shard_qps: int, total_qps: int, library: str = ""):
    """One-GPU kernel time of a `shard_qps` launch and of the whole batch, by
    linear interpolation of the committed batch scan (profiles/batch_scan.json,
    tools/batch_scan.py, box family at n = 16, m = 32), and the speed-up the
    kernel alone allows: T(total) / T(shard).  None outside the scanned range,
    and None when the scan was taken on another revision of the hot kernel
    than the loaded library's (its `revision` not among kernel_revisions)."""
    path = os.path.join(ROOT, "profiles", "batch_scan.json")
    if (n, m, family) != (16, 32, "box") or not os.path.exists(path):
        return None
    scan = json.load(open(path))
    if library and scan.get("revision") not in kernel_revisions(library):
        return None
    # back-to-back launch times where the scan has them (bench.py's timed
    # steps are queued without a wait), else the waited-for single launches
    kind = "_b2b_us" if any(k.endswith("_b2b_us") for k in scan) else "_us"
    pts = sorted((int(m_.group(1)), v) for k, v in scan.items()
                 for m_ in [re.match(r"^B(\d+)" + kind + "$", k)] if m_)

    def t_us(b):
        for (b0, t0), (b1, t1) in zip(pts, pts[1:]):
            if b0 <= b <= b1:
                return t0 + (t1 - t0) * (b - b0) / (b1 - b0)
        return None
    ts, tt = t_us(shard_qps), t_us(total_qps)
    if ts is None or tt is None:
        return None
    return {"shard_kernel_ms": ts * 1e-3, "total_kernel_ms": tt * 1e-3, "kernel_bound_speedup": tt / ts,
            "source": "profiles/batch_scan.json (one GPU, kernel time vs batch, "
                      + ("launches back to back)" if kind == "_b2b_us" else "single launches)"),
            "revision": scan.get("revision")}


def valu_ceiling(traffic, waves: int, kern_ms: float):
    """The kernel's issue-rate bound: every VALU instruction class of the
    committed PMC pass (SQ_INSTS_VALU_FMA_F64 / _MUL_F64 / _ADD_F64 /
    _TRANS_F64 per wave; the rest of SQ_INSTS_VALU as 32-bit) charged its
    measured issue cost, issued back to back on every SIMD at the peak clock,
    against the measured kernel time."""
    cls = (traffic or {}).get("valu_classes")
    if not cls or not cls.get("VALU"):
        return None
    f64 = {k: cls.get(k, 0.0) for k in ("FMA_F64", "MUL_F64", "ADD_F64", "TRANS_F64")}
    b32 = max(0.0, cls["VALU"] - sum(f64.values()))
    cycles = sum(VALU_COST[k] * v for k, v in f64.items()) + VALU_COST["B32"] * b32
    ms = cycles * waves / SIMDS / (CLOCK_GHZ * 1e9) * 1e3
    return {"valu_insts_per_wave": cls["VALU"], "classes_per_wave": dict(f64, B32=b32),
            "cycles_per_class": VALU_COST, "issue_cycles_per_wave": cycles,
            "ceiling_ms": ms, "kernel_ms": kern_ms, "frac": ms / kern_ms, "source": traffic.get("valu_source"),
            "note": "time if every SIMD issued the wave's instructions back to back at their measured costs "
                    "(2.4 GHz, no stall)"}


# --------------------------------------------------------------------------- CPU share
def cpu_share() -> int:
    """CPUs this process may use: its affinity set, capped by a cgroup CPU quota
    and by the OMP_NUM_THREADS share the GPU box sets (16 per GPU there)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


# --------------------------------------------------------------------------- CPU baseline
def _cpu_worker(args):
    lib_path, fn, P, q, iters, seconds = args
    import ctypes

    import numpy as np
    L = ctypes.CDLL(lib_path)
    dp = ctypes.POINTER(ctypes.c_double)
    x0 = np.zeros_like(q)
    x = np.zeros_like(q)
    done, chunk, i = 0, 64, 0
    t0 = time.perf_counter()
    while True:
        j = min(i + chunk, len(q))
        getattr(L, fn)(ctypes.c_uint(j - i), P[i:j].ctypes.data_as(dp), q[i:j].ctypes.data_as(dp),
                       x0[i:j].ctypes.data_as(dp), ctypes.c_uint(iters), x[i:j].ctypes.data_as(dp))
        done += j - i
        i = 0 if j >= len(q) else j
        el = time.perf_counter() - t0
        if el >= seconds:
            return done, el


def cpu_run(fn: str, iters: int, H, f, seconds: float, procs: int, lib_name: str = "libqpref_n16_10.so"):
    """The compiled reference solver `fn` (oracle/ref_driver.c over the
    unmodified qp_solvers.c, built for N_DIM and the ADMM box of `lib_name`)
    on the given QPs, one forked process per CPU (the reference is not
    thread-safe: static pools kmalloc.c:37-42)."""
    import multiprocessing as mp

    import numpy as np
    torch_mod = sys.modules.get("torch")
    if torch_mod is not None and torch_mod.cuda.is_initialized():
        # forked workers would inherit the HIP runtime state (and a profiler's
        # signal handlers): the config sweep's SIGSEGV of round 3
        raise RuntimeError("bench.cpu_run: the GPU is initialised in this process; run the CPU leg first")
    lib = os.path.join(ROOT, "oracle", "_ref", lib_name)
    if not os.path.exists(lib):
        return None
    P, q = np.ascontiguousarray(H), np.ascontiguousarray(f)
    per = max(1, len(q) // procs)
    jobs = [(lib, fn, P[k * per:(k + 1) * per], q[k * per:(k + 1) * per], iters, seconds) for k in range(procs)]
    with mp.get_context("fork").Pool(procs) as pool:
        res = pool.map(_cpu_worker, jobs)
    return sum(d / el for d, el in res)


def cpu_baselines(H, f, seconds: float, procs: int):
    """cpu_baseline (reference admm(), the reference's only constrained
    solver) plus the reference Newton for the like-for-like rows."""
    lib = os.path.join(ROOT, "oracle", "_ref", "libqpref_n16_10.so")
    if not os.path.exists(lib):
        return ({"value": None, "unit": "QPs/s", "cores": 0, "kind": "reference",
                 "sample": "oracle/_ref/libqpref_n16_10.so missing (build with make -C oracle ref)"}, None)
    admm = cpu_run("ref_admm_batch", 10000, H, f, seconds, procs)
    newton = cpu_run("ref_newton_batch", 10, H, f, seconds / 2, procs)
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:  # noqa: BLE001
        model = "unknown"
    host = os.cpu_count() or procs
    base = {"value": admm, "unit": "QPs/s", "cores": procs, "kind": "reference",
            "solver": "qp_solvers.c admm() (the reference's only constrained solver), box +-10 compiled in, "
                      "ADMM_ITERATIONS 1e4 (config.h:38)",
            "sample": f"the batch's first {len(f)} QPs (restated on the CPU) cycled for {seconds:.0f} s per "
                      f"process, {procs} forked processes = this process's CPU share",
            "cpu_model": model, "host_cpus": host,
            "per_core": admm / procs,
            "host_extrapolated": admm / procs * host,
            "host_extrapolated_note": f"per-core rate x all {host} host CPUs (linear; not measured: the "
                                      f"GPU box grants {procs} CPUs to this job)"}
    return base, newton


# --------------------------------------------------------------------------- multi-GPU launch
def relaunch(n: int) -> int:
    """`--gpus N` outside torchrun: run this script under torch.distributed.run
    as a child process (nothing here has touched the GPU) and return its code."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


# --------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--global-batch", type=int, default=METRIC_BATCH,
                    help="total QPs sharded over the GPUs (strong scaling; default: the metric's 1M)")
    ap.add_argument("--batch", type=int, default=0, help="QPs per GPU (weak scaling; overrides --global-batch)")
    ap.add_argument("--gather", action="store_true",
                    help="after the timed region, gather x/lam/active/status to rank 0 over RCCL and time it")
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--family", choices=["box", "dense"], default="box")
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-procs", type=int, default=0, help="0 = this process's CPU share")
    ap.add_argument("--cpu-sample", type=int, default=4096)
    ap.add_argument("--ref-batch", type=int, default=65536, help="QPs for the GPU Newton/ADMM replica rows")
    ap.add_argument("--box-reps", type=int, default=10, help="timed qpb_solve_box calls on the same QPs (0: skip)")
    ap.add_argument("--dense-reps", type=int, default=10, help="timed qpb_solve calls on the dense family (0: skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--check", action="store_true", help="verify statuses after the timed region")
    ap.add_argument("--pipeline-streams", type=int, default=2,
                    help="after the timed steps, the same K batches alternating over this many HIP streams "
                         "(a serving loop: one batch's drain overlaps the next one's ramp-up), reported "
                         "beside the line's single-stream value (0 or 1: skip)")
    ap.add_argument("--settle-seconds", type=float, default=0.1,
                    help="before the warmup steps, back-to-back solves of the same batch for about this long: "
                         "after the CPU leg (or process start) the GPU is idle, and its first ~30 launches run "
                         "up to 10 %% slower while its clocks ramp (tools/warm_state.py); reported (0: skip)")
    ap.add_argument("--sustain-seconds", type=float, default=6.0,
                    help="after the timed steps, back-to-back solves of the same batch for about this long "
                         "(clock and thermal steady state), reported beside the line's value (0: skip)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(relaunch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)

    import torch
    # CPU baseline first: its worker processes are forked, which is only safe
    # before this process initialises the GPU.  The sample is the first
    # cpu_sample QPs of the GPU batch, restated on the CPU (oracle.family_generate).
    cpu, cpu_newton = None, None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.family == "box" and args.n == 16:
        procs = args.cpu_procs or cpu_share()
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle  # CPU restatement of qpb_generate: the first QPs of the GPU batch
        Hc, fc, _, _ = oracle.family_generate(args.n, args.cpu_sample, args.seed, "box")
        cpu, cpu_newton = cpu_baselines(Hc, fc, args.cpu_seconds, procs)
        del Hc, fc
    # one GPU per rank; QPB_DIST_BACKEND=gloo (with ranks sharing a card) rehearses
    # the N>1 path on a one-GPU box -- the driver's runs use RCCL ("nccl")
    backend = os.environ.get("QPB_DIST_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    import qpb
    from qpb.dist import check_gathered, gather_results, max_over_ranks, shard

    dist_info = None
    if world > 1:
        # which GPUs the ranks actually drive (RCCL must see N distinct devices)
        import torch.distributed as dist
        props = torch.cuda.get_device_properties(device)
        mine = {"rank": rank, "local_rank": local, "device": device.index,
                "pci_bus_id": getattr(props, "pci_bus_id", None), "uuid": str(getattr(props, "uuid", ""))}
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
        ids = [(r["pci_bus_id"], r["uuid"]) for r in ranks]
        dist_info = {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "ranks": ranks,
                     "distinct_devices": len(set(ids)) == world}
        if dist_info["backend"] == "nccl" and not dist_info["distinct_devices"]:
            raise SystemExit(f"bench.py: RCCL ranks share a GPU: {ranks}")

    n, m = args.n, 2 * args.n
    if args.batch:
        start, B = rank * args.batch, args.batch
        total_B = args.batch * world
    else:
        total_B = args.global_batch
        start, B = shard(total_B, rank, world)
    # rank r owns QP indices [start, start + B): the same QPs as that slice of
    # a one-GPU run (Philox keyed by the global QP index)
    H, f, A, b = qpb.generate(n, B, args.seed, family=args.family, first=start, shift=1.0, box=10.0, device=device)
    stream = torch.cuda.current_stream()
    sol = qpb.solve(H, f, A, b, stream=stream)  # allocate outputs once
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    # settle: the GPU out of its idle clocks before the warmup steps (every
    # rank, the same span, launch groups of 5 with a sync between groups)
    settle = None
    if args.settle_seconds > 0:
        barrier()
        tw, kw = time.perf_counter(), 0
        while time.perf_counter() - tw < args.settle_seconds:
            for _ in range(5):
                qpb.solve(H, f, A, b, out=sol, stream=stream)
            kw += 5
            torch.cuda.synchronize()
        settle = {"seconds": time.perf_counter() - tw, "launches": kw,
                  "what": "the line's solve back to back before the warmup steps: the GPU's first ~30 "
                          "launches after idle run up to 10 % slower while its clocks ramp "
                          "(tools/warm_state.py, profiles/r06/warm)"}
    for _ in range(args.warmup):
        qpb.solve(H, f, A, b, out=sol, stream=stream)
    # HIP events on the stream the kernel is launched on, one pair around the
    # K launches (a pair around every launch slowed them by ~0.4 %,
    # tools/event_overhead.py): the average launch duration, gaps included
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(args.steps):
        qpb.solve(H, f, A, b, out=sol, stream=stream)
    ev1.record(stream)
    barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    local_step_ms = elapsed / args.steps * 1e3
    elapsed = max_over_ranks(elapsed, device)
    if dist_info is not None:
        # per rank: its shard, its kernel time (HIP events on its launch stream)
        # and its own step time, beside the one-GPU kernel-time prediction for a
        # shard of that size (profiles/batch_scan.json): a speed-up short of N
        # then reads as the kernel's per-launch fixed cost, not communication
        mine = {"rank": rank, "shard_first": start, "shard_qps": B, "kernel_ms": kern_ms,
                "step_ms": local_step_ms}
        per = [None] * world
        dist.all_gather_object(per, mine)
        dist_info["per_rank"] = per
        pred = shard_time_prediction(n, m, args.family, B, total_B, qpb.version())
        if pred:
            dist_info["single_gpu_prediction"] = pred
    gather_ms, gather = None, None
    if args.gather and world > 1:  # the trivial result gather of SURVEY.md §8e, outside the timed steps
        barrier()
        tg = time.perf_counter()
        local = {"x": sol.x, "lam": sol.lam, "active": sol.active, "status": sol.status}
        full = gather_results(local, total_B)
        barrier()
        gather_ms = max_over_ranks((time.perf_counter() - tg) * 1e3, device)
        # every rank's exact shard digest against its rows of the gathered batch
        # (qpb.dist.check_gathered; after the timed gather), every status a valid code
        digests_ok = check_gathered(full, local, total_B)
        if rank == 0:
            checked = bool(full["x"].shape[0] == total_B and digests_ok
                           and ((full["status"] >= 0) & (full["status"] <= 4)).all())
            gather = {"dst": 0, "collective": "gather (x, lam, active, status) to rank 0",
                      "bytes_per_qp": 8 * (n + m) + 4 * ((m + 31) // 32) + 4, "checked": checked,
                      "check": "each rank's integer digest of its shard == the digest of its rows on rank 0"}
        del full

    # pipelined leg, outside the timed steps: K batches over S streams, each
    # stream with its own outputs; barrier + max over ranks as above.  The
    # line's value stays the single-stream one (one pass per step, in order).
    pipelined = None
    if args.pipeline_streams > 1:
        S = args.pipeline_streams
        pstreams = [torch.cuda.Stream(device=device) for _ in range(S)]
        psols = [qpb.solve(H, f, A, b, stream=ps) for ps in pstreams]
        barrier()
        tp = time.perf_counter()
        for k in range(args.steps):
            qpb.solve(H, f, A, b, out=psols[k % S], stream=pstreams[k % S])
        barrier()
        pel = max_over_ranks(time.perf_counter() - tp, device)
        same = all(torch.equal(ps.x, sol.x) and torch.equal(ps.status, sol.status) for ps in psols)
        pipelined = {"streams": S, "value": total_B * args.steps / pel, "ms_per_step": pel / args.steps * 1e3,
                     "answers_equal": bool(same),
                     "what": "the same K steps alternating over S HIP streams: a batch's drain (its last "
                             "waves finishing) overlaps the next batch's ramp-up (every wave slot loading)"}
        del psols

    # sustained leg, outside the timed steps: the same solve back to back for
    # about --sustain-seconds (launched 20 at a time, the host checking the
    # clock between groups), barrier + max over ranks as above
    sustained = None
    if args.sustain_seconds > 0:
        barrier()
        ts = time.perf_counter()
        ks = 0
        while True:
            for _ in range(20):
                qpb.solve(H, f, A, b, out=sol, stream=stream)
            ks += 20
            torch.cuda.synchronize()
            done = time.perf_counter() - ts >= args.sustain_seconds
            if world > 1:  # every rank stops after the same number of groups (all past the span)
                done = max_over_ranks(0.0 if done else 1.0, device) == 0.0
            if done:
                break
        barrier()
        sel = max_over_ranks(time.perf_counter() - ts, device)
        sustained = {"seconds": sel, "steps": ks, "value": total_B * ks / sel, "ms_per_step": sel / ks * 1e3,
                     "what": "the line's solve back to back for the whole span (launch groups of 20, a host "
                             "sync between groups): the rate once clocks and temperature have settled"}

    st = sol.status.cpu()
    it = sol.iters.cpu().double()
    ok_frac = float((st == 0).double().mean())
    if args.check:
        assert ok_frac == 1.0, torch.bincount(st.long())

    # like-for-like rows (N = 1): the reference's Newton and ADMM as GPU replicas
    like = None
    if rank == 0 and world == 1 and n == 16 and args.family == "box" and args.ref_batch > 0:
        Br = min(args.ref_batch, B)
        x0 = torch.zeros((Br, n), dtype=torch.float64, device=device)
        like = {"qps": Br, "inputs": "the first QPs of the bench batch (P = H, q = f), x0 = 0, ADMM box +-10"}
        for name, mode, iters in (("newton", qpb.REF_NEWTON, 10), ("admm", qpb.REF_ADMM, 10000)):
            qpb.ref_solve(mode, H[:Br], f[:Br], x0, iterations=iters, box=(-10.0, 10.0), stream=stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            qpb.ref_solve(mode, H[:Br], f[:Br], x0, iterations=iters, box=(-10.0, 10.0), stream=stream)
            e1.record(stream)
            torch.cuda.synchronize()
            gpu_rate = Br / (e0.elapsed_time(e1) * 1e-3)
            cpu_rate = (cpu or {}).get("value") if name == "admm" else cpu_newton
            like[name] = {"gpu_qps_per_s": gpu_rate, "cpu_reference_qps_per_s": cpu_rate,
                          "iterations_arg": iters,
                          "ratio": (gpu_rate / cpu_rate) if cpu_rate else None}
        if cpu:
            like["cpu_cores"] = cpu["cores"]

    # the box fast path (A = [I; -I] implicit, reported
    # separately): the same QPs through qpb_solve_box, outside the timed steps
    box = None
    if rank == 0 and world == 1 and n <= 16 and args.family == "box" and args.box_reps > 0:
        ub = b[:, :n].contiguous()
        lb = (-b[:, n:]).contiguous()
        bsol = qpb.solve_box(H, f, lb, ub, stream=stream)
        bev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.box_reps)]
        torch.cuda.synchronize()
        for e0, e1 in bev:
            e0.record(stream)
            qpb.solve_box(H, f, lb, ub, out=bsol, stream=stream)
            e1.record(stream)
        torch.cuda.synchronize()
        box_ms = sum(a.elapsed_time(e) for a, e in bev) / len(bev)
        bbytes = 8 * (n * n + 3 * n) + 8 * 3 * n + 4 + 4  # H, f, lb, ub in; x, lam (2n), mask, status out
        box = {"api": "qpb_solve_box (lb <= x <= ub, A = [I; -I] implicit)", "qps_per_s": B / (box_ms * 1e-3),
               "kernel_ms": box_ms, "bytes_per_qp": bbytes,
               "hbm_frac": B * bbytes / (box_ms * 1e-3) / (HBM_PEAK_GBS * 1e9),
               "same_active_set_as_dense": bool(torch.equal(bsol.active, sol.active)),
               "ok_frac": float((bsol.status == 0).double().mean())}
        del bsol

    # the dense family (random normalised A rows) at the same
    # batch: the same kernel on QPs whose constraints are not a box in disguise
    dense = None
    if rank == 0 and world == 1 and n <= 16 and args.family == "box" and args.dense_reps > 0:
        Hd, fd, Ad, bd = qpb.generate(n, B, args.seed, family="dense", shift=1.0, box=10.0, device=device)
        dsol = qpb.solve(Hd, fd, Ad, bd, stream=stream)
        dev_ = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                for _ in range(args.dense_reps)]
        torch.cuda.synchronize()
        for e0, e1 in dev_:
            e0.record(stream)
            qpb.solve(Hd, fd, Ad, bd, out=dsol, stream=stream)
            e1.record(stream)
        torch.cuda.synchronize()
        dense_ms = sum(a.elapsed_time(e) for a, e in dev_) / len(dev_)
        dbytes = bytes_per_qp(n, m)
        dit = dsol.iters.double()
        dense = {"family": "dense (A rows ~ N(0, I) normalised, b ~ U[0.1, 1) * 10)", "qps_per_s": B / (dense_ms * 1e-3),
                 "kernel_ms": dense_ms, "bytes_per_qp": dbytes,
                 "hbm_frac": B * dbytes / (dense_ms * 1e-3) / (HBM_PEAK_GBS * 1e9),
                 "ok_frac": float((dsol.status == 0).double().mean()), "iters_mean": float(dit.mean()),
                 "iters_max": int(dit.max())}
        del Hd, fd, Ad, bd, dsol

    total_qps = total_B * args.steps
    value = total_qps / elapsed
    if pipelined:
        pipelined["gain"] = pipelined["value"] / value - 1.0
    if sustained:
        sustained["ratio_to_value"] = sustained["value"] / value
    bpq = bytes_per_qp(n, m)
    achieved = B * bpq / (kern_ms * 1e-3) / 1e9
    traffic = pmc_traffic(n, m, B, args.family, qpb.version())

    if rank == 0:
        line = {
            "metric": (BASELINE_METRIC if (n, m) == (16, 32) else f"QPs/sec (whole node) at n={n},m={m}; % HBM roofline"),
            "value": value,
            "unit": "QPs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if args.batch else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic: qpb_generate on the GPU (Philox keyed by QP index, seed {args.seed}), "
                    f"conditioned {args.family} family of SURVEY.md §8d",
            "config": {"workload": f"batched active-set QP solve, n={n}, m={m} "
                                   f"({'box as dense A=[I;-I]' if args.family == 'box' else 'dense random A'}), "
                                   f"{total_B} QPs in total, {B} per GPU ({baseline_config(n, total_B, world)})",
                       "n": n, "m": m, "batch_per_gpu": B, "global_batch": total_B,
                       "family": args.family, "parallelism": f"qp-shard x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic["bytes"] if traffic else None,
                         "traffic_source": traffic["source"] if traffic else None,
                         "kernel": ("qpb::gi_dense_kernel" if n <= 16 and m <= 32
                                    else "qpb::wv::gi_wave_kernel" if n <= 32 and m <= 64
                                    else "qpb::gram::gi_gram_kernel"), "bytes_per_qp": bpq,
                         "bytes_per_launch": B * bpq, "kernel_ms": kern_ms},
            "valu_ceiling": valu_ceiling(traffic, (B + 3) // 4 if n <= 16 and m <= 32 else B, kern_ms),
            "cpu_baseline": cpu,
            "like_for_like": like,
            "box_fast_path": box,
            "solver_stats": {"ok_frac": ok_frac, "iters_mean": float(it.mean()), "iters_max": int(it.max())},
            "gather_ms": gather_ms,
            "gather": gather,
            "dense_family": dense,
            "pipelined": pipelined,
            "settle": settle,
            "sustained": sustained,
            "distributed": dist_info,
            "library": qpb.version(),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
