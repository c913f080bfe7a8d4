"""Multi-process path on the GPU: the qpb solve under QP-index sharding.

Two ranks (gloo; both on the box's one card -- the driver's 8-GPU runs use
RCCL, one card per rank) each generate their shard with qpb_generate (keyed by
the global QP index), solve it with qpb_solve through the C-ABI and all-gather
the results.  The gathered batch must equal the single-process solve of the
whole batch bit for bit.  Then bench.py --gpus 2 must run two ranks and report
n_gpus = 2 (it relaunches itself under torch.distributed.run).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, total, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import qpb
    from qpb.dist import gather_results, shard
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    start, count = shard(total, rank, world)
    H, f, A, b = qpb.generate(16, count, 99, family="dense", first=start, device=dev)
    sol = qpb.solve(H, f, A, b)
    torch.cuda.synchronize()
    local = {k: getattr(sol, k).cpu() for k in ("x", "lam", "active", "status")}
    full = gather_results(local, total)
    if rank == 0:
        torch.save({k: v for k, v in full.items()}, os.path.join(out_dir, "gathered.pt"))
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def qpb():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
    import qpb as q
    return q


@pytest.mark.parametrize("total", [4097, 20000])
def test_two_rank_qpb_shards_equal_one_batch(qpb, tmp_path, total):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(2, _port(), total, str(tmp_path)), nprocs=2, join=True)
    got = torch.load(os.path.join(tmp_path, "gathered.pt"), weights_only=True)
    H, f, A, b = qpb.generate(16, total, 99, family="dense", first=0)
    sol = qpb.solve(H, f, A, b)
    torch.cuda.synchronize()
    for k in ("x", "lam", "active", "status"):
        assert torch.equal(got[k], getattr(sol, k).cpu()), k
    assert (got["status"] == qpb.OK).all()


def test_bench_gpus_2_runs_two_ranks(qpb):
    """The N > 1 path SCALE uses (bench.py relaunching itself under
    torch.distributed.run), with the result gather to rank 0 (--gather) and
    the self-describing `distributed` block."""
    env = dict(os.environ, QPB_DIST_BACKEND="gloo")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--global-batch", "8192",
           "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--gather", "--sustain-seconds", "0.5"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2
    assert line["config"]["global_batch"] == 8192
    assert line["config"]["batch_per_gpu"] == 4096
    assert line["solver_stats"]["ok_frac"] == 1.0
    d = line["distributed"]
    assert d["world_size"] == 2 and d["backend"] == "gloo"
    assert sorted(x["rank"] for x in d["ranks"]) == [0, 1]
    assert line["gather_ms"] is not None and line["gather_ms"] >= 0.0
    assert line["gather"]["checked"] is True
    # per rank: its shard, its own kernel time (HIP events) and step time, and
    # the one-GPU prediction for a launch of that shard size
    per = sorted(d["per_rank"], key=lambda x: x["rank"])
    assert [(x["shard_first"], x["shard_qps"]) for x in per] == [(0, 4096), (4096, 4096)]
    assert all(x["kernel_ms"] > 0.0 and x["step_ms"] >= x["kernel_ms"] * 0.5 for x in per)
    pred = d["single_gpu_prediction"]
    assert pred["shard_kernel_ms"] > 0.0 and pred["total_kernel_ms"] > pred["shard_kernel_ms"]
    assert 1.0 < pred["kernel_bound_speedup"] <= 2.0
    # the pipelined leg (two streams per rank, max over ranks) gives the same answers
    pl = line["pipelined"]
    assert pl["streams"] == 2 and pl["answers_equal"] is True and pl["value"] > 0.0
    # the sustained leg: both ranks stop after the same launch groups, past the span
    su = line["sustained"]
    assert su["steps"] >= 20 and su["steps"] % 20 == 0 and su["seconds"] >= 0.5 and su["value"] > 0.0


def _rccl_worker(rank, port, total, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    import qpb
    from qpb.dist import gather_results
    H, f, A, b = qpb.generate(16, total, 99, family="dense", first=0, device=dev)
    sol = qpb.solve(H, f, A, b)
    full = gather_results({k: getattr(sol, k) for k in ("x", "lam", "active", "status")}, total, dst=0)
    t = torch.tensor([1.5, -2.0], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.barrier()
    torch.cuda.synchronize()
    torch.save({"backend": dist.get_backend(), "reduced": t.cpu(), "device": str(full["x"].device),
                **{k: v.cpu() for k, v in full.items()}}, os.path.join(out_dir, "rccl.pt"))
    dist.destroy_process_group()


def test_rccl_gather_and_reduce_one_rank(qpb, tmp_path):
    """The RCCL ("nccl" backend) code path of the multi-GPU line on this box's
    one GPU: process-group init with device_id, qpb.dist.gather_results
    (dist.gather of device tensors to rank 0), an all_reduce and a barrier,
    as bench.py --gpus N --gather runs them per rank.  One rank: the box has
    one card, and RCCL refuses two ranks on one device (bench.py checks
    distinct devices).  The gathered batch equals the direct solve."""
    import torch.multiprocessing as mp
    total = 4096
    mp.spawn(_rccl_worker, args=(_port(), total, str(tmp_path)), nprocs=1, join=True)
    got = torch.load(os.path.join(tmp_path, "rccl.pt"), weights_only=True)
    assert got["backend"] == "nccl"
    assert got["device"].startswith("cuda")
    assert torch.equal(got["reduced"], torch.tensor([1.5, -2.0], dtype=torch.float64))
    H, f, A, b = qpb.generate(16, total, 99, family="dense", first=0)
    sol = qpb.solve(H, f, A, b)
    torch.cuda.synchronize()
    for k in ("x", "lam", "active", "status"):
        assert torch.equal(got[k], getattr(sol, k).cpu()), k
