"""Multi-process (world size 2, gloo on CPU) tests of the sharding path used
by bench.py / qpb.dist: contiguous QP shards, max-over-ranks timing and the
final result gather reproduce the single-process batch exactly."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
from qpb.dist import shard  # noqa: E402


def test_shard_covers_batch_exactly():
    for total in (0, 1, 7, 65536, 1048576, 1000003):
        for world in (1, 2, 3, 8):
            ranges = [shard(total, r, world) for r in range(world)]
            assert ranges[0][0] == 0
            for (s0, c0), (s1, _) in zip(ranges, ranges[1:]):
                assert s0 + c0 == s1
            assert sum(c for _, c in ranges) == total
            assert max(c for _, c in ranges) - min(c for _, c in ranges) <= 1


def _worker(rank, world, port, total, ret):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from qpb.dist import gather_results, max_over_ranks, shard as sh
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    start, count = sh(total, rank, world)
    # the rank's shard of one global problem set (generated globally, sliced)
    H, f, A, b = O.family_conditioned(123, total, 4, box=2.0)
    xs, lam, st = [], [], []
    for i in range(start, start + count):
        r = O.active_set_solve(H[i], f[i], A[i], b[i])
        xs.append(r.x), lam.append(r.lam), st.append(r.status)
    local = {"x": torch.tensor(np.array(xs).reshape(count, 4)), "lam": torch.tensor(np.array(lam).reshape(count, 8)),
             "status": torch.tensor(np.array(st, dtype=np.int32))}
    full = gather_results(local, total)  # to rank 0
    every = gather_results(local, total, dst=None)  # all-gather
    t = max_over_ranks(float(rank + 1))
    assert (full is None) == (rank != 0)
    for k, v in every.items():
        ret[f"every_{rank}_{k}"] = v.numpy()
    if rank == 0:
        ret["x"] = full["x"].numpy()
        ret["lam"] = full["lam"].numpy()
        ret["status"] = full["status"].numpy()
        ret["tmax"] = t
    dist.destroy_process_group()


@pytest.mark.parametrize("total", [9, 16])
def test_two_rank_shard_solve_gather(total):
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(2, port, total, ret), nprocs=2, join=True)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    H, f, A, b = O.family_conditioned(123, total, 4, box=2.0)
    ref = np.array([O.active_set_solve(H[i], f[i], A[i], b[i]).x for i in range(total)])
    assert np.array_equal(ret["x"], ref)
    assert (ret["status"] == 0).all()
    assert ret["tmax"] == 2.0
    for r in range(2):  # the all-gather form gives every rank the same batch
        assert np.array_equal(ret[f"every_{r}_x"], ref)
        assert np.array_equal(ret[f"every_{r}_lam"], ret["lam"])


def _digest_worker(rank, world, port, ret):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from qpb.dist import check_gathered, gather_results, shard as sh
    total = 11
    start, count = sh(total, rank, world)
    g = torch.Generator().manual_seed(7)
    X = torch.randn(total, 4, generator=g, dtype=torch.float64)
    S = torch.arange(total, dtype=torch.int32)
    local = {"x": X[start:start + count].clone(), "status": S[start:start + count].clone()}
    full = gather_results(local, total)
    ret[f"ok_{rank}"] = check_gathered(full, local, total)
    # rank 0 corrupts one element of rank 1's rows, then swaps two of its own rows
    if rank == 0:
        full["x"].view(torch.int64)[start + count, 2] ^= 1  # the lowest mantissa bit
    ret[f"bad_{rank}"] = check_gathered(full, local, total)
    if rank == 0:
        full["x"].view(torch.int64)[start + count, 2] ^= 1
        full["x"][[0, 1]] = full["x"][[1, 0]]
    ret[f"swap_{rank}"] = check_gathered(full, local, total)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_check_digests_catch_corruption_and_misplacement(world):
    """qpb.dist.check_gathered (bench.py --gather's check): every rank's exact
    integer digest of its shard against its rows of the batch gathered to rank
    0 -- equal for a correct gather, unequal for one flipped low bit in another
    rank's rows and for two swapped rows."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_digest_worker, args=(world, port, ret), nprocs=world, join=True)
    assert all(ret[f"ok_{r}"] is True for r in range(world))  # 11 QPs: uneven shards
    assert ret["bad_0"] is False and all(ret[f"bad_{r}"] is True for r in range(1, world))  # only rank 0 holds the batch
    assert ret["swap_0"] is False
