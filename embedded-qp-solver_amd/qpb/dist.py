"""qpb.dist -- multi-GPU sharding of a QP batch.

One process per GPU (torchrun).  Every QP is independent, so the batch is
split into contiguous index ranges, one per rank, and each rank solves its
range with no communication.  The only collective is the optional final
result gather over RCCL/xGMI (backend "nccl" = RCCL on ROCm; "gloo" on CPU
for tests): x, lam, active words and status of every rank to rank 0 (or, on
request, to every rank).
"""
from __future__ import annotations


def shard(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [start, start + count) of `total` QPs for `rank`; the first
    total % world ranks take one extra QP."""
    if world < 1 or not 0 <= rank < world or total < 0:
        raise ValueError("bad shard arguments")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def max_over_ranks(value: float, device=None) -> float:
    """Max of a per-rank scalar (bench timing: the slowest rank defines the step)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    # RCCL reduces device tensors; gloo (CPU rehearsals) host tensors
    dev = device if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_results(local: dict, total: int, dst: int | None = 0):
    """Gather per-rank result shards (dict of tensors with a leading batch
    dimension, contiguous shards in rank order) into full-batch tensors.

    dst = rank r (default 0, SURVEY.md §8e's gather to one GPU): rank r gets
    the full batch, every other rank None -- (world - 1) shards cross the
    links once.  dst = None: an all-gather, the full batch on every rank
    (world x the traffic).  Shards may differ in length by one QP (see
    shard()); they travel padded to the longest and are trimmed here."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    rank = dist.get_rank()
    counts = [shard(total, r, world)[1] for r in range(world)]
    maxc = max(counts)
    out = {}
    for key, t in local.items():
        if t.shape[0] != counts[rank]:
            raise ValueError(f"gather_results: {key} has {t.shape[0]} rows, rank {rank}'s shard is {counts[rank]}")
        pad = torch.zeros((maxc,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[: t.shape[0]] = t
        if dst is None:
            parts = [torch.empty_like(pad) for _ in range(world)]
            dist.all_gather(parts, pad)
        else:
            parts = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
            dist.gather(pad, parts, dst=dst)
        out[key] = torch.cat([p[:c] for p, c in zip(parts, counts)], 0) if parts is not None else None
    return out if (dst is None or rank == dst) else None


def shard_digest(local: dict) -> dict:
    """Exact, summation-order-independent digest of a result shard (dict of
    tensors with a leading batch dimension): per tensor, the integer sums of
    the low and high 32 bits of every element's bit pattern and a
    position-weighted sum of its low 16 bits (weights (i mod 65521) + 1), so a
    corrupted, missing or misplaced element changes it.  Integer sums do not
    depend on the reduction order, so a shard and the same rows of a gathered
    batch give equal digests whatever their alignment."""
    import torch
    out = {}
    for key, t in local.items():
        v = t.contiguous().reshape(-1)
        if v.element_size() == 8:
            v = v.view(torch.int64)
        else:
            v = v.view(torch.int32).to(torch.int64)
        lo, hi = v & 0xFFFFFFFF, (v >> 32) & 0xFFFFFFFF
        w = torch.arange(v.numel(), device=v.device, dtype=torch.int64) % 65521 + 1
        out[key] = (int(lo.sum()), int(hi.sum()), int(((v & 0xFFFF) * w).sum()), int(v.numel()))
    return out


def check_gathered(full: dict, local: dict, total: int) -> bool:
    """Every rank's shard digest equals the digest of its rows of the batch
    gathered to rank 0 (`full`, None on the other ranks).  Collective: every
    rank calls it; the answer is meaningful on the rank that holds `full`."""
    import torch.distributed as dist
    world = dist.get_world_size()
    mine = shard_digest(local)
    every = [None] * world
    dist.all_gather_object(every, mine)
    if full is None:
        return True
    for r, d in enumerate(every):
        start, count = shard(total, r, world)
        if d != shard_digest({k: full[k][start:start + count] for k in local}):
            return False
    return True
