"""Multi-GPU sharding of a chunk list.

Chunks are independent SHA-1 messages, so N GPUs split the chunk list into
N contiguous slices and hash them with no data-path collective (no RCCL
traffic, xGMI unused by design).  The only cross-rank operations are the
control-plane ones a benchmark or service needs: a barrier, the max of the
per-rank times, and the AND of the per-rank parity flags.

Used by bench.py (one process per GPU, torch.distributed over RCCL) and
covered on CPU by tests/test_distributed.py (gloo, world size 2).
"""
from __future__ import annotations


def weak_shard(rank: int, per_rank: int) -> tuple[int, int]:
    """Weak scaling: every rank hashes its own `per_rank` chunks (global
    chunk ids rank*per_rank ..), so per-GPU work is fixed as N grows."""
    return rank * per_rank, per_rank


def strong_shard(rank: int, world: int, total: int) -> tuple[int, int]:
    """Strong scaling: a fixed list of `total` chunks split into `world`
    contiguous slices whose sizes differ by at most one chunk."""
    base, extra = divmod(total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def byte_balanced_cuts(lengths, world: int) -> list[int]:
    """Cut points (len world+1) splitting a ragged chunk list into contiguous
    slices of near-equal byte counts (what SHA1CHUNK_ALL_DEVICES does in
    sha1_runtime.hip for host batches)."""
    total = sum(int(x) for x in lengths)
    cuts = [0]
    acc, d = 0, 1
    for i, L in enumerate(lengths):
        acc += int(L)
        while d < world and acc * world >= total * d:
            cuts.append(i + 1)
            d += 1
    while len(cuts) < world:
        cuts.append(len(lengths))
    cuts.append(len(lengths))
    return cuts


def max_over_ranks(values, device=None) -> list[float]:
    """Element-wise max over ranks (identity without an initialised group)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [float(v) for v in values]
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.tolist()]


def all_ranks_ok(flag: bool, device=None) -> bool:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return bool(flag)
    t = torch.tensor([1.0 if flag else 0.0], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item() > 0.5)
