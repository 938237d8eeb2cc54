"""Multi-GPU sharding of a chunk list.

Chunks are independent SHA-1 messages, so N GPUs split the chunk list into
N contiguous slices and hash them with no data-path collective (no RCCL
traffic, xGMI unused by design).  The only cross-rank operations are the
control-plane ones a benchmark or service needs: a barrier, the max of the
per-rank times, and the AND of the per-rank parity flags.

Used by bench.py (one process per GPU, torch.distributed over RCCL) and
covered on CPU by tests/test_distributed.py (gloo, world sizes 2 and 8).
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


def weak_golden_shard(rank: int, per_rank: int, total: int) -> tuple[int, int, int | None]:
    """Weak scaling over the ids of a fixed list of `total` chunks whose
    k-way strong shards have golden aggregates (bench.py's config-4 weak leg:
    65536 chunks per rank = one shard of the 4-way split of 262144): rank r
    takes shard r mod k, k = total / per_rank, so every rank's bytes have a
    reference digest-of-digests at any N.  Returns (first, count, shard
    index), or the plain weak shard and None when per_rank does not divide
    total."""
    if per_rank <= 0 or total % per_rank:
        return weak_shard(rank, per_rank) + (None,)
    k = total // per_rank
    first, count = strong_shard(rank % k, k, total)
    return first, count, rank % k


def strong_golden_agg(golden: dict, world: int, rank: int, total: int) -> str | None:
    """The reference golden digest-of-digests of rank `rank`'s strong shard
    (bench.py's `strong` leg): config 4's `world`-way split when the list is
    config 4's whole list, else None (no golden for that shape)."""
    c4 = golden["config4"]
    if total != c4["chunks"]:
        return None
    aggs = c4["shard_aggs"].get(str(world))
    return aggs[rank] if aggs is not None and 0 <= rank < len(aggs) else None


def weak_golden_agg(golden: dict, rank: int, per_rank: int) -> tuple[int, int, str | None]:
    """bench.py's `weak_config4` leg: rank `rank`'s chunk range
    (weak_golden_shard over config 4's list) and the golden aggregate of that
    range, None when per_rank does not divide the list."""
    c4 = golden["config4"]
    first, count, k_idx = weak_golden_shard(rank, per_rank, c4["chunks"])
    if k_idx is None:
        return first, count, None
    aggs = c4["shard_aggs"].get(str(c4["chunks"] // per_rank))
    return first, count, aggs[k_idx] if aggs is not None else None


def strong_report(total: int, chunk_len: int, world: int, ms_n: float, kern_ms_n: float,
                  ms_1: float, kern_ms_1: float, parity: bool, parity_1: bool,
                  steps: int) -> dict:
    """The `strong` object of bench.py's JSON line: `total` chunks split over
    `world` GPUs took ms_n per step (max over ranks), the whole list on one
    GPU ms_1.  GiB/s counts every chunk byte of the list; speed-up and
    efficiency are against the one-GPU time."""
    speedup = ms_1 / ms_n if ms_n > 0 else 0.0
    return {
        "workload": f"BASELINE config 4: {total} x {chunk_len} B chunks split over {world} GPU(s), "
                    "device-resident",
        "chunks_total": total, "chunks_per_gpu": -(-total // world) if world else total,
        "n_gpus": world, "steps": steps,
        "ms_per_step": round(ms_n, 4), "kernel_ms": round(kern_ms_n, 4),
        "value": round(total * chunk_len / (ms_n * 1e-3) / 2**30, 3) if ms_n > 0 else 0.0,
        "unit": "GiB/s",
        "one_gpu_ms_per_step": round(ms_1, 4), "one_gpu_kernel_ms": round(kern_ms_1, 4),
        "speedup": round(speedup, 4), "efficiency": round(speedup / world, 4) if world else 0.0,
        "parity": bool(parity), "one_gpu_parity": bool(parity_1),
        "scaling": "strong",
    }


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


class DeviceMapError(RuntimeError):
    """A multi-rank run would put two ranks on one GPU (or a rank on none)."""


def device_for_local_rank(local_rank: int, local_world: int, device_count: int,
                          shared_ok: bool = False) -> int:
    """The GPU of local rank `local_rank`: one process per GPU, rank r on
    device r.  A node that exposes fewer devices than it runs local ranks
    would stack ranks onto shared GPUs and time a plausible but wrong curve,
    so that raises -- unless `shared_ok` (the gloo rehearsal of several ranks
    on one card, SHA1_BENCH_DIST_BACKEND=gloo), which maps round robin."""
    if device_count <= 0:
        raise DeviceMapError("no GPU visible to this rank")
    if local_world > device_count and not shared_ok:
        raise DeviceMapError(
            f"{local_world} local ranks but only {device_count} visible GPU(s): one rank per GPU "
            "is required (set HIP_VISIBLE_DEVICES / --nproc-per-node to match)")
    if local_rank < 0 or (local_rank >= device_count and not shared_ok):
        raise DeviceMapError(f"local rank {local_rank} has no GPU of its own ({device_count} visible)")
    return local_rank % device_count


def device_identity(host: str, rank: int, local_rank: int, ordinal: int, props) -> dict:
    """What a rank records about its GPU (bench.py gathers these on rank 0):
    the ordinal and the physical identity (PCI domain:bus:device and UUID)."""
    pci = None
    if props is not None and hasattr(props, "pci_bus_id"):
        pci = "%04x:%02x:%02x" % (getattr(props, "pci_domain_id", 0), props.pci_bus_id,
                                  getattr(props, "pci_device_id", 0))
    uuid = str(getattr(props, "uuid", "")) if props is not None else ""
    return {"rank": rank, "host": host, "local_rank": local_rank, "device": ordinal,
            "pci": pci, "uuid": uuid}


def check_distinct_devices(identities: list[dict], shared_ok: bool = False) -> None:
    """Raise when two ranks on one host share a physical GPU (same UUID, or
    same PCI address where no UUID is reported)."""
    if shared_ok:
        return
    seen: dict = {}
    for ident in identities:
        phys = ident.get("uuid") or ident.get("pci") or f"ordinal {ident.get('device')}"
        key = (ident.get("host"), phys)
        if key in seen:
            raise DeviceMapError(f"ranks {seen[key]} and {ident.get('rank')} share GPU {phys} on "
                                 f"{ident.get('host')}: a scaling run needs one GPU per rank")
        seen[key] = ident.get("rank")


def gather_identities(ident: dict) -> list[dict]:
    """Every rank's identity, in rank order (just this one without a group)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [ident]
    out: list = [None] * dist.get_world_size()
    dist.all_gather_object(out, ident)
    return out


def max_over_ranks(values, device=None) -> list[float]:
    """Element-wise max over ranks (identity without an initialised group;
    with one, the all_reduce runs even at world size 1)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [float(v) for v in values]
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.tolist()]


def all_ranks_ok(flag: bool, device=None) -> bool:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return bool(flag)
    t = torch.tensor([1.0 if flag else 0.0], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item() > 0.5)
