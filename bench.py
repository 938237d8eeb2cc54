#!/usr/bin/env python3
"""Benchmark: device-resident SHA-1 over 512 KiB chunks (BASELINE.json metric).

One step = one pass of the hot path (SHA1Guts over every block of every
chunk, sha.c:176-451, as shahash does per chunk, chunk.c:35-51) over one
batch of synthetic chunks already resident in HBM.  Default workload =
BASELINE config 2: 4096 x 524288 B per GPU.  Multi-GPU (torchrun, one rank
per GPU): every rank hashes its own 4096 chunks (global chunk ids
4096*rank ..), no data-path collective -> weak scaling; the only
collectives are the timing barrier and the max-over-ranks reduction.

Prints ONE JSON line on rank 0 with `roofline` (dominant kernel vs the HBM
peak, per-launch time from HIP events on the kernel's own stream; `traffic`
from the committed rocprofv3 PMC pass, profiles/traffic_*.json),
`binding_limit` (the limit that actually binds the workload's regime: at
<= 2 groups of 64 chunks per CU one chunk's serial instruction stream --
SHA-1 is serial inside a chunk and one wave issues one instruction per 4
cycles, so config 2's 4096 chunks = 64 waves cannot fill 1024 SIMDs -- and
beyond that the SIMDs' VALU time), `valu_ceiling` (the
chip's SHA-1 VALU ceiling in the roofline's GB/s) and `cpu_baseline` (the
reference sha.c, compiled from its sources into oracle/_ref, timed on this
host's cores on the same chunks).

--streams P (default 1) keeps P independent batches in flight on P HIP
streams (each its own 4096 distinct chunks); the default measures one batch
at a time.

`strong` (same JSON line): BASELINE config 4 -- the fixed list of 262144 x
512 KiB chunks split into N contiguous shards, one per rank (shard.strong_shard,
no collective) -- timed like the main leg (barrier + synchronize around K
steps, max over ranks), with its speed-up and efficiency against the one-GPU
time of the whole 262144-chunk list, measured on rank 0's GPU in the same run
(at N = 1 the shard is the whole list).  Parity: every rank's digest-of-digests
against the reference golden shard aggregate of the N-way split.
`value` stays the weak config-2 number, so the N = 1 line is BENCH's.

`weak_config4` (same line): config 4's weak scaling, 65536 chunks per GPU
(SURVEY.md 8d), rank r hashing shard r mod 4 of the 4-way split of the
config-4 list (shard.weak_golden_shard), checked against that shard's golden
aggregate; timed like `strong`.

`file` (N = 1): SURVEY 8f rank 1, make-chunks on a real file -- chunks
0..16383 of the config-3 corpus (8 GiB) written to a temp file, hashed by
make_chunks in-process (sha1chunk_hash_fd) and by the repo's make-chunks CLI;
all 16384 digests checked against the reference golden aggregates.
`master_verify` (N = 1): SURVEY 8f rank 3, 1000 verify_chunk_hash GETs at
seeded random indices of that file (packet_handler.c:434 -> chunk.c:204-217),
master index against the per-call path; the reference chunk.c's per-call
cost is timed in cpu_baseline.

`latency_one_chunk` (N = 1): the peer's synchronous receive-side verify,
verify_hash() (job.c:217-228) on one 512 KiB chunk through the library, in a
child process: cold (first call, HIP start-up included) and warm, next to the
reference sha.c -O2 on one host core (cpu_baseline leg).
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import importlib
import json
import os
import socket
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s device-resident SHA-1 over 512KB chunks; % of HBM-read roofline"
CHUNK_LEN = 524288  # constants.h:14
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
# Issue-floor models of the kernels.  Instruction
# counts per 64-B block of each kernel's steady-state loop, read from the
# compiled gfx950 ISA by tools/isa_mix.py (profiles/isa_mix_r02.json):
#  * split kernel (<= 2 groups of 64 chunks per CU): the rounds-only consumer
#    wave issues CONSUMER_INSTR_PER_BLOCK instructions per block (400 round
#    VALU + 20 ds_read_b128 of the schedule + 5 feed-forward adds + scalars),
#    and one wave issues one instruction per 4.0 cycles (straight-line
#    streams: tools/issue_probe.hip -> profiles/issue_r01.json; the
#    "vector-instruction ISSUE cost" row of MI355X_MICROARCH.md).  The floor
#    is one chunk's serial chain: blocks x instructions x 4 cycles.
#  * fused kernel (more groups): the SIMD's VALU time.  The fused loop issues
#    613.75 VALU per block per wave of 64 chunks (621.75 before round 4's
#    fresh-register byte swap), and a SIMD completes about
#    one VALU instruction every 4 cycles whatever its class: the PMC passes at
#    131072 chunks (2 waves per SIMD) give 4.17 cycles per VALU per SIMD at the
#    clock the chip holds, and 4 waves per SIMD take the same time per wave
#    (profiles/pmc_shape_r03.json).  The round-2 model
#    of 2 cycles for the "full-rate" ops (2043.5 cycles per block) is not
#    reached by any kernel or microbenchmark here, so the ceiling below uses
#    4 cycles per VALU: 2455 SIMD cycles per wave-block.
# Measured counterpart: the same compression on register data with no
# memory traffic, every SIMD holding 8 waves, reaches 3940 GB/s of message
# bytes (tools/microbench.hip compress_test "512 x 1024",
# profiles/microbench_issue_r01.json), 97 % of this ceiling at 2.4 GHz.
COMPRESS_ONLY_GBS = 3939.8
CONSUMER_INSTR_PER_BLOCK = 427.75
ROUND_VALU_PER_BLOCK = 400
FUSED_VALU_PER_BLOCK = 613.75  # tools/isa_mix.py, profiles/fused_vmov_r04.json
FUSED_SIMD_CYCLES_PER_BLOCK = FUSED_VALU_PER_BLOCK * 4.0
ISSUE_CYCLES = 4.0
CLOCK_HZ = 2.4e9  # MI355X max engine clock; the chip holds it at config-2 occupancy
SIMDS_PER_CU = 4
NAMED_WORKLOADS = {4096: "BASELINE config 2", 32768: "config 4 shard, 1 of 8 GPUs",
                   65536: "config 3 size, device-resident", 262144: "config 4 whole, one GPU"}


def _regime(n: int, cus: int, kernel: str) -> str:
    """The kernel `kernel` (or AUTO's choice, sha1_runtime.hip choose_kernel /
    split_unit) for n chunks on `cus` CUs, honouring the same A/B overrides
    the library reads (SHA1CHUNK_FORCE_KERNEL behind AUTO,
    SHA1CHUNK_SPLIT_UNIT for the split shape)."""
    groups = (n + 63) // 64
    if kernel == "auto":
        forced = os.environ.get("SHA1CHUNK_FORCE_KERNEL")
        if forced in ("lane", "fused", "split"):
            kernel = forced
        else:
            kernel = "split" if groups <= 2 * cus else "fused"
    if kernel == "split":
        unit = os.environ.get("SHA1CHUNK_SPLIT_UNIT")
        if unit is None:
            unit = "4" if groups <= cus else ("11" if groups <= 2 * cus else "1")
        return {"4": "split_u4_2prod", "11": "split_u2_8wave", "1": "split_u1"}.get(
            unit.strip(), f"split_unit{unit.strip()}")
    return kernel


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--chunks", type=int, default=4096, help="chunks per GPU")
    ap.add_argument("--chunk-len", type=int, default=524288)
    ap.add_argument("--kernel", default="auto", choices=["auto", "lane", "fused", "split"])
    ap.add_argument("--streams", type=int, default=1, help="independent batches in flight")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="cap on the all-cores CPU-baseline rows (0 = every usable core)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--strong-total", type=int, default=262144,
                    help="chunks of the strong-scaling list (BASELINE config 4); 0 = skip")
    ap.add_argument("--strong-steps", type=int, default=10)
    ap.add_argument("--weak4-chunks", type=int, default=65536,
                    help="chunks per GPU of the config-4 weak-scaling leg (SURVEY.md 8d); 0 = skip")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the config 1 / 3 / 5, file and master-verify legs (N = 1 only)")
    ap.add_argument("--file-chunks", type=int, default=16384,
                    help="512 KiB chunks of the file / master_verify legs' temp file (0 = skip)")
    return ap.parse_args()


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    # RCCL carries only the control plane (barrier, max time, parity AND);
    # SHA1_BENCH_DIST_BACKEND=gloo rehearses several ranks on one GPU.
    backend = os.environ.get("SHA1_BENCH_DIST_BACKEND", "nccl")
    cdev = "cuda" if backend == "nccl" else "cpu"
    shared_ok = backend != "nccl"  # only the gloo rehearsal may stack ranks on one card
    shard = importlib.import_module("congestion-control-with-bittorren_amd.shard")
    # one rank per GPU: a node exposing fewer GPUs than local ranks fails
    # here instead of timing ranks stacked on shared devices
    try:
        dev = shard.device_for_local_rank(local, local_world, torch.cuda.device_count(), shared_ok)
    except shard.DeviceMapError as e:
        print(f"bench.py rank {rank}: {e}", file=sys.stderr, flush=True)
        sys.exit(2)
    # SHA1_BENCH_FORCE_PG=1 (under torchrun): a process group even at N = 1,
    # so a one-GPU box runs the RCCL control plane (init with device_id,
    # barrier, all_reduce MAX/MIN) that an 8-GPU node runs
    use_pg = world > 1 or os.environ.get("SHA1_BENCH_FORCE_PG") == "1"
    if use_pg:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(dev)
    # every rank's physical GPU, gathered on every rank: two ranks on one
    # host sharing a GPU end the run (exit 2) on all ranks
    idents = shard.gather_identities(shard.device_identity(
        socket.gethostname(), rank, local, dev, torch.cuda.get_device_properties(dev)))
    try:
        shard.check_distinct_devices(idents, shared_ok)
    except shard.DeviceMapError as e:
        print(f"bench.py rank {rank}: {e}", file=sys.stderr, flush=True)
        if use_pg:
            dist.destroy_process_group()
        sys.exit(2)
    pkg = importlib.import_module("congestion-control-with-bittorren_amd")
    pkg.set_device(dev)

    n, L, P = a.chunks, a.chunk_len, max(1, a.streams)
    # weak scaling: rank r owns chunk ids [n*r, n*(r+1)); with P in-flight
    # batches each batch is its own disjoint range of ids
    first, _ = shard.weak_shard(rank * P, n)
    bufs = [torch.empty(n * L, dtype=torch.uint8, device="cuda") for _ in range(P)]
    digs = [torch.zeros((n, 20), dtype=torch.uint8, device="cuda") for _ in range(P)]
    streams = [torch.cuda.Stream() for _ in range(P)]
    for p in range(P):
        pkg.synth_fill_device(bufs[p], first + p * n, n, L, stream=streams[p])
    torch.cuda.synchronize()

    def step(i, ev0=None, ev1=None):
        p = i % P
        if ev0 is not None:
            ev0.record(streams[p])
        pkg.hash_uniform_device(bufs[p], L, n, digs[p], stream=streams[p], kernel=a.kernel)
        if ev1 is not None:
            ev1.record(streams[p])

    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(a.steps)]
    if use_pg:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i, (e0, e1) in enumerate(evs):
        step(i, e0, e1)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if use_pg:
        dist.barrier()
    kern_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))
    elapsed, kern_ms = shard.max_over_ranks([t1 - t0, kern_ms], device=cdev)

    # ---- parity of the timed output (every rank, against the reference) ----
    # Checked with the standard library's SHA-1 (hashlib), independent of
    # both the engine and oracle/: the digest-of-digests of a 4096-chunk
    # range against the reference-generated golden aggregate, otherwise a
    # sample of chunks re-hashed from the device buffer's own bytes.
    golden = json.load(open(os.path.join(ROOT, "tests/golden/golden.json")))
    parity = True
    for p in range(P):
        got = digs[p].cpu().numpy()
        b = first // n + p  # index of this batch's 4096-chunk range
        if n == 4096 and L == CHUNK_LEN and b < len(golden["weak4096"]):
            parity &= hashlib.sha1(got.tobytes()).hexdigest() == golden["weak4096"][b]
        else:
            idx = np.unique(np.linspace(0, n - 1, min(n, 16)).astype(np.int64))
            for i in idx:
                chunk = bufs[p][int(i) * L:(int(i) + 1) * L].cpu().numpy().tobytes()
                parity &= hashlib.sha1(chunk).digest() == got[int(i)].tobytes()
    parity = shard.all_ranks_ok(parity, device=cdev)

    ms_per_step = elapsed / a.steps * 1e3
    total_bytes = world * n * L
    value = total_bytes / (elapsed / a.steps) / 2**30
    alg_bytes = n * (L + 20)  # per launch: every chunk byte read once + its digest
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    blocks = (L + 8) // 64 + 1  # SHA-1 compressions per chunk (sha.c:536-543 padding)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    regime = _regime(n, cus, a.kernel)
    groups = (n + 63) // 64
    # VALU ceiling of the chip for SHA-1 (every SIMD busy with the fused
    # kernel's op mix at the max clock), in the same GB/s as the roofline
    valu_peak = cus * SIMDS_PER_CU * 64 * 64 / FUSED_SIMD_CYCLES_PER_BLOCK * CLOCK_HZ / 1e9
    if regime in ("split_u4_2prod", "split_u2_8wave"):
        floor_ms = blocks * CONSUMER_INSTR_PER_BLOCK * ISSUE_CYCLES / CLOCK_HZ * 1e3
        binding = {
            "limit": "per-chunk serial instruction issue (SHA-1 is serial inside a chunk; "
                     f"{groups} groups of 64 chunks on {cus * SIMDS_PER_CU} SIMDs)",
            "kernel": regime, "floor_ms": round(floor_ms, 4), "achieved_ms": round(kern_ms, 4),
            "frac": round(floor_ms / kern_ms, 4),
            "model": f"{blocks} blocks x {CONSUMER_INSTR_PER_BLOCK} consumer instructions x "
                     f"{ISSUE_CYCLES:g} cyc / 2.4 GHz (profiles/isa_mix_r02.json)",
            "rounds_only_floor_ms": round(blocks * ROUND_VALU_PER_BLOCK * ISSUE_CYCLES
                                          / CLOCK_HZ * 1e3, 4),
        }
    elif regime == "fused":
        waves_per_simd = groups / (cus * SIMDS_PER_CU)
        floor_ms = waves_per_simd * blocks * FUSED_SIMD_CYCLES_PER_BLOCK / CLOCK_HZ * 1e3
        binding = {
            "limit": "SIMD VALU issue (every SIMD busy)", "kernel": regime,
            "floor_ms": round(floor_ms, 4), "achieved_ms": round(kern_ms, 4),
            "frac": round(floor_ms / kern_ms, 4),
            "model": f"{waves_per_simd:g} waves/SIMD x {blocks} blocks x "
                     f"{FUSED_SIMD_CYCLES_PER_BLOCK:g} SIMD cycles / 2.4 GHz ({FUSED_VALU_PER_BLOCK} VALU "
                     "per block x 4 cycles, profiles/isa_mix_r02.json); the chip holds "
                     "~2.2 GHz under this load (profiles/pmc_shape_r03.json)",
        }
    else:  # forced lane kernel, 1-block or A/B split shapes: not modelled
        binding = {"limit": "not modelled", "kernel": regime, "achieved_ms": round(kern_ms, 4)}
    label = f"{n} x {L} B chunks per GPU, device-resident"
    if L == CHUNK_LEN and n in NAMED_WORKLOADS:
        label += f" ({NAMED_WORKLOADS[n]})"

    result = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (splitmix64 corpus, SURVEY.md 8d), resident in HBM",
        "config": {"workload": label,
                   "chunks_per_gpu": n, "chunk_bytes": L, "kernel": regime,
                   "kernel_requested": a.kernel, "streams": P,
                   "parallelism": f"chunk-sharded x{world}, no collective",
                   "devices": idents},
        "parity": parity,
        # HBM is the metric's denominator (BASELINE.json), not the binding
        # limit: see binding_limit and valu_ceiling
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": _traffic(n, L),
            "kernel_ms": round(kern_ms, 4),
        },
        "valu_ceiling": {
            "achieved": round(achieved, 2), "peak": round(valu_peak, 1), "unit": "GB/s",
            "frac": round(achieved / valu_peak, 4),
            "model": f"{cus * SIMDS_PER_CU} SIMDs x 64 chunks x 64 B per "
                     f"{FUSED_SIMD_CYCLES_PER_BLOCK:g} SIMD cycles ({FUSED_VALU_PER_BLOCK:g} VALU x 4) at 2.4 GHz",
            "measured_compress_only": COMPRESS_ONLY_GBS,
            "frac_of_measured": round(achieved / COMPRESS_ONLY_GBS, 4),
        },
        "binding_limit": binding,
    }
    # free the config-2 buffers before the strong leg's 128 GiB / N
    del bufs, digs
    torch.cuda.empty_cache()
    if a.strong_total > 0:
        result["strong"] = _strong_leg(pkg, shard, torch, dist, world, rank, cdev, a, golden)
    if a.weak4_chunks > 0:
        result["weak_config4"] = _weak4_leg(pkg, shard, torch, dist, world, rank, cdev, a, golden)
    if rank == 0 and world == 1 and a.strong_total == 262144 and not a.no_configs:
        # the per-GPU shards of the 1->8 strong curve that one GPU can time
        # (VERDICT r4 next #1): N = 8 (32768 chunks, two groups of 64 per
        # CU, the 8-wave split shape) and N = 2 (131072); N = 4's shard
        # (65536) is weak_config4's workload
        result["config4_shard8"] = _shard_leg(pkg, shard, torch, golden, 8, 1, a)
        result["config4_shard2"] = _shard_leg(pkg, shard, torch, golden, 2, 1, a)
        result["strong_projection"] = _strong_projection(result)
    fpath, reqs = None, None
    try:
        if rank == 0 and world == 1 and not a.no_configs:
            # the other BASELINE configs on this GPU, each checked against the
            # reference's golden digests (configs 1, 3, 5; 2 and 4 are above)
            result["config5"] = _config5_leg(pkg, torch, golden)
            result["config3_e2e"] = _config3_leg(pkg, torch, golden)
            result["config1"] = _config1_leg(golden)
            result["verify_queue"] = _verify_queue_leg(result["config3_e2e"].get("pinned_h2d_GiBps"))
            if a.file_chunks > 0:
                # a failed file leg must not cost the bench line (no room for
                # the temp file, a tool missing): its object says why
                try:
                    fpath = _write_corpus_file(pkg, torch, a.file_chunks)
                    result["file"], fdig = _file_leg(pkg, fpath, golden,
                                                     result["config3_e2e"].get("pinned_h2d_GiBps"))
                    result["master_verify"], reqs = _master_verify_leg(fpath, fdig)
                except Exception as e:
                    result.setdefault("file", {"error": repr(e)[:300]})
                    if fpath and "master_verify" not in result:
                        result["master_verify"] = {"error": repr(e)[:300]}
        if rank == 0 and world == 1 and not a.no_latency:
            result["latency_one_chunk"] = _latency_one_chunk(dev)
        if rank == 0 and world == 1 and not a.no_cpu_baseline:
            from oracle import oracle as O  # the CPU baseline leg only: the reference sha.c, timed
            result["cpu_baseline"] = _cpu_baseline(O, n, L, golden, a.cpu_threads or None)
            if "latency_one_chunk" in result:
                result["latency_one_chunk"]["reference_sha_c_one_core_ms"] = \
                    result["cpu_baseline"].pop("one_chunk_ms")
            if "config1" in result:
                ref = _reference_cli(golden)
                result["cpu_baseline"]["config1_reference_cli"] = ref
                c1 = result["config1"]
                c1["reference_cli_median_ms"] = ref["median_ms"]
                for k in ("default", "device", "host_small"):
                    c1[k]["vs_reference"] = round(c1[k]["median_ms"] / ref["median_ms"], 3)
            if fpath and reqs:
                ref = _reference_master_verify(fpath, reqs)
                result["cpu_baseline"]["master_verify_reference"] = ref
                mv = result["master_verify"]
                for k in ("O0", "O2"):
                    if ref.get(k, {}).get("rest_median_ms"):
                        mv[f"reference_{k}_per_get_ms"] = ref[k]["rest_median_ms"]
                if ref.get("O0", {}).get("rest_median_ms") and mv.get("index", {}).get("rest_median_ms"):
                    mv["index_speedup_vs_reference_O0"] = round(
                        ref["O0"]["rest_median_ms"] / mv["index"]["rest_median_ms"], 1)
            if fpath and "cli" in result.get("file", {}):
                ref = _reference_file_cli(fpath)
                result["cpu_baseline"]["file_reference_cli"] = ref
                if ref.get("GiBps"):
                    fl = result["file"]
                    fl["reference_cli_GiBps"] = ref["GiBps"]
                    fl["cli_vs_reference"] = round(fl["cli"]["GiBps"] / ref["GiBps"], 1)
    finally:
        if fpath and os.path.exists(fpath):
            os.unlink(fpath)
    if use_pg:
        result["config"]["control_plane"] = f"torch.distributed {backend}, world {world}"
    if rank == 0:
        print(json.dumps(result), flush=True)
    if use_pg:
        dist.destroy_process_group()


def _time_launches(pkg, torch, buf, L, n, dig, stream, steps, warmup):
    """warmup untimed launches, then `steps` launches bracketed by
    synchronize: (wall seconds, mean HIP-event ms per launch)."""
    for _ in range(warmup):
        pkg.hash_uniform_device(buf, L, n, dig, stream=stream)
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(steps)]
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record(stream)
        pkg.hash_uniform_device(buf, L, n, dig, stream=stream)
        e1.record(stream)
    torch.cuda.synchronize()
    return time.perf_counter() - t0, float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))


def _strong_leg(pkg, shard, torch, dist, world, rank, cdev, a, golden):
    """BASELINE config 4 strong scaling: the fixed list of `total` chunks
    split into `world` contiguous shards (no collective on the data path)."""
    total, L, K = a.strong_total, CHUNK_LEN, max(1, a.strong_steps)
    first, cnt = shard.strong_shard(rank, world, total)
    st = torch.cuda.Stream()
    buf = torch.empty(max(cnt, 1) * L, dtype=torch.uint8, device="cuda")
    dig = torch.zeros((max(cnt, 1), 20), dtype=torch.uint8, device="cuda")
    pkg.synth_fill_device(buf, first, cnt, L, stream=st)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    # 3 untimed launches: with every CU busy the clock ramps up over the first
    # ~20 ms of load (32768 chunks: 8.3, 6.9, 6.5, 6.4 ms for the first
    # dispatches, then 6.36; profiles/pmc_shape_r03.json)
    wall, kern_ms = _time_launches(pkg, torch, buf, L, cnt, dig, st, K, 3)
    if world > 1:
        dist.barrier()
    wall, kern_ms = shard.max_over_ranks([wall, kern_ms], device=cdev)
    got = dig[:cnt].cpu().numpy()
    want = shard.strong_golden_agg(golden, world, rank, total)
    ok = want is not None and hashlib.sha1(got.tobytes()).hexdigest() == want
    parity = shard.all_ranks_ok(ok, device=cdev)
    del buf, dig
    torch.cuda.empty_cache()
    ms_n = wall / K * 1e3
    # the one-GPU time of the whole list: at N = 1 that is this leg; at N > 1
    # rank 0 hashes all `total` chunks on its own GPU while the others wait
    one_ms, one_kern_ms, one_parity = ms_n, kern_ms, parity
    if world > 1:
        if rank == 0:
            buf = torch.empty(total * L, dtype=torch.uint8, device="cuda")
            dig = torch.zeros((total, 20), dtype=torch.uint8, device="cuda")
            pkg.synth_fill_device(buf, 0, total, L, stream=st)
            torch.cuda.synchronize()
            w1, one_kern_ms = _time_launches(pkg, torch, buf, L, total, dig, st, K, 3)
            one_ms = w1 / K * 1e3
            one_parity = hashlib.sha1(dig.cpu().numpy().tobytes()).hexdigest() == \
                golden["config4"]["agg"]
            del buf, dig
            torch.cuda.empty_cache()
        dist.barrier()
    return shard.strong_report(total, L, world, ms_n, kern_ms, one_ms, one_kern_ms, parity,
                               one_parity, K)


def _shard_leg(pkg, shard, torch, golden, k, r, a) -> dict:
    """Shard r of the k-way contiguous split of config 4's 262144-chunk list
    (shard.strong_shard), hashed on this GPU: the per-GPU work of the strong
    curve at N = k.  Timed like `strong` (3 untimed launches, then K),
    checked against the reference golden shard aggregate, with the kernel's
    issue floor for its regime."""
    total, L, K = a.strong_total, CHUNK_LEN, max(1, a.strong_steps)
    first, cnt = shard.strong_shard(r, k, total)
    st = torch.cuda.Stream()
    buf = torch.empty(cnt * L, dtype=torch.uint8, device="cuda")
    dig = torch.zeros((cnt, 20), dtype=torch.uint8, device="cuda")
    pkg.synth_fill_device(buf, first, cnt, L, stream=st)
    torch.cuda.synchronize()
    wall, kern_ms = _time_launches(pkg, torch, buf, L, cnt, dig, st, K, 3)
    ok = hashlib.sha1(dig.cpu().numpy().tobytes()).hexdigest() == golden["config4"]["shard_aggs"][str(k)][r]
    del buf, dig
    torch.cuda.empty_cache()
    cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    regime = _regime(cnt, cus, "auto")
    blocks = (L + 8) // 64 + 1
    out = {"workload": f"shard {r} of the {k}-way split of BASELINE config 4 ({cnt} x {L} B, "
                       f"chunks {first}..{first + cnt - 1}), device-resident, one GPU",
           "chunks": cnt, "steps": K, "ms_per_step": round(wall / K * 1e3, 4), "kernel_ms": round(kern_ms, 4),
           "GiBps": round(cnt * L / (kern_ms * 1e-3) / 2**30, 2),
           "hbm_frac": round(cnt * (L + 20) / (kern_ms * 1e-3) / (HBM_PEAK_GBS * 1e9), 5),
           "kernel": regime, "parity": bool(ok),
           "parity_ref": f"digest-of-digests == golden config4.shard_aggs[{k}][{r}] (reference sha.c)"}
    if regime.startswith("split"):
        floor = blocks * CONSUMER_INSTR_PER_BLOCK * ISSUE_CYCLES / CLOCK_HZ * 1e3
        out["floor_ms"] = round(floor, 4)
        out["floor_frac"] = round(floor / kern_ms, 4)
        out["floor_model"] = (f"one chunk's serial chain: {blocks} blocks x {CONSUMER_INSTR_PER_BLOCK} "
                              f"consumer instructions x {ISSUE_CYCLES:g} cyc / 2.4 GHz")
    else:
        waves_per_simd = (cnt + 63) // 64 / (cus * SIMDS_PER_CU)
        floor = waves_per_simd * blocks * FUSED_SIMD_CYCLES_PER_BLOCK / CLOCK_HZ * 1e3
        out["floor_ms"] = round(floor, 4)
        out["floor_frac"] = round(floor / kern_ms, 4)
        out["floor_model"] = f"SIMD VALU issue: {waves_per_simd:g} waves/SIMD x {blocks} blocks x " \
                             f"{FUSED_SIMD_CYCLES_PER_BLOCK:g} cyc / 2.4 GHz"
    return out


def _strong_projection(result) -> dict:
    """Config 4's strong curve as one GPU predicts it: the shards are equal
    and independent (no collective), so N GPUs take as long as one GPU takes
    for its 262144/N-chunk shard.  Speed-up = the whole list's kernel time
    (`strong`, N = 1) / the shard's."""
    one = result.get("strong", {}).get("one_gpu_kernel_ms")
    shards = {"2": result.get("config4_shard2"), "4": result.get("weak_config4"),
              "8": result.get("config4_shard8")}
    out = {"basis": "one-GPU kernel time of the whole 262144-chunk list / of one shard "
                    "(N = 4: weak_config4, whose 65536 chunks are one shard of the 4-way split)"}
    if one:
        out["speedup"] = {n: round(one / v["kernel_ms"], 3) for n, v in shards.items() if v and v.get("kernel_ms")}
        out["efficiency"] = {n: round(x / int(n), 4) for n, x in out["speedup"].items()}
    out["parity"] = all(v.get("parity", False) for v in shards.values() if v)
    return out


def _weak4_leg(pkg, shard, torch, dist, world, rank, cdev, a, golden):
    """Config 4's weak scaling (65536 chunks per GPU): every
    rank hashes its own `per` chunks, no collective on the data path.  Rank r
    takes shard r % 4 of the 4-way split of the config-4 list (for the
    default 65536 chunks per rank), so its digest-of-digests has a reference
    golden aggregate at any N; the bytes are the same synthetic chunks either
    way.  Timed like the other legs (3 untimed launches, barrier + synchronize
    around K, max over ranks)."""
    per, L, K = a.weak4_chunks, CHUNK_LEN, max(1, a.strong_steps)
    first, _, want = shard.weak_golden_agg(golden, rank, per)
    st = torch.cuda.Stream()
    buf = torch.empty(per * L, dtype=torch.uint8, device="cuda")
    dig = torch.zeros((per, 20), dtype=torch.uint8, device="cuda")
    pkg.synth_fill_device(buf, first, per, L, stream=st)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall, kern_ms = _time_launches(pkg, torch, buf, L, per, dig, st, K, 3)
    if world > 1:
        dist.barrier()
    wall, kern_ms = shard.max_over_ranks([wall, kern_ms], device=cdev)
    ok = want is not None and hashlib.sha1(dig.cpu().numpy().tobytes()).hexdigest() == want
    parity = shard.all_ranks_ok(ok, device=cdev)
    del buf, dig
    torch.cuda.empty_cache()
    ms = wall / K * 1e3
    return {
        "workload": f"{per} x {L} B chunks per GPU, device-resident (config 4 weak scaling)",
        "chunks_per_gpu": per, "n_gpus": world, "steps": K,
        "ms_per_step": round(ms, 4), "kernel_ms": round(kern_ms, 4),
        "value": round(world * per * L / 2**30 / (ms / 1e3), 2), "unit": "GiB/s",
        "per_gpu_hbm_frac": round(per * (L + 20) / (kern_ms / 1e3) / (HBM_PEAK_GBS * 1e9), 5),
        "kernel": _regime(per, 256, "auto"),
        "parity": bool(parity),
        "parity_ref": "each rank's digest-of-digests vs golden config4 shard_aggs[k][rank % k], "
                      "k = 262144 / chunks per GPU",
    }


def _latency_one_chunk(dev: int) -> dict:
    """verify_hash (job.c:217-228) on one 512 KiB chunk through the library in
    a child process: the first call (library load included) and the median
    of 20 warm calls, with the library's default routing (one message on the
    host: csrc/sha1_host.c, the device still required and checked through
    the KFD topology, so no HIP start-up) and on the kernels
    (SHA1CHUNK_HOST_SMALL=0: one lane's serial chain, HIP start-up in the
    first call)."""
    import subprocess
    code = (
        "import ctypes, hashlib, json, os, sys, time\n"
        "import numpy as np\n"
        "L = 524288\n"
        "data = np.random.default_rng(5).integers(0, 256, L, dtype=np.uint8).tobytes()\n"
        "hexd = hashlib.sha1(data).hexdigest().encode()\n"
        "t0 = time.perf_counter()\n"
        "lib = ctypes.CDLL(sys.argv[1])\n"
        "lib.verify_hash.argtypes = [ctypes.c_char_p, ctypes.c_char_p]\n"
        "if sys.argv[2] != '0':\n"
        "    lib.sha1chunk_set_device(int(sys.argv[2]))  # device 0 is the default, as for the peer\n"
        "t1 = time.perf_counter()\n"
        "assert lib.verify_hash(hexd, data) == 0\n"
        "t2 = time.perf_counter()\n"
        "warm = []\n"
        "for _ in range(20):\n"
        "    a = time.perf_counter(); r = lib.verify_hash(hexd, data); warm.append(time.perf_counter() - a)\n"
        "    assert r == 0\n"
        "bad = bytes(data[:7]) + bytes([data[7] ^ 1]) + bytes(data[8:])\n"
        "assert lib.verify_hash(hexd, bad) == 1\n"
        "sys.stdout.flush()\n"
        "print('LATENCY ' + json.dumps({'probe_ms': (t1 - t0) * 1e3, 'first_call_ms': (t2 - t1) * 1e3,\n"
        "      'warm_ms': float(np.median(warm)) * 1e3, 'warm_min_ms': min(warm) * 1e3}))\n")
    libp = os.path.join(ROOT, "congestion-control-with-bittorren_amd", "libsha1chunk.so")

    def child(extra_env):
        env = _env_without_knob(extra_env)
        r = subprocess.run([sys.executable, "-c", code, libp, str(dev)], capture_output=True,
                           text=True, timeout=120, env=env)
        line = [x for x in r.stdout.splitlines() if x.startswith("LATENCY ")]
        if r.returncode != 0 or not line:
            raise RuntimeError((r.stderr or r.stdout)[-300:])
        return json.loads(line[-1][8:])

    try:
        d = child({})
        dv = child({"SHA1CHUNK_HOST_SMALL": "0"})
    except Exception as e:  # a failed probe must not cost the bench line
        return {"error": repr(e)[:300]}
    return {"path": "verify_hash -> get_chunk_hash -> shahash (job.c:217-228), the library's default "
                    "routing: one message is hashed on the host (csrc/sha1_host.c, x86 SHA extensions; "
                    "a gfx950 device is still required, checked through the KFD topology)",
            "cold_ms": round(d["probe_ms"] + d["first_call_ms"], 3),
            "cold_first_call_ms": round(d["first_call_ms"], 3),
            "warm_ms": round(d["warm_ms"], 3), "warm_min_ms": round(d["warm_min_ms"], 3),
            "bytes": CHUNK_LEN,
            "device": {"knob": "SHA1CHUNK_HOST_SMALL=0 (every call on the kernels)",
                       "path": "shahash -> sha1chunk_hash_batch(n=1): one lane of the split kernel",
                       "cold_ms": round(dv["probe_ms"] + dv["first_call_ms"], 3),
                       "cold_first_call_ms": round(dv["first_call_ms"], 3),
                       "warm_ms": round(dv["warm_ms"], 3), "warm_min_ms": round(dv["warm_min_ms"], 3)}}


class _CaptureStderr:
    """Collect what C code writes to fd 2 inside the block (the runtime's
    SHA1CHUNK_MIXED_DEBUG plan line)."""

    def __enter__(self):
        import tempfile
        sys.stderr.flush()
        self._tmp = tempfile.TemporaryFile(mode="w+b")
        self._saved = os.dup(2)
        os.dup2(self._tmp.fileno(), 2)
        self.text = ""
        return self

    def __exit__(self, *exc):
        sys.stderr.flush()
        os.dup2(self._saved, 2)
        os.close(self._saved)
        self._tmp.seek(0)
        self.text = self._tmp.read().decode(errors="replace")
        self._tmp.close()


def _chain_floor_ms(length: int) -> float:
    """One chunk's serial instruction stream on the split kernel's consumer
    wave (the bound of a batch whose longest chunk runs alone on a SIMD)."""
    blocks = (length + 8) // 64 + 1
    return blocks * CONSUMER_INSTR_PER_BLOCK * ISSUE_CYCLES / CLOCK_HZ * 1e3


def _mixed_run(pkg, torch, lens: np.ndarray, reps: int = 5, warm: int = 2, layout: str = "arrival",
               forced=()) -> dict:
    """A device-resident mixed-length batch (chunk i = synthetic chunk i at
    lens[i] bytes, 128-byte aligned) through AUTO -- the length sort and,
    above one group of 64 per CU, the mixed kernel's persistent dispatch
    with its device-side plan.  layout "arrival": the chunks back to back in
    index order (as received); "longest_first": back to back in descending
    length order (the same chunks and digests, laid out so every sorted
    group's chunks lie together).  `forced`: plans ("mode,H,F") run through
    SHA1CHUNK_MIXED_PLAN on the same buffer after AUTO, for comparison.
    Timed with HIP events on the call's stream (sort + plan + hash), median
    of `reps` after `warm`."""
    n = int(lens.size)
    if layout == "arrival":
        off, total = pkg.sha1chunk.ragged_layout(lens)
    else:
        # the device's order: descending SHA-1 block counts, stable
        # (sha1_sort.hip), so every sorted group's chunks lie together
        keys = np.minimum((lens.astype(np.int64) + 9 + 63) // 64, 65535)
        order = np.argsort(-keys, kind="stable")
        o2, total = pkg.sha1chunk.ragged_layout(lens[order])
        off = np.empty_like(o2)
        off[order] = o2
    st = torch.cuda.Stream()
    d_base = torch.zeros(total + 128, dtype=torch.uint8, device="cuda")
    d_off = torch.from_numpy(off.astype(np.int64)).cuda()
    d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
    dig = torch.zeros((n, 20), dtype=torch.uint8, device="cuda")
    st.wait_stream(torch.cuda.current_stream())  # the zero fills and copies above run on torch's stream
    pkg.synth_fill_ragged_device(d_base, d_off, d_len, 0, stream=st)
    torch.cuda.synchronize()

    def timed():
        for _ in range(warm):
            pkg.hash_device(d_base, d_off, d_len, dig, stream=st)
        torch.cuda.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(reps)]
        t0 = time.perf_counter()
        for e0, e1 in evs:
            e0.record(st)
            pkg.hash_device(d_base, d_off, d_len, dig, stream=st)
            e1.record(st)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / reps
        # the plan the runtime used (one more, untimed call with the debug line on)
        plan = stages = None
        os.environ["SHA1CHUNK_MIXED_DEBUG"] = "1"
        try:
            with _CaptureStderr() as cap:
                pkg.hash_device(d_base, d_off, d_len, dig, stream=st)
                torch.cuda.synchronize()
        finally:
            del os.environ["SHA1CHUNK_MIXED_DEBUG"]
        for line in cap.text.splitlines():
            if line.startswith("sha1chunk mixed plan:"):
                plan = line.split(":", 1)[1].strip()
            if line.startswith("sha1chunk mixed planner stages:"):
                stages = line.split(":", 1)[1].strip()
        return (float(np.median([e0.elapsed_time(e1) for e0, e1 in evs])), wall, plan, dig.cpu().numpy(),
                stages)

    ms, wall, plan, got, stages = timed()
    vs = {}
    for f in forced:
        os.environ["SHA1CHUNK_MIXED_PLAN"] = f
        try:
            fms, _, fplan, fgot, _ = timed()
        finally:
            del os.environ["SHA1CHUNK_MIXED_PLAN"]
        vs[f] = {"kernel_ms": round(fms, 4), "plan": fplan, "auto_over_forced": round(ms / fms, 4),
                 "same_digests": bool(np.array_equal(fgot, got))}
    payload = int(lens.astype(np.uint64).sum())
    longest = int(lens.max())
    floor = _chain_floor_ms(longest)
    del d_base, d_off, d_len, dig
    torch.cuda.empty_cache()
    out = {"chunks": n, "layout": layout, "payload_bytes": payload, "kernel_ms": round(ms, 4),
           "wall_ms_per_call": round(wall * 1e3, 4),
           "payload_GiBps": round(payload / (ms * 1e-3) / 2**30, 2),
           "hbm_frac": round((payload + 20 * n) / (ms * 1e-3) / (HBM_PEAK_GBS * 1e9), 5),
           "longest_chunk_bytes": longest, "longest_chain_floor_ms": round(floor, 4),
           "floor_frac": round(floor / ms, 4),
           "plan": plan or "no mixed kernel (<= one group of 64 per CU: split shape)",
           "_digests": got}
    if stages:  # the planner's stage end times in the untimed debug call (us since its start)
        out["planner_stages_untimed_call"] = stages
    if vs:
        out["forced"] = vs
    return out


def _config5_leg(pkg, torch, golden) -> dict:
    """BASELINE config 5 (mixed 4 KiB - 1 MiB, the received-chunk verify
    shape, packet_handler.c:469-472 -> job.c:217-228): the 16384-chunk batch
    checked digest by digest against the reference's golden file, and the
    same length law at 4x (65536 chunks, the persistent mixed kernel's
    regime) against its reference golden aggregate, and at 8x (131072) in
    arrival and longest-first layouts, each beside a forced plan (the mixed
    planner's layout- and clock-aware choice)."""
    import hashlib
    lens = np.fromfile(os.path.join(ROOT, "tests/golden/mixed_16384_len.bin"), "<u4")
    want = np.fromfile(os.path.join(ROOT, "tests/golden/mixed_16384.bin"), np.uint8).reshape(-1, 20)
    ok_lens = hashlib.sha1(lens.tobytes()).hexdigest() == golden["config5"]["lengths_sha1"]
    r16 = _mixed_run(pkg, torch, lens)
    r16["parity"] = bool(ok_lens and np.array_equal(r16.pop("_digests"), want))
    r16["parity_ref"] = "all 16384 digests == tests/golden/mixed_16384.bin (reference sha.c)"
    g4 = golden.get("config5x4")
    out = {"workload": "BASELINE config 5: mixed 4 KiB-1 MiB chunks, device-resident, AUTO",
           "n16384": r16}
    if g4:
        lens4 = pkg.sha1chunk.mixed_lengths(g4["chunks"])
        r64 = _mixed_run(pkg, torch, lens4)
        d = r64.pop("_digests")
        r64["parity"] = bool(hashlib.sha1(lens4.tobytes()).hexdigest() == g4["lengths_sha1"] and
                             hashlib.sha1(d.tobytes()).hexdigest() == g4["agg"])
        r64["parity_ref"] = "digest-of-digests == golden config5x4.agg (reference sha.c)"
        out["n65536"] = r64
    g8 = golden.get("config5x8")
    if g8:
        # the law at 8x in both layouts, AUTO against the best forced plan of
        # the round-4 grids (tools/mixed_verify.sh: H = 187, F = 4 in both)
        lens8 = pkg.sha1chunk.mixed_lengths(g8["chunks"])
        ok_l8 = hashlib.sha1(lens8.tobytes()).hexdigest() == g8["lengths_sha1"]
        for lay in ("arrival", "longest_first"):
            r = _mixed_run(pkg, torch, lens8, layout=lay, forced=("0,187,4",))
            d = r.pop("_digests")
            r["parity"] = bool(ok_l8 and hashlib.sha1(d.tobytes()).hexdigest() == g8["agg"] and
                               all(v["same_digests"] for v in r["forced"].values()))
            r["parity_ref"] = "digest-of-digests == golden config5x8.agg (reference sha.c); forced plans: same digests"
            out[f"n131072_{lay}"] = r
    out["parity"] = all(v["parity"] for k, v in out.items() if k.startswith("n"))
    return out


def _config3_leg(pkg, torch, golden, reps: int = 2) -> dict:
    """BASELINE config 3: 65536 x 512 KiB from PINNED host memory through
    sha1chunk_hash_batch (H2D || hash || D2H on the runtime's two-slot
    pipeline), whole-call wall time; the raw pinned H2D rate of the same
    box measured in the same run, and the digest-of-digests against the
    reference's golden aggregate."""
    import hashlib
    n, L = 65536, CHUNK_LEN
    t_pin = time.perf_counter()
    host = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
    t_pin = time.perf_counter() - t_pin
    piece = 2048
    tmp = torch.empty(piece * L, dtype=torch.uint8, device="cuda")
    for c0 in range(0, n, piece):
        pkg.synth_fill_device(tmp, c0, piece, L)
        host[c0 * L:(c0 + piece) * L].copy_(tmp)
    torch.cuda.synchronize()
    hv = host.numpy()
    off = np.arange(n, dtype=np.uint64) * L
    ln = np.full(n, L, np.uint32)
    _ = pkg.hash_batch(hv[: 64 * L], off[:64], ln[:64])  # warm: slots, streams, code object
    ts, dig = [], None
    for _ in range(reps):
        t0 = time.perf_counter()
        dig = pkg.hash_batch(hv, off, ln)
        ts.append(time.perf_counter() - t0)
    sec = float(np.median(ts))
    parity = hashlib.sha1(dig.tobytes()).hexdigest() == golden["config3"]["agg"]
    # raw pinned H2D over 4 GiB pieces of the same host buffer
    nb = 1 << 32
    dev_buf = torch.empty(nb, dtype=torch.uint8, device="cuda")
    h2d = []
    for k in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dev_buf.copy_(host[k * nb:(k + 1) * nb], non_blocking=True)
        torch.cuda.synchronize()
        h2d.append(time.perf_counter() - t0)
    h2d_gib = nb / float(np.median(h2d)) / 2**30
    del dev_buf, tmp, host, hv
    torch.cuda.empty_cache()
    e2e = n * L / sec / 2**30
    return {"workload": "BASELINE config 3: 65536 x 524288 B from pinned host memory, "
                        "H2D || hash || D2H (sha1chunk_hash_batch)",
            "chunks": n, "bytes": n * L, "seconds": round(sec, 4),
            "runs_s": [round(t, 4) for t in ts], "e2e_GiBps": round(e2e, 2),
            "pinned_h2d_GiBps": round(h2d_gib, 2), "e2e_over_h2d": round(e2e / h2d_gib, 4),
            "pin_alloc_s": round(t_pin, 2), "parity": bool(parity),
            "parity_ref": "digest-of-digests == golden config3.agg (reference sha.c)"}


def _verify_queue_leg(h2d_gibps, reps: int = 5) -> dict:
    """SURVEY 8(f) rank 2, the received-chunk verify queue (reliable_udp.c:121
    session buffer, filled at :339; packet_handler.c:472 -> job.c:217-228):
    16384 x 512 KiB host chunks, reassembled by 4 receive threads in 1484-byte
    DATA payloads, 20 % corrupted in place before the verify, through
    tools/vq_zc_bench (C, linked against libsha1chunk.so): zero-copy
    (sha1chunk_vq_reserve / commit / release), the reference's own call
    shape (fill a malloc'd session buffer, sha1chunk_vq_submit), and the
    receive threads' fills alone (reserve, fill, release: no verify) as the
    bound both sit under.  The payload pieces come from 64 distinct source
    chunks (32 MiB, cache-resident), as a receive path copies each datagram
    from a just-received packet buffer (peer.c:81 recvfrom ->
    reliable_udp.c:339 memcpy); zero-copy is timed once more with 4096
    distinct source chunks (2 GiB read from DRAM), the round-5 shape, whose
    host memory traffic swings it run to run (profiles/vq_reps_d*.jsonl).
    The receive threads run on the GPU's NUMA node, one per L3 domain (CCD)
    of it (--pin l3: a NIC-local receive path with a CCD per thread; left to
    float over the node, --pin gpu, `submit` passes ranged 25.9-36.2 GiB/s
    against 27.7-29.6, zero-copy the same either way, profiles/vq_l3.jsonl;
    the library's helper threads are placed on the node by default,
    SHA1CHUNK_NUMA) and every pass records where its threads and pages were
    and the cgroup's CPU throttling.  One process per
    mode, `reps` passes each (--reps): the median pass is the reported GiB/s,
    min, max and every pass beside it -- from the DRAM source single passes
    swing +-15 % with the host's memory traffic, the fills alone as much
    (profiles/vq_reps_r06a.jsonl); from the cache-resident one zero-copy
    passes stay within 6 % (profiles/vq_reps_d64.jsonl).
    Every result is checked against the verdict the reference golden digests
    give (tests/golden/synth_4096x512k.bin); GiB/s next to this run's pinned
    H2D."""
    import subprocess
    tool = os.path.join(ROOT, "tools", "vq_zc_bench")
    out = {"workload": "16384 x 524288 B host chunks, 4 receive threads filling 1484-byte pieces, "
                       "20 % corrupted, persistent drain", "pinned_h2d_GiBps": h2d_gibps, "passes_per_mode": reps}
    if not os.path.exists(tool):
        out["error"] = "tools/vq_zc_bench not built (make -C congestion-control-with-bittorren_amd tools)"
        return out
    out["source"] = "64 distinct source chunks (32 MiB, cache-resident: the packet buffers a receive path " \
                    "copies from); zero_copy_dram_source: 4096 (2 GiB)"
    for mode, key, distinct in (("fill", "fill_only", 64), ("reserve", "zero_copy", 64), ("submit", "submit", 64),
                                ("reserve", "zero_copy_dram_source", 4096)):
        try:
            r = subprocess.run([tool, "--mode", mode, "--chunks", "16384", "--producers", "4",
                                "--distinct", str(distinct), "--pieces", "1", "--pin", "l3", "--reps", str(reps),
                                "--golden", os.path.join(ROOT, "tests/golden/synth_4096x512k.bin")],
                               capture_output=True, text=True, timeout=180, cwd=ROOT)
            good = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
            if r.returncode != 0 or len(good) != reps:
                out[key] = {"error": f"rc {r.returncode}, {len(good)} passes: {(r.stderr or r.stdout)[-300:]}"}
                continue
        except Exception as e:  # a failed mode must not cost the bench line
            out[key] = {"error": repr(e)[:300]}
            continue
        rates = [g["GiBps"] for g in good]
        med = good[int(np.argsort(rates)[len(rates) // 2])]
        rec = dict(med)
        rec["GiBps"] = float(np.median(rates))
        rec["GiBps_passes"] = rates
        rec["GiBps_min"], rec["GiBps_max"] = min(rates), max(rates)
        rec["spread"] = round((max(rates) - min(rates)) / rec["GiBps"], 4)
        rec["produce_seconds_passes"] = [g["produce_seconds"] for g in good]
        rec["placement_passes"] = [{"producer_cpus": [q["cpu_start"] for q in g["placement"]["producers"]],
                                    "producer_nodes": sorted({q["node_end"] for q in g["placement"]["producers"]}),
                                    "cgroup_nr_throttled": g["placement"]["cgroup_nr_throttled"]} for g in good]
        if mode != "fill":
            rec["parity"] = all(bool(g.get("results_correct")) and g.get("flagged") == len(range(2, 16384, 5))
                                for g in good)
        if h2d_gibps:
            rec["over_h2d"] = round(rec["GiBps"] / h2d_gibps, 4)
        out[key] = rec
    fill = out.get("fill_only", {}).get("GiBps")
    for key in ("zero_copy", "submit"):
        if fill and "GiBps" in out.get(key, {}):
            out[key]["over_fill_only"] = round(out[key]["GiBps"] / fill, 4)
    out["parity"] = all(out.get(k, {}).get("parity", False) for k in ("zero_copy", "submit", "zero_copy_dram_source"))
    out["parity_ref"] = "every chunk's 0/1 == (its bytes hash to the reference golden digest); 3277 flagged, " \
                        "every pass"
    return out


def _write_corpus_file(pkg, torch, chunks: int) -> str:
    """Chunks 0..chunks-1 of the synthetic corpus (config 3's first chunks),
    generated on the device, written to a temp file ($TMPDIR)."""
    import shutil
    import tempfile
    need = chunks * CHUNK_LEN
    free = shutil.disk_usage(tempfile.gettempdir()).free
    if free < need + (1 << 30):
        raise RuntimeError(f"{tempfile.gettempdir()}: {free} bytes free, the file leg needs {need} + 1 GiB")
    fd, path = tempfile.mkstemp(prefix="sha1bench_file_", suffix=".dat")
    piece = 1024
    tmp = torch.empty(piece * CHUNK_LEN, dtype=torch.uint8, device="cuda")
    host = torch.empty(piece * CHUNK_LEN, dtype=torch.uint8, pin_memory=True)
    try:
        with os.fdopen(fd, "wb", buffering=0) as f:
            for c0 in range(0, chunks, piece):
                k = min(piece, chunks - c0)
                pkg.synth_fill_device(tmp, c0, k, CHUNK_LEN)
                host[:k * CHUNK_LEN].copy_(tmp[:k * CHUNK_LEN])
                torch.cuda.synchronize()
                f.write(memoryview(host.numpy())[:k * CHUNK_LEN])
    except BaseException:
        os.unlink(path)
        raise
    del tmp, host
    torch.cuda.empty_cache()
    return path


def _file_leg(pkg, path: str, golden, h2d_gibps, reps: int = 3):
    """make-chunks on a real file (make_chunks.c:14-62 ->
    chunk.c:15-27), the file in the page cache: make_chunks in-process
    (sha1chunk_hash_fd: parallel pread into pinned slots -> H2D -> kernel ->
    D2H) and the repo's make-chunks CLI as a whole process, median of `reps`
    after one warm call each; the file's page-cache read rate beside them.
    Parity: every 4096-chunk block's digest-of-digests against the reference
    golden weak4096 aggregates (all chunks), the golden config-3 samples in
    range, and the CLI's "%d %s" lines against the in-process digests."""
    import subprocess
    size = os.path.getsize(path)
    n = (size + CHUNK_LEN - 1) // CHUNK_LEN
    buf = bytearray(64 << 20)
    mv = memoryview(buf)
    t0 = time.perf_counter()
    with open(path, "rb", buffering=0) as f:
        while f.readinto(mv):
            pass
    read_gibs = size / (time.perf_counter() - t0) / 2**30
    pkg.make_chunks(path)  # warm: device, pinned slots
    ts, digs = [], None
    for _ in range(reps):
        t0 = time.perf_counter()
        digs = pkg.make_chunks(path)
        ts.append(time.perf_counter() - t0)
    d = np.frombuffer(b"".join(digs), np.uint8).reshape(-1, 20)
    cli = os.path.join(ROOT, "congestion-control-with-bittorren_amd", "make-chunks")
    env = _env_without_knob()
    cts, out = [], ""
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        r = subprocess.run([cli, path], capture_output=True, text=True, env=env, timeout=300)
        cts.append(time.perf_counter() - t0)
        if r.returncode != 0:
            raise RuntimeError(f"make-chunks rc {r.returncode}: {r.stderr[-300:]}")
        out = r.stdout
    lines = out.splitlines()
    cli_ok = lines == [f"{i} {d[i].tobytes().hex()}" for i in range(n)]
    blocks = [hashlib.sha1(d[b * 4096:(b + 1) * 4096].tobytes()).hexdigest() == golden["weak4096"][b]
              for b in range(n // 4096) if b < len(golden["weak4096"])]
    samples = {int(k): v for k, v in golden["config3"]["sample"].items() if int(k) < n}
    samp_ok = all(d[k].tobytes().hex() == v for k, v in samples.items())
    whole = n % 4096 == 0 and len(blocks) == n // 4096
    parity = bool(len(d) == n and cli_ok and all(blocks) and samp_ok and whole)
    sec, csec = float(np.median(ts)), float(np.median(cts[1:]))
    return ({"workload": f"make-chunks on a {size} B file ({n} x 512 KiB: chunks 0..{n - 1} of the config-3 "
                         "corpus) in the page cache",
             "chunks": n, "bytes": size,
             "in_process": {"path": "make_chunks -> sha1chunk_hash_fd (pread ring -> H2D -> kernel -> D2H)",
                            "seconds": round(sec, 4), "runs_s": [round(t, 4) for t in ts],
                            "GiBps": round(size / sec / 2**30, 2)},
             "cli": {"path": "make-chunks <file> (whole process: start, HIP init, hash, 16384 output lines)",
                     "seconds": round(csec, 4), "first_s": round(cts[0], 4),
                     "runs_s": [round(t, 4) for t in cts[1:]], "GiBps": round(size / csec / 2**30, 2)},
             "page_cache_read_GiBps": round(read_gibs, 2), "pinned_h2d_GiBps": h2d_gibps,
             "parity": parity,
             "parity_ref": f"digest-of-digests of each 4096-chunk block == golden weak4096[b] ({len(blocks)} "
                           f"blocks, all {n} digests; reference sha.c), {len(samples)} golden config3 samples, "
                           "CLI lines == in-process digests"},
            d)


def _master_verify_leg(path: str, digests, requests: int = 1000, seed: int = 6):
    """the sender's verify on GET (packet_handler.c:434 ->
    chunk.c:204-217 verify_chunk_hash: re-read and re-hash 512 KiB of the
    master file per request), `requests` GETs at seeded random indices of
    the file through tools/master_verify_bench (C, linked against
    libsha1chunk.so), one FILE* kept open, each call timed: the master index
    (default: the second verify against a file builds a digest table in one
    streamed device pass, later GETs are lookups) and the per-call path
    (SHA1CHUNK_MASTER_INDEX=0: read + host hash per GET, the default routing
    of one message).  verify_chunk_hash exits(-1) on a mismatch, so a
    finished run verified every GET against the expected digests (the file
    leg's, golden-checked); a run with wrong digests must exit 255."""
    import subprocess
    import tempfile
    tool = os.path.join(ROOT, "tools", "master_verify_bench")
    if not os.path.exists(tool):
        return {"error": "tools/master_verify_bench not built (make -C congestion-control-with-bittorren_amd "
                         "tools)"}, None
    n = len(digests)
    idx = np.random.default_rng(seed).integers(0, n, requests)
    reqs = [(int(i), digests[int(i)].tobytes().hex()) for i in idx]
    # the master index serves a file only once its last change is older than
    # SHA1CHUNK_MASTER_SETTLE_MS (default 2 s, chunk.c rewrite guard)
    age = time.time() - os.stat(path).st_ctime
    if age < 2.2:
        time.sleep(2.2 - age)
    out = {"workload": f"{requests} verify_chunk_hash GETs at seeded random indices of the {n}-chunk file, "
                       "one FILE* (a send session's master file, reliable_udp.c:180)",
           "requests": requests}
    with tempfile.TemporaryDirectory() as td:
        rq = os.path.join(td, "req.txt")
        with open(rq, "w") as f:
            f.writelines(f"{i} {h}\n" for i, h in reqs)
        for name, extra in (("index", {}), ("per_call", {"SHA1CHUNK_MASTER_INDEX": "0"})):
            js = os.path.join(td, f"{name}.json")
            r = subprocess.run([tool, path, rq, js], capture_output=True, text=True,
                               env=_env_without_knob(extra), timeout=300)
            if r.returncode != 0 or not os.path.exists(js):
                out[name] = {"error": f"rc {r.returncode}: {r.stderr[-300:]}"}
                continue
            out[name] = json.load(open(js))
        out["index"]["path"] = "second GET builds the file's digest table (one streamed device pass); later " \
                               "GETs are lookups"
        out["per_call"]["path"] = "SHA1CHUNK_MASTER_INDEX=0: fseek + fread 512 KiB + shahash on the host per GET"
        bad = os.path.join(td, "bad.txt")
        with open(bad, "w") as f:
            f.writelines(f"{reqs[0][0]} {'0' * 40}\n" for _ in range(3))
        r = subprocess.run([tool, path, bad, os.path.join(td, "bad.json")], capture_output=True, text=True,
                           env=_env_without_knob(), timeout=120)
        out["mismatch_exits"] = r.returncode == 255 and "Unmatched chunk hashes" in r.stderr
    i, p = out.get("index", {}), out.get("per_call", {})
    if i.get("rest_median_ms") and p.get("rest_median_ms"):
        out["index_speedup_vs_per_call"] = round(p["rest_median_ms"] / i["rest_median_ms"], 1)
    out["parity"] = bool(i.get("verified") == requests and p.get("verified") == requests and out["mismatch_exits"])
    out["parity_ref"] = "every GET verified by verify_chunk_hash itself (exit(-1) on mismatch) against the file " \
                        "leg's golden-checked digests; wrong digests exit 255"
    return out, reqs


def _reference_master_verify(path: str, reqs, requests: int = 200) -> dict:
    """The reference chunk.c's verify_chunk_hash (+ sha.c, utility.c,
    packet.c; our timing main, tools/master_verify_bench.c) built from its
    sources into oracle/_ref with its Makefile's flags and at -O2, `requests`
    GETs each.  Indices below 8192 only: the reference seeks through a
    uint32_t offset (chunk.c:193), which wraps past 4 GiB."""
    import subprocess
    import tempfile
    sub = [(i, h) for i, h in reqs if i < 8192][:requests]
    out = {"requests": len(sub), "note": "indices < 8192 (chunk.c:193 seeks via a uint32_t offset)"}
    with tempfile.TemporaryDirectory() as td:
        rq = os.path.join(td, "req.txt")
        with open(rq, "w") as f:
            f.writelines(f"{i} {h}\n" for i, h in sub)
        for k, exe in (("O0", "master_verify_ref"), ("O2", "master_verify_ref_O2")):
            tool = os.path.join(ROOT, "oracle", "_ref", exe)
            js = os.path.join(td, f"{k}.json")
            if not os.path.exists(tool):
                out[k] = {"error": f"oracle/_ref/{exe} not built"}
                continue
            r = subprocess.run([tool, path, rq, js], capture_output=True, text=True, timeout=300)
            out[k] = json.load(open(js)) if r.returncode == 0 and os.path.exists(js) else \
                {"error": f"rc {r.returncode}: {r.stderr[-200:]}"}
    out["O0"]["build"] = "reference Makefile flags (-g, no -O)"
    out["O2"]["build"] = "-O2"
    return out


def _reference_file_cli(path: str, chunks: int = 1024) -> dict:
    """The reference's own make-chunks (oracle/_ref, its Makefile's flags) on
    the first `chunks` chunks of the file leg's file (a bounded sample: the
    whole 8 GiB would take ~25 s at -O0)."""
    import subprocess
    import tempfile
    fd, sp = tempfile.mkstemp(prefix="sha1bench_ref_", suffix=".dat")
    try:
        with os.fdopen(fd, "wb") as o, open(path, "rb") as f:
            o.write(f.read(chunks * CHUNK_LEN))
        exe = os.path.join(ROOT, "oracle", "_ref", "make-chunks")
        t0 = time.perf_counter()
        r = subprocess.run([exe, sp], capture_output=True, text=True, timeout=300)
        sec = time.perf_counter() - t0
        if r.returncode != 0:
            return {"error": f"rc {r.returncode}"}
        return {"sample": f"first {chunks} chunks ({chunks * CHUNK_LEN} B) of the file leg's file",
                "seconds": round(sec, 3), "GiBps": round(chunks * CHUNK_LEN / sec / 2**30, 3),
                "lines": len(r.stdout.splitlines())}
    finally:
        os.unlink(sp)


def _env_without_knob(extra=None) -> dict:
    """The environment with the library's default routing (no
    SHA1CHUNK_HOST_SMALL), plus `extra`."""
    env = {k: v for k, v in os.environ.items() if k != "SHA1CHUNK_HOST_SMALL"}
    env.update(extra or {})
    return env


def _run_cli(argv, env_extra, reps):
    """Whole-process wall times (s) of `reps` runs of a CLI, and its stdout."""
    import subprocess
    env = _env_without_knob(env_extra)
    ts, out = [], None
    for _ in range(reps):
        t0 = time.perf_counter()
        r = subprocess.run(argv, capture_output=True, text=True, env=env, timeout=120)
        ts.append(time.perf_counter() - t0)
        if r.returncode != 0:
            raise RuntimeError(f"{argv[0]} rc {r.returncode}: {r.stderr[-300:]}")
        out = r.stdout
    return ts, out


def _cli_rows_ok(stdout: str, golden) -> bool:
    rows = [line.split() for line in stdout.strip().splitlines()]
    return [r[1] for r in rows] == golden["fixtures"]["C.chunks_file"] and \
        [int(r[0]) for r in rows] == list(range(len(rows)))


def _ctar_file() -> str:
    import gzip
    import tempfile
    path = os.path.join(tempfile.gettempdir(), f"sha1bench_C_{os.getpid()}.tar")
    with gzip.open(os.path.join(ROOT, "tests/golden/C.tar.gz")) as f, open(path, "wb") as o:
        o.write(f.read())
    return path


def _config1_leg(golden, reps: int = 7) -> dict:
    """BASELINE config 1: `make-chunks tmp/C.tar` (make_chunks.c:14-62 ->
    chunk.c:15-27), the repo's CLI as a whole process, first run and median
    of the rest: the library's default routing (a regular file of <= 4 MiB
    is hashed on the host, csrc/frontend.c), the kernels
    (SHA1CHUNK_HOST_SMALL=0) and the explicit knob at the file's size.
    Output must equal the reference's tmp/C.chunks (CRLF stripped).  The
    reference's own CLI is timed in cpu_baseline."""
    path = _ctar_file()
    cli = os.path.join(ROOT, "congestion-control-with-bittorren_amd", "make-chunks")
    res = {"workload": "BASELINE config 1: make-chunks tmp/C.tar (2 MiB, 4 chunks), whole process",
           "file_bytes": os.path.getsize(path)}
    try:
        for name, env in (("default", {}), ("device", {"SHA1CHUNK_HOST_SMALL": "0"}),
                          ("host_small", {"SHA1CHUNK_HOST_SMALL": str(os.path.getsize(path))})):
            ts, out = _run_cli([cli, path], env, reps)
            res[name] = {"first_ms": round(ts[0] * 1e3, 3),
                         "median_ms": round(float(np.median(ts[1:])) * 1e3, 3),
                         "parity": _cli_rows_ok(out, golden)}
        res["default"]["route"] = "host (regular file <= 4 MiB, the library's default)"
        res["device"]["route"] = "gfx950 kernels (SHA1CHUNK_HOST_SMALL=0)"
        res["parity"] = all(res[k]["parity"] for k in ("default", "device", "host_small"))
    finally:
        os.unlink(path)
    return res


def _traffic(n: int, L: int):
    """HBM bytes per launch from the committed rocprofv3 PMC pass (FETCH_SIZE
    x2 gfx950 correction + WRITE_SIZE), if one was recorded for this shape."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*.json")), reverse=True):
        try:
            rec = json.load(open(path))
        except Exception:
            continue
        if rec.get("chunks") == n and rec.get("chunk_bytes") == L and "bytes_per_launch" in rec:
            return rec["bytes_per_launch"]
    return None


def usable_cores() -> dict:
    """Host cores this process may use: the CPU affinity mask, capped by the
    cgroup CPU quota (v2 cpu.max or v1 cfs_quota_us / cfs_period_us), with
    how it was derived and the CPU model."""
    import math
    aff = len(os.sched_getaffinity(0))
    quota, src = None, "no cgroup CPU quota"
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota, src = int(q) / int(per), f"cgroup v2 cpu.max {q}/{per}"
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota, src = q / per, f"cgroup v1 cfs {q}/{per}"
        except (OSError, ValueError):
            pass
    usable = aff if quota is None else max(1, min(aff, math.floor(quota)))
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"usable": usable, "affinity": aff, "os_cpu_count": os.cpu_count(),
            "quota_cpus": quota, "derivation": f"min(sched_getaffinity {aff}, {src})",
            "cpu_model": model}


def _cpu_baseline(O, n, L, golden, max_threads=None) -> dict:
    """The reference sha.c (oracle/_ref) on this host's cores over the same
    synthetic chunks as config 2 (chunks 0..4095, generated once): built -O2
    and with the reference Makefile's own flags (-g, no -O; Makefile:3), each
    on 1 thread and on every usable core (chunk-strided pthreads), then the
    repo's restatement (oracle/sha1_oracle.c) the same four ways; every row's
    digests checked against the reference golden file.  `value` is the
    reference -O2 all-cores row.  Also the peer's per-chunk verify on one
    core."""
    cores = usable_cores()
    allc = cores["usable"] if max_threads is None else max(1, min(cores["usable"], max_threads))
    sample = min(n, 4096)
    data = O.synth_chunks(0, sample, L)
    off = np.arange(sample, dtype=np.uint64) * L
    ln = np.full(sample, L, np.uint32)
    want = np.fromfile(os.path.join(ROOT, "tests/golden/synth_4096x512k.bin"),
                       np.uint8).reshape(-1, 20)[:sample] if L == O.CHUNK_LEN else None
    rows = []
    # the reference sha.c (kind "reference") on the whole sample; the repo's
    # restatement (kind "port") on 1 thread over its first 1024
    # chunks only, to keep the leg short
    for kind in ("reference", "port"):
        for opt in ("O2", "O0"):
            for threads in (1, allc):
                m = sample if kind == "reference" or threads > 1 else min(sample, 1024)
                times, ok = [], True
                # at least ~2 s of wall per row (one pass at 1 thread)
                while len(times) < 5 and sum(times) < 2.0:
                    secs, dig = O.time_batch(data[:m * L], off[:m], ln[:m], threads, opt, kind)
                    times.append(secs)
                    ok &= want is not None and bool(np.array_equal(dig, want[:m]))
                secs = float(np.median(times))
                rows.append({"kind": kind,
                             "build": "-O2" if opt == "O2" else "reference Makefile flags (-g, -O0)",
                             "threads": threads, "chunks": m, "seconds": round(secs, 4), "passes": len(times),
                             "GiBps": round(m * L / secs / 2**30, 4), "parity": ok})
    one = [O.time_batch(data[i * L:(i + 1) * L], off[:1], ln[:1], 1, "O2")[0] for i in range(16)]
    head = rows[1]
    return {"value": head["GiBps"], "unit": "GiB/s", "cores": head["threads"], "kind": "reference",
            "sample": f"chunks 0..{sample - 1} x {L} B of the config-2 corpus, reference sha.c -O2, "
                      f"{head['threads']} pthreads chunk-strided (every usable core), median of "
                      f"{head['passes']} passes; digests match reference golden: {head['parity']}",
            "rows": rows, "cores_usable": cores["usable"], "cores_derivation": cores,
            "parity": all(r["parity"] for r in rows),
            "one_chunk_ms": round(float(np.median(one)) * 1e3, 3)}


def _reference_cli(golden, reps: int = 7) -> dict:
    """The reference's own make-chunks (make_chunks.c chunk.c sha.c utility.c
    packet.c with its Makefile flags, built from its sources into
    oracle/_ref) on tmp/C.tar: BASELINE config 1's CPU baseline."""
    path = _ctar_file()
    try:
        ts, out = _run_cli([os.path.join(ROOT, "oracle", "_ref", "make-chunks"), path], {}, reps)
    finally:
        os.unlink(path)
    return {"first_ms": round(ts[0] * 1e3, 3), "median_ms": round(float(np.median(ts[1:])) * 1e3, 3),
            "parity": _cli_rows_ok(out, golden)}


if __name__ == "__main__":
    main()
