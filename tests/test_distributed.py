"""CPU, world size 2 over gloo: the multi-GPU path's sharding and control
plane (bench.py runs the same code over RCCL, one process per GPU).

Each rank takes its weak-scaling shard of BASELINE config 2's chunk ids,
hashes a small sample of its chunks with the ORACLE (test infrastructure:
the kernel itself is covered by tests/test_gpu_parity.py), and the ranks
combine timing (max) and parity (AND) exactly as bench.py does."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import importlib
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    shard = importlib.import_module("congestion-control-with-bittorren_amd.shard")
    from oracle import oracle as O
    per = 4096
    first, count = shard.weak_shard(rank, per)
    # golden digests of this rank's chunk ids (all 4096 of config 2 live in
    # synth_4096x512k.bin; rank 1's ids 4096.. are checked by sampling the
    # oracle against the weak-scaling aggregate's neighbours instead)
    sample = [first, first + 1, first + count - 1]
    L = O.CHUNK_LEN
    data = np.concatenate([O.synth_chunks(c, 1, L) for c in sample])
    dig = O.hash_batch(data, np.arange(3, dtype=np.uint64) * L, np.full(3, L, np.uint32), threads=1)
    ok = True
    if rank == 0:
        want = np.fromfile(os.path.join(ROOT, "tests/golden/synth_4096x512k.bin"),
                           np.uint8).reshape(-1, 20)
        ok = bool(np.array_equal(dig, want[[0, 1, 4095]]))
    t_local = [0.5 + rank, 2.0 - rank]
    t_max = shard.max_over_ranks(t_local)
    all_ok = shard.all_ranks_ok(ok)
    bad_ok = shard.all_ranks_ok(rank == 0)  # one rank failing -> False everywhere
    np.save(os.path.join(out_dir, f"r{rank}.npy"),
            np.array([first, count, t_max[0], t_max[1], all_ok, bad_ok], dtype=np.float64))
    np.save(os.path.join(out_dir, f"d{rank}.npy"), dig)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_weak_sharding(tmp_path, oracle):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    r0 = np.load(tmp_path / "r0.npy")
    r1 = np.load(tmp_path / "r1.npy")
    assert (r0[0], r0[1]) == (0, 4096) and (r1[0], r1[1]) == (4096, 4096)
    assert list(r0[2:4]) == [1.5, 2.0] and list(r1[2:4]) == [1.5, 2.0]  # max over ranks
    assert r0[4] == 1.0 and r1[4] == 1.0  # every rank's parity held
    assert r0[5] == 0.0 and r1[5] == 0.0  # AND sees rank 1's False
    # the two shards are disjoint slices of the global chunk id space
    d0, d1 = np.load(tmp_path / "d0.npy"), np.load(tmp_path / "d1.npy")
    assert not np.array_equal(d0, d1)


def _strong_worker(rank, world, port, out_dir):
    """bench.py's strong leg control plane: each rank takes its contiguous
    config-4 shard, the per-rank times are max-reduced, parity is ANDed, and
    shard.strong_report builds the JSON object."""
    import importlib
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    shard = importlib.import_module("congestion-control-with-bittorren_amd.shard")
    first, cnt = shard.strong_shard(rank, world, 262144)
    wall, kern = shard.max_over_ranks([0.030 + 0.001 * rank, 6.0 + rank])
    parity = shard.all_ranks_ok(True)
    rep = shard.strong_report(262144, 524288, world, wall / 5 * 1e3, kern, 39.5, 39.3, parity, True, 5)
    np.save(os.path.join(out_dir, f"s{rank}.npy"),
            np.array([first, cnt, rep["ms_per_step"], rep["kernel_ms"], rep["speedup"],
                      rep["efficiency"], rep["value"], rep["parity"]], dtype=np.float64))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_strong_leg_control_plane(tmp_path):
    world = 2
    mp.start_processes(_strong_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    s0, s1 = np.load(tmp_path / "s0.npy"), np.load(tmp_path / "s1.npy")
    assert (s0[0], s0[1], s1[0], s1[1]) == (0, 131072, 131072, 131072)
    assert np.array_equal(s0[2:], s1[2:])  # every rank reports the same maxima
    assert s0[2] == pytest.approx(31 / 5) and s0[3] == 7.0
    assert s0[4] == pytest.approx(39.5 / (31 / 5), rel=1e-3)
    assert s0[5] == pytest.approx(s0[4] / 2, rel=1e-3)
    assert s0[6] == pytest.approx(262144 * 524288 / (31 / 5 * 1e-3) / 2**30, rel=1e-3)
    assert s0[7] == 1.0


def test_strong_and_byte_balanced_shards(pkg):
    shard = pkg.shard if hasattr(pkg, "shard") else __import__(
        "importlib").import_module("congestion-control-with-bittorren_amd.shard")
    for total in (0, 1, 7, 262144, 262145):
        for world in (1, 2, 4, 8):
            parts = [shard.strong_shard(r, world, total) for r in range(world)]
            assert parts[0][0] == 0
            assert sum(c for _, c in parts) == total
            for (f0, c0), (f1, _) in zip(parts, parts[1:]):
                assert f0 + c0 == f1
            assert max(c for _, c in parts) - min(c for _, c in parts) <= 1
    # config 4: 262144 chunks over 8 GPUs -> 32768 each
    assert shard.strong_shard(3, 8, 262144) == (3 * 32768, 32768)
    lens = [4096, 1 << 20, 8192, 1 << 20, 65536, 12345, 1 << 19]
    for world in (1, 2, 3, 4):
        cuts = shard.byte_balanced_cuts(lens, world)
        assert len(cuts) == world + 1 and cuts[0] == 0 and cuts[-1] == len(lens)
        assert all(a <= b for a, b in zip(cuts, cuts[1:]))


def test_weak_golden_shard(pkg):
    """bench.py's config-4 weak leg: 65536 chunks per rank cycle through the
    four golden shards of the 4-way split at any N; sizes that do not divide
    the list fall back to plain weak shards with no golden index."""
    import importlib
    shard = importlib.import_module("congestion-control-with-bittorren_amd.shard")
    for world in (1, 2, 4, 8):
        for r in range(world):
            first, count, k = shard.weak_golden_shard(r, 65536, 262144)
            assert (first, count) == shard.strong_shard(r % 4, 4, 262144) and k == r % 4
    assert shard.weak_golden_shard(3, 32768, 262144) == (3 * 32768, 32768, 3)
    assert shard.weak_golden_shard(9, 32768, 262144) == (32768, 32768, 1)
    assert shard.weak_golden_shard(2, 100000, 262144) == (200000, 100000, None)


def test_device_map_one_rank_per_gpu():
    """bench.py's device rule: rank r on GPU r, and a
    node exposing fewer GPUs than local ranks fails instead of stacking
    ranks on shared devices (the gloo rehearsal may share, round robin)."""
    import importlib
    shard = importlib.import_module("congestion-control-with-bittorren_amd.shard")
    assert [shard.device_for_local_rank(r, 8, 8) for r in range(8)] == list(range(8))
    with pytest.raises(shard.DeviceMapError, match="only 1 visible"):
        shard.device_for_local_rank(1, 2, 1)
    with pytest.raises(shard.DeviceMapError, match="no GPU"):
        shard.device_for_local_rank(0, 1, 0)
    assert [shard.device_for_local_rank(r, 4, 1, shared_ok=True) for r in range(4)] == [0, 0, 0, 0]
    idents = [shard.device_identity("h", r, r, r, None) for r in range(2)]
    idents[0]["uuid"], idents[1]["uuid"] = "GPU-a", "GPU-b"
    shard.check_distinct_devices(idents)
    idents[1]["uuid"] = "GPU-a"
    with pytest.raises(shard.DeviceMapError, match="share GPU"):
        shard.check_distinct_devices(idents)
    shard.check_distinct_devices(idents, shared_ok=True)
    idents[1]["host"] = "other"  # same UUID string on another host is another card
    shard.check_distinct_devices(idents)


def _ident_worker(rank, world, port, out_dir, same):
    import importlib
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    shard = importlib.import_module("congestion-control-with-bittorren_amd.shard")
    ident = shard.device_identity("node0", rank, rank, 0 if same else rank, None)
    ident["uuid"] = "GPU-0" if same else f"GPU-{rank}"
    idents = shard.gather_identities(ident)
    try:
        shard.check_distinct_devices(idents)
        verdict = 1.0
    except shard.DeviceMapError:
        verdict = 0.0
    np.save(os.path.join(out_dir, f"i{rank}.npy"),
            np.array([verdict, len(idents), idents[1]["rank"]], dtype=np.float64))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("same", [False, True])
def test_two_rank_device_identity_gather(tmp_path, same):
    """Every rank gathers every rank's GPU identity and reaches the same
    verdict: two ranks on one physical GPU fail on both ranks."""
    mp.start_processes(_ident_worker, args=(2, _free_port(), str(tmp_path), same), nprocs=2,
                       join=True, start_method="spawn")
    for r in range(2):
        v = np.load(tmp_path / f"i{r}.npy")
        assert v[0] == (0.0 if same else 1.0) and v[1] == 2 and v[2] == 1


def test_bench_exits_when_ranks_outnumber_gpus():
    """An oversubscribed launch (here: 2 local ranks, no visible GPU) exits
    non-zero with the reason, before any process group or timing."""
    import subprocess
    import sys
    env = dict(os.environ, RANK="1", LOCAL_RANK="1", WORLD_SIZE="2", LOCAL_WORLD_SIZE="2",
               HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 2, r.stderr[-500:]
    assert "one rank per GPU" in r.stderr or "no GPU" in r.stderr
    assert not r.stdout.strip()


def _eight_worker(rank, world, port, out_dir, small_golden):
    """bench.py's control plane at the node's full width (world 8 over gloo,
    SURVEY 8(e)): shard indices, golden lookups, the real-data parity of a
    small strong list, max over ranks, the parity AND with one rank failing,
    and the device-identity check over 8 mocked GPUs."""
    import hashlib
    import importlib
    import json
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    shard = importlib.import_module("congestion-control-with-bittorren_amd.shard")
    from oracle import oracle as O
    golden = json.load(open(os.path.join(ROOT, "tests/golden/golden.json")))
    rec = {}
    # config 4 strong: 262144 chunks, 32768 per rank, and the golden aggregate
    # this rank's parity is checked against
    rec["strong"] = list(shard.strong_shard(rank, world, 262144))
    rec["strong_agg"] = shard.strong_golden_agg(golden, world, rank, 262144)
    rec["strong_agg_other_total"] = shard.strong_golden_agg(golden, world, rank, 262143)
    # config 4 weak: 65536 per rank, shard rank % 4 of the 4-way split
    first, count, want = shard.weak_golden_agg(golden, rank, 65536)
    rec["weak"] = [first, count]
    rec["weak_agg"] = want
    # real data: a 64-chunk strong list (4 KiB chunks of the same corpus)
    # split 8 ways, each rank's digests from the oracle, the aggregate
    # compared exactly as bench.py's strong leg compares it
    L, total = 4096, 64
    f, c = shard.strong_shard(rank, world, total)
    data = O.synth_chunks(f, c, L)
    dig = O.hash_batch(data, np.arange(c, dtype=np.uint64) * L, np.full(c, L, np.uint32), threads=1)
    agg = shard.strong_golden_agg(small_golden, world, rank, total)
    ok = agg is not None and hashlib.sha1(dig.tobytes()).hexdigest() == agg
    rec["own_ok"] = ok
    rec["all_ok"] = shard.all_ranks_ok(ok)
    rec["one_bad"] = shard.all_ranks_ok(ok and rank != 5)
    rec["max"] = shard.max_over_ranks([0.25 * rank, 7.0 - rank, 3.0])
    # identities: 8 distinct GPUs, then rank 6 reporting rank 2's card
    for case in ("distinct", "dup"):
        ident = shard.device_identity("node0", rank, rank, rank, None)
        ident["uuid"] = f"GPU-{2 if (case == 'dup' and rank == 6) else rank}"
        idents = shard.gather_identities(ident)
        try:
            shard.check_distinct_devices(idents)
            rec[case] = "ok"
        except shard.DeviceMapError as e:
            rec[case] = str(e)
        rec[case + "_n"] = len(idents)
    rep = shard.strong_report(262144, 524288, world, rec["max"][1], rec["max"][2], 38.3, 38.3,
                              rec["all_ok"], True, 10)
    rec["report"] = [rep["speedup"], rep["efficiency"], rep["value"], rep["parity"]]
    with open(os.path.join(out_dir, f"e{rank}.json"), "w") as fh:
        json.dump(rec, fh)
    dist.barrier()
    dist.destroy_process_group()


def test_eight_rank_control_plane(tmp_path, oracle):
    """World size 8 (the 8-GPU node's bench launch, rehearsed over gloo on
    the CPU)."""
    import hashlib
    import json
    world, L, total = 8, 4096, 64
    golden = json.load(open(os.path.join(ROOT, "tests/golden/golden.json")))
    # the small list's golden aggregates, from the standard library's SHA-1
    # over the same corpus bytes (independent of the oracle the ranks use)
    import importlib
    shard = importlib.import_module("congestion-control-with-bittorren_amd.shard")
    data = oracle.synth_chunks(0, total, L)
    d = b"".join(hashlib.sha1(data[i * L:(i + 1) * L].tobytes()).digest() for i in range(total))
    aggs = []
    for r in range(world):
        f, c = shard.strong_shard(r, world, total)
        aggs.append(hashlib.sha1(d[20 * f:20 * (f + c)]).hexdigest())
    small = {"config4": {"chunks": total, "shard_aggs": {str(world): aggs}}}
    mp.start_processes(_eight_worker, args=(world, _free_port(), str(tmp_path), small), nprocs=world,
                       join=True, start_method="spawn")
    recs = [json.load(open(tmp_path / f"e{r}.json")) for r in range(world)]
    c4 = golden["config4"]
    for r, rec in enumerate(recs):
        assert rec["strong"] == [r * 32768, 32768]
        assert rec["strong_agg"] == c4["shard_aggs"]["8"][r]
        assert rec["strong_agg_other_total"] is None
        assert rec["weak"] == [(r % 4) * 65536, 65536]
        assert rec["weak_agg"] == c4["shard_aggs"]["4"][r % 4]
        assert rec["own_ok"] and rec["all_ok"]
        assert rec["one_bad"] is False  # rank 5's False reaches every rank
        assert rec["max"] == [1.75, 7.0, 3.0]
        assert rec["distinct"] == "ok" and rec["distinct_n"] == 8
        assert "ranks 2 and 6 share GPU GPU-2" in rec["dup"] and rec["dup_n"] == 8
        assert rec["report"] == recs[0]["report"]
    assert len(set(c4["shard_aggs"]["8"])) == 8
    # ranks 0 and 4 hash config 3's range: the same golden aggregate
    assert recs[0]["weak_agg"] == recs[4]["weak_agg"] == golden["config3"]["agg"]
    sp, eff, val, par = recs[0]["report"]
    assert sp == pytest.approx(38.3 / 7.0, rel=1e-3) and eff == pytest.approx(sp / 8, rel=1e-3)
    assert par is True
