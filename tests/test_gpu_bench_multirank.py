"""bench.py's multi-GPU path (one process per GPU, torch.distributed.run),
rehearsed with 2 ranks on the one GPU of the test box over gloo
(SHA1_BENCH_DIST_BACKEND=gloo; RCCL refuses two ranks on one device).

Weak leg: each rank hashes its own 4096 chunks of config 2 (global ids
4096 r ..) and checks the digest-of-digests against the reference golden
aggregate; strong leg: BASELINE config 4's 262144 chunks split in two
contiguous shards, each checked against the golden shard aggregate of the
2-way split, plus the whole list on rank 0 against the golden aggregate;
config-4 weak leg: 65536 chunks per rank, rank r checked against the golden
shard r of the 4-way split.  The JSON line is rank 0's; both parities are ANDed over ranks."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_weak_and_strong(pkg):
    env = dict(os.environ, SHA1_BENCH_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", "3", "--warmup", "1", "--strong-steps", "1", "--no-latency", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["parity"] is True and d["scaling"] == "weak"
    assert d["value"] > 0 and d["roofline"]["frac"] > 0
    st = d["strong"]
    assert st["n_gpus"] == 2 and st["chunks_per_gpu"] == 131072 and st["chunks_total"] == 262144
    assert st["parity"] is True and st["one_gpu_parity"] is True
    assert st["speedup"] > 0 and st["efficiency"] == pytest.approx(st["speedup"] / 2, rel=1e-3)
    w4 = d["weak_config4"]
    assert w4["n_gpus"] == 2 and w4["chunks_per_gpu"] == 65536 and w4["parity"] is True
    assert w4["value"] == pytest.approx(2 * 65536 * 524288 / 2**30 / (w4["ms_per_step"] / 1e3), rel=1e-3)


def test_bench_rccl_control_plane_one_rank(pkg):
    """The RCCL control plane bench.py uses on an 8-GPU node (process group
    over "nccl" = RCCL with device_id, barrier, all_reduce MAX of the times,
    all_reduce MIN of the parity flags), run at world size 1 on the test box
    (SHA1_BENCH_FORCE_PG=1 under torch.distributed.run): same JSON line,
    parity on every leg."""
    env = dict(os.environ, SHA1_BENCH_FORCE_PG="1")
    env.pop("SHA1_BENCH_DIST_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--steps", "3", "--warmup", "1", "--strong-steps", "1", "--no-latency", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["config"]["control_plane"] == "torch.distributed nccl, world 1"
    assert d["n_gpus"] == 1 and d["parity"] is True and d["value"] > 0
    assert d["strong"]["parity"] is True and d["weak_config4"]["parity"] is True
