"""GPU: the devices the multi-device paths shard over are distinct physical
GPUs.  SHA1CHUNK_ALL_DEVICES (host batches) and
SHA1CHUNK_FILE_DEVICES (make_chunks) put one host thread on each logical
device; without the SHA1CHUNK_VIRTUAL_DEVICES test knob every logical device
is its own GPU, named by its PCI address."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import importlib, json, sys
sys.path.insert(0, sys.argv[1])
pkg = importlib.import_module("congestion-control-with-bittorren_amd")
n = pkg.device_count()
print(json.dumps([pkg.sha1chunk.device_pci_bus_id(d) for d in range(n)]))
"""


def _bus_ids(env_extra):
    env = {k: v for k, v in os.environ.items() if k != "SHA1CHUNK_VIRTUAL_DEVICES"}
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT], capture_output=True, text=True, env=env,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    import json
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
def test_all_devices_are_distinct_gpus(pkg):
    ids = _bus_ids({})
    assert ids and all(ids), ids
    if len(ids) < 2:
        pytest.skip(f"one GPU visible ({ids[0]}): nothing to tell apart")
    assert len(set(ids)) == len(ids), ids


@pytest.mark.gpu
def test_virtual_devices_share_the_physical_gpu(pkg):
    """The test knob maps logical device d to physical d % n, and the PCI
    address says so (how a shared GPU shows up)."""
    phys = _bus_ids({})
    virt = _bus_ids({"SHA1CHUNK_VIRTUAL_DEVICES": "3"})
    assert len(virt) == 3
    assert virt == [phys[d % len(phys)] for d in range(3)], (phys, virt)


@pytest.mark.gpu
def test_all_devices_batch_matches_golden(pkg, golden):
    """SHA1CHUNK_ALL_DEVICES over every visible GPU: the reference golden
    digests of config 2's first 256 chunks."""
    n, L = 256, pkg.sha1chunk.CHUNK_LEN
    import torch
    buf = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    pkg.synth_fill_device(buf, 0, n, L)
    torch.cuda.synchronize()
    host = buf.cpu().numpy()
    got = pkg.hash_batch(host, np.arange(n, dtype=np.uint64) * L, np.full(n, L, np.uint32),
                         all_devices=True)
    want = np.fromfile(os.path.join(ROOT, "tests/golden/synth_4096x512k.bin"), np.uint8).reshape(-1, 20)[:n]
    assert np.array_equal(got, want)
