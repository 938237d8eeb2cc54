"""sha1chunk_receive_cpus (include/sha1chunk.h): the CPUs a verify queue's
receive thread should run on -- one L3 domain of the GPU's NUMA node per
receive thread ("Verify queue placement").  Checked
against the box's own sysfs: the domains partition the node's allowed CPUs,
each is exactly a shared_cpu_list (within the allowed node CPUs), slots wrap
round robin, and SHA1CHUNK_NUMA=off widens them to every allowed CPU."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cpulist(text):
    out = set()
    for piece in text.strip().split(","):
        if not piece:
            continue
        a, _, b = piece.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


def _read(path):
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return ""


def _node_cpus(bdf):
    node = _read(f"/sys/bus/pci/devices/{bdf.lower()}/numa_node").strip()
    if not node or int(node) < 0:
        return None
    return _cpulist(_read(f"/sys/devices/system/node/node{int(node)}/cpulist"))


@pytest.fixture(scope="module", autouse=True)
def dev(pkg):
    # torch's HIP runtime first, as every GPU test module does: the library's
    # backend then shares the process's already-loaded runtime
    import torch
    assert torch.cuda.is_available(), "GPU tests need a device"
    torch.cuda.set_device(0)
    pkg.set_device(0)
    return torch


def _domains(pkg, dev):
    first, n = pkg.sha1chunk.receive_cpus(dev, 0)
    return [pkg.sha1chunk.receive_cpus(dev, s)[0] for s in range(n)], n, first


def test_receive_cpus_partition_the_node(pkg):
    dev = 0
    doms, n, first = _domains(pkg, dev)
    assert n >= 1 and all(doms)
    allowed = os.sched_getaffinity(0)
    node = _node_cpus(pkg.sha1chunk.device_pci_bus_id(dev))
    base = allowed & node if node and allowed & node else allowed
    union = set()
    for d in doms:
        assert not union & set(d), "domains overlap"
        union |= set(d)
        # exactly its first CPU's L3 list (where sysfs has one), within base
        l3 = _read(f"/sys/devices/system/cpu/cpu{d[0]}/cache/index3/shared_cpu_list")
        if l3:
            assert set(d) == _cpulist(l3) & (base - (union - set(d)))
    assert union == base
    # round robin: slot n is slot 0 again; the domain count comes back each time
    again, n2 = pkg.sha1chunk.receive_cpus(dev, n)
    assert again == first and n2 == n
    assert pkg.sha1chunk.receive_cpus(dev, 2 * n + 1)[0] == doms[1 % n]


def test_receive_cpus_rejects_a_bad_device(pkg):
    with pytest.raises(pkg.Sha1ChunkError) as ei:
        pkg.sha1chunk.receive_cpus(pkg.sha1chunk.device_count() + 3, 0)
    assert ei.value.code == pkg.sha1chunk.EINVAL


def test_receive_cpus_numa_off_uses_every_allowed_cpu():
    """SHA1CHUNK_NUMA=off (read once per process): the domains of the whole
    affinity mask."""
    code = (
        "import json, os, sys; sys.path.insert(0, %r)\n"
        "import torch; assert torch.cuda.is_available()\n"
        "import importlib; pkg = importlib.import_module('congestion-control-with-bittorren_amd')\n"
        "first, n = pkg.sha1chunk.receive_cpus(0, 0)\n"
        "u = set()\n"
        "for s in range(n): u |= set(pkg.sha1chunk.receive_cpus(0, s)[0])\n"
        "print(json.dumps({'n': n, 'union': sorted(u), 'allowed': sorted(os.sched_getaffinity(0))}))\n"
    ) % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, SHA1CHUNK_NUMA="off"))
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["union"] == out["allowed"]
