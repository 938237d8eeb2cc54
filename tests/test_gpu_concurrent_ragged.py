"""Device-resident ragged batches from several threads at once, each on its
own stream: every AUTO call sorts its batch, checks its layout and plans it
in stream-ordered scratch of its own (sha1_sort.hip, plan_layout_kernel,
plan_mixed_kernel), then runs the persistent mixed kernel, whose workgroups
pull jobs from that call's own counter -- so concurrent calls must neither
share scratch nor wait on each other's workgroups.  More groups than CUs
(the mixed path), mixed lengths, chunks scattered over the buffer; every
digest against a single-stream run, a sample against hashlib."""
import hashlib
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(pkg):
    import torch
    assert torch.cuda.is_available(), "GPU tests need a device"
    torch.cuda.set_device(0)
    pkg.set_device(0)
    return torch


def _batch(rng, cus, k):
    n = 64 * (cus + 40 + 7 * k) - 13  # more groups than CUs: the mixed kernel
    lens = rng.integers(0, 9000, n).astype(np.uint32)
    lens[rng.choice(n, 2 * cus, replace=False)] = rng.integers(20000, 60000, 2 * cus)
    step = (lens.astype(np.uint64) + 15) // 16 * 16
    perm = rng.permutation(n)
    off = np.zeros(n, np.uint64)
    off[perm] = np.concatenate([[0], np.cumsum(step[perm])[:-1]]).astype(np.uint64)
    host = rng.integers(0, 256, int((off + lens).max()) + 64, dtype=np.uint8)
    return host, off, lens


def test_concurrent_ragged_streams(pkg, dev, monkeypatch):
    torch = dev
    for k in ("SHA1CHUNK_MIXED_PLAN", "SHA1CHUNK_MIXED", "SHA1CHUNK_MIXED_DEBUG", "SHA1CHUNK_FORCE_KERNEL"):
        monkeypatch.delenv(k, raising=False)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    rng = np.random.default_rng(2718)
    jobs = []
    for k in range(4):
        host, off, lens = _batch(rng, cus, k)
        d = (torch.from_numpy(host).cuda(), torch.from_numpy(off.astype(np.int64)).cuda(),
             torch.from_numpy(lens.astype(np.int32)).cuda())
        want = torch.zeros((lens.size, 20), dtype=torch.uint8, device="cuda")
        pkg.hash_device(*d, want)  # alone, on the default stream
        torch.cuda.synchronize()
        jobs.append((host, off, lens, d, want.cpu().numpy()))
    errors = []

    def work(k):
        try:
            host, off, lens, d, want = jobs[k]
            st = torch.cuda.Stream()
            outs = []
            with torch.cuda.stream(st):
                for _ in range(6):
                    dig = torch.zeros((lens.size, 20), dtype=torch.uint8, device="cuda")
                    pkg.hash_device(*d, dig, stream=st)
                    outs.append(dig)
            st.synchronize()
            for dig in outs:
                got = dig.cpu().numpy()
                bad = np.flatnonzero((got != want).any(axis=1))
                assert bad.size == 0, (k, bad[:8])
        except Exception as e:  # noqa: BLE001 -- reported below with the thread
            errors.append((k, repr(e)))

    threads = [threading.Thread(target=work, args=(k,)) for k in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in threads), "a caller did not finish"
    assert not errors, errors
    for host, off, lens, _, want in jobs:
        for i in np.unique(np.linspace(0, lens.size - 1, 10).astype(np.int64)):
            o, L = int(off[i]), int(lens[i])
            assert hashlib.sha1(host[o:o + L].tobytes()).digest() == want[i].tobytes()
