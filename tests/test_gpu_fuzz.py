"""Seeded randomized parity: many small ragged batches through every kernel
and every split shape the library builds, bit-exact against the oracle
(oracle/sha1_oracle.c, pinned to the reference's golden vectors by
tests/test_oracle.py).  Lengths concentrate on the padding boundaries of
sha.c:536-543 (len % 64 in {55, 56, 63, 0}) and the 16-byte alignment the
bulk load paths depend on."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KERNELS = ["lane", "fused", "split", "auto"]
SPLIT_UNITS = [1, 4, 11]  # the product library's split shapes


def _lengths(rng, n):
    kind = rng.integers(0, 4, n)
    base = rng.integers(0, 3000, n) * 64
    edge = rng.choice(np.array([0, 1, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128]), n)
    lens = np.where(kind == 0, base + edge,                       # near block edges
           np.where(kind == 1, rng.integers(0, 200000, n),        # anything
           np.where(kind == 2, 65536 + rng.integers(-70, 70, n),  # long, near-equal
                    edge)))                                        # tiny
    return np.clip(lens, 0, None).astype(np.uint32)


@pytest.fixture(scope="module")
def dev(pkg):
    import torch
    assert torch.cuda.is_available(), "GPU tests need a device"
    torch.cuda.set_device(0)
    pkg.set_device(0)
    return torch


# SHA1CHUNK_FUZZ_SEEDS widens the run (the committed log profiles/fuzz_r01.log
# is one 200-seed pass on MI355X)
@pytest.mark.parametrize("seed", range(int(os.environ.get("SHA1CHUNK_FUZZ_SEEDS", "12"))))
def test_random_batches_every_kernel(pkg, dev, oracle, seed, monkeypatch):
    torch = dev
    rng = np.random.default_rng(7000 + seed)
    n = int(rng.integers(1, 400))
    lens = _lengths(rng, n)
    align = int(rng.choice([1, 4, 16, 64]))
    step = (lens.astype(np.uint64) + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align)
    step += rng.integers(0, 3, n).astype(np.uint64) * np.uint64(align)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(step)[: n - 1]
    off += np.uint64(int(rng.integers(0, 4)) * align)
    host = rng.integers(0, 256, int(off[-1] + lens[-1]) + 64, dtype=np.uint8)
    want = oracle.hash_batch(host, off, lens)
    d_host = torch.from_numpy(host).cuda()
    d_off = torch.from_numpy(off.astype(np.int64)).cuda()
    d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
    kernels = KERNELS + [f"split:{u}" for u in rng.choice(SPLIT_UNITS, 3, replace=False)]
    for k in kernels:
        if k.startswith("split:"):
            monkeypatch.setenv("SHA1CHUNK_SPLIT_UNIT", k.split(":")[1])
            name = "split"
        else:
            monkeypatch.delenv("SHA1CHUNK_SPLIT_UNIT", raising=False)
            name = k
        dig = torch.zeros((n, 20), dtype=torch.uint8, device="cuda")
        pkg.hash_device(d_host, d_off, d_len, dig, kernel=name)
        torch.cuda.synchronize()
        got = dig.cpu().numpy()
        bad = np.nonzero((got != want).any(axis=1))[0]
        assert bad.size == 0, f"seed {seed} kernel {k} n={n} align={align}: {bad.size} bad, " \
                              f"first {bad[:6]} lens {lens[bad[:6]]}"
    monkeypatch.delenv("SHA1CHUNK_SPLIT_UNIT", raising=False)
    # the host-memory path (pageable numpy): packing + pipeline
    got = pkg.hash_batch(host, off, lens)
    assert np.array_equal(got, want), f"seed {seed}: host batch"


# The mixed kernel (more groups of 64 than CUs, AUTO on a ragged device
# batch): random batches of mostly short chunks with a few long ones, in
# caller order or scrambled, each through the device plan, two random forced
# mode-0 plans and the 8-wave mode.
@pytest.mark.parametrize("seed", range(int(os.environ.get("SHA1CHUNK_FUZZ_SEEDS", "12")) // 3 + 1))
def test_random_batches_mixed_kernel(pkg, dev, oracle, seed, monkeypatch):
    torch = dev
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    rng = np.random.default_rng(9100 + seed)
    G = int(rng.integers(cus + 1, 5 * cus))
    n = 64 * G - int(rng.integers(0, 64))
    lens = _lengths(rng, n) % 4000
    lens[rng.choice(n, int(rng.integers(1, 3 * cus)), replace=False)] = rng.integers(20000, 90000)
    align = int(rng.choice([1, 16, 64]))
    step = (lens.astype(np.uint64) + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(step)[: n - 1]
    if rng.integers(0, 2):  # caller order scrambled: scattered groups
        perm = rng.permutation(n)
        off, lens = off[perm].copy(), lens[perm].copy()
    host = rng.integers(0, 256, int(off.max() + 90000) + 64, dtype=np.uint8)
    want = oracle.hash_batch(host, off, lens)
    d_host = torch.from_numpy(host).cuda()
    d_off = torch.from_numpy(off.astype(np.int64)).cuda()
    d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
    hcap = min(G, 4 * cus, 4096)
    plans = [None] + [f"0,{int(rng.choice([0, int(rng.integers(0, hcap + 1)), hcap, G]))},"
                      f"{int(rng.choice([4, 8]))}" for _ in range(2)] + ["1,0,0"]
    for p in plans:
        if p is None:
            monkeypatch.delenv("SHA1CHUNK_MIXED_PLAN", raising=False)
        else:
            monkeypatch.setenv("SHA1CHUNK_MIXED_PLAN", p)
        dig = torch.zeros((n, 20), dtype=torch.uint8, device="cuda")
        pkg.hash_device(d_host, d_off, d_len, dig)
        torch.cuda.synchronize()
        got = dig.cpu().numpy()
        bad = np.nonzero((got != want).any(axis=1))[0]
        assert bad.size == 0, f"seed {seed} plan {p or 'device'} n={n} align={align}: {bad.size} bad, " \
                              f"first {bad[:6]} lens {lens[bad[:6]]}"
    monkeypatch.delenv("SHA1CHUNK_MIXED_PLAN", raising=False)


# The receive path's verify queue (sha1chunk_vq_*, the batched verify_hash of
# job.c:217-228): random interleavings of submit / non-blocking poll / flush /
# partial drains with a small result buffer, random batch sizes, growth on or
# off and 1 or 4 copy threads (chunks above 64 KiB are copied in pieces by the
# copy pool).  Every tag must come back exactly once with verify_hash's 0/1,
# and pending must count what is still owed.
# Both queue implementations: batch launches and the persistent drain
# (SHA1CHUNK_VQ_MODE=persistent, with a 1 ms idle exit and a small ring so
# the drain leaves and is relaunched, and both rings wrap, within a test).
@pytest.mark.parametrize("mode", ["batch", "persistent"])
@pytest.mark.parametrize("seed", range(int(os.environ.get("SHA1CHUNK_FUZZ_SEEDS", "12")) // 2 + 1))
def test_random_verify_queue_interleavings(pkg, dev, oracle, seed, monkeypatch, mode):
    import time
    rng = np.random.default_rng(9900 + seed)
    monkeypatch.setenv("SHA1CHUNK_VQ_MODE", mode)
    monkeypatch.setenv("SHA1CHUNK_VQ_IDLE_MS", str(int(rng.choice([1, 20]))))
    monkeypatch.setenv("SHA1CHUNK_VQ_RING_MIB", str(int(rng.choice([8, 64]))))
    monkeypatch.setenv("SHA1CHUNK_VQ_GROW", str(int(rng.integers(0, 2))))
    monkeypatch.setenv("SHA1CHUNK_VQ_THREADS", str(int(rng.choice([1, 4]))))
    batch = int(rng.choice([1, 3, 8, 32, 100]))
    maxlen = int(rng.choice([200000, 524288]))
    n = int(rng.integers(1, 260))
    lens = np.minimum(_lengths(rng, n), maxlen)
    data = rng.integers(0, 256, int(lens.max()) + 4096, dtype=np.uint8)
    want, got, owed = {}, {}, 0
    with pkg.VerifyQueue(batch=batch, max_chunk_len=maxlen) as q:
        for t in range(n):
            start = int(rng.integers(0, 4096))
            chunk = data[start:start + int(lens[t])].tobytes()
            dig = oracle.shahash(chunk)
            bad = bool(rng.random() < 0.25)
            if bad:
                k = int(rng.integers(0, 20))
                dig = dig[:k] + bytes([dig[k] ^ (1 << int(rng.integers(0, 8)))]) + dig[k + 1:]
            tag = int(rng.integers(0, 1 << 62)) * 4 + t % 4  # sparse, unordered tags
            while tag in want:
                tag += 4
            want[tag] = int(bad)
            q.submit(chunk, dig, tag)
            owed += 1
            op = rng.random()
            if op < 0.3:
                res = q.poll(max_results=int(rng.integers(1, 8)))
            elif op < 0.4:
                q.flush()
                res = []
            elif op < 0.45:
                res = q.poll(wait=True, max_results=int(rng.integers(1, 64)))
            else:
                res = []
            for tg, m in res:
                assert tg not in got, f"seed {seed}: tag returned twice"
                got[tg] = m
            owed -= len(res)
            assert q.pending == owed
        t0 = time.time()
        while q.pending and time.time() - t0 < 60:
            res = q.poll(wait=bool(rng.integers(0, 2)), max_results=int(rng.integers(1, 50)))
            for tg, m in res:
                assert tg not in got, f"seed {seed}: tag returned twice"
                got[tg] = m
        assert q.pending == 0
    assert got == want, f"seed {seed} batch {batch} n {n}: " \
                        f"{sum(got.get(k) != v for k, v in want.items())} wrong"
