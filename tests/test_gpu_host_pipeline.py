"""GPU parity of the host-batch pipeline (BASELINE config 3: chunk bytes start
and end in host memory -> pinned H2D + hash + D2H on two alternating slots).

The reference hashes a file's chunks one at a time from a host buffer
(chunk.c:15-27 fread + shahash, driven from make_chunks.c:47).  Here
sha1chunk_hash_batch takes the whole host batch and runs it through the
runtime's two-slot ring (csrc/sha1_runtime.hip hash_host / stage_and_launch):
 * pinned, contiguous chunks -> "direct" slots (one hipMemcpyAsync straight
   from the caller's memory, no host copy);
 * pageable chunks -> "packed" slots (pack threads copy into pinned staging);
 * ragged, byte-misaligned chunks -> packed at 128-byte device alignment.
Every case moves >= 2 GiB and fills the ring >= 3 times; the runtime's
SHA1CHUNK_HOST_DEBUG lines prove which mode and how many slot fills ran.
Digests are checked against the reference-generated golden vectors (every
digest where the golden set has them, the digest-of-digests otherwise).
"""
import os
import re
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
L512 = 524288
SLOT_RE = re.compile(r"sha1chunk host slot (\d): (\d+) chunks (\d+) bytes (direct|packed)")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(pkg):
    import torch
    assert torch.cuda.is_available(), "GPU tests need a device"
    assert pkg.device_count() >= 1, pkg.lib().sha1chunk_last_error()
    torch.cuda.set_device(0)
    pkg.set_device(0)
    return torch


def _fill_host_synth(pkg, torch, host_u8, first, n, step=4096):
    """host_u8[i*L512 : (i+1)*L512] = synthetic chunk first+i (SURVEY 8d corpus),
    generated on the device step chunks at a time and copied down."""
    d = torch.empty(step * L512, dtype=torch.uint8, device="cuda")
    for s in range(0, n, step):
        k = min(step, n - s)
        pkg.synth_fill_device(d, first + s, k, L512)
        host_u8[s * L512:(s + k) * L512].copy_(d[:k * L512])
    torch.cuda.synchronize()
    del d


def _slots(capfd):
    err = capfd.readouterr().err
    return [(int(a), int(m), int(b), mode) for a, m, b, mode in SLOT_RE.findall(err)]


def test_config3_pinned_direct_pipeline(pkg, dev, oracle, golden, capfd, monkeypatch):
    """All of config 3: 65536 x 512 KiB (32 GiB) in pinned host memory, one
    sha1chunk_hash_batch call.  The slots alternate 0/1, each a direct copy of
    a contiguous run of the caller's pinned buffer; every sampled digest and
    the digest-of-digests equal the reference's."""
    torch = dev
    n = 65536
    host = torch.empty(n * L512, dtype=torch.uint8, pin_memory=True)
    _fill_host_synth(pkg, torch, host, 0, n)
    arr = host.numpy()
    monkeypatch.setenv("SHA1CHUNK_HOST_DEBUG", "1")
    capfd.readouterr()
    t0 = time.perf_counter()
    got = pkg.hash_batch(arr, np.arange(n, dtype=np.uint64) * L512, np.full(n, L512, np.uint32))
    secs = time.perf_counter() - t0
    slots = _slots(capfd)
    print(f"config 3 pinned end-to-end: {n * L512 / secs / 2**30:.1f} GiB/s ({secs * 1e3:.0f} ms)")
    assert len(slots) >= 3 and all(s[3] == "direct" for s in slots), slots[:4]
    assert [s[0] for s in slots] == [i % 2 for i in range(len(slots))]
    assert sum(s[1] for s in slots) == n and sum(s[2] for s in slots) == n * L512
    for i, h in golden["config3"]["sample"].items():
        assert got[int(i)].tobytes().hex() == h, i
    want = np.fromfile(os.path.join(GOLDEN, "synth_4096x512k.bin"), np.uint8).reshape(-1, 20)
    assert np.array_equal(got[:4096], want)
    assert oracle.digest_of_digests(got).hex() == golden["config3"]["agg"]
    del arr, host


@pytest.mark.parametrize("slot_mib", ["256", None])
def test_pageable_packed_pipeline(pkg, dev, oracle, golden, capfd, monkeypatch, slot_mib):
    """8192 x 512 KiB (4 GiB) in ordinary pageable memory: every slot is
    packed by the pack threads into pinned staging.  256 MiB slots wrap the
    ring 16 times, the default (1 GiB) 4 times.  Every one of the first 4096
    digests and both 4096-chunk aggregates equal the reference's."""
    torch = dev
    n = 8192
    host = torch.empty(n * L512, dtype=torch.uint8)  # pageable
    _fill_host_synth(pkg, torch, host, 0, n)
    arr = host.numpy()
    monkeypatch.setenv("SHA1CHUNK_HOST_DEBUG", "1")
    if slot_mib:
        monkeypatch.setenv("SHA1CHUNK_HOST_SLOT_MIB", slot_mib)
    capfd.readouterr()
    got = pkg.hash_batch(arr, np.arange(n, dtype=np.uint64) * L512, np.full(n, L512, np.uint32))
    slots = _slots(capfd)
    expect_fills = n * L512 // ((int(slot_mib) << 20) if slot_mib else (1 << 30))
    assert len(slots) == expect_fills and all(s[3] == "packed" for s in slots), slots[:4]
    assert sum(s[1] for s in slots) == n
    want = np.fromfile(os.path.join(GOLDEN, "synth_4096x512k.bin"), np.uint8).reshape(-1, 20)
    assert np.array_equal(got[:4096], want)
    assert [oracle.digest_of_digests(got[r * 4096:(r + 1) * 4096]).hex() for r in range(2)] == \
        golden["weak4096"][:2]
    del arr, host


@pytest.mark.parametrize("pinned", [False, True])
def test_ragged_misaligned_host_pipeline(pkg, dev, oracle, golden, capfd, monkeypatch, pinned):
    """The config-5 mixed-length law (4 KiB .. 1 MiB, ragged tails; 16384
    chunks, 3.0 GiB) laid out in host memory at byte offsets with 1..15-byte
    gaps (no chunk 16-byte aligned in general) and in a shuffled order, through
    256 MiB slots (>= 12 fills).  Pinned or not, the slots are packed (the
    chunks are neither contiguous nor 16-byte multiples).  Every digest equals
    the reference's golden digest of that chunk."""
    torch = dev
    n = 16384
    lens = oracle.mixed_lengths(n)
    rng = np.random.default_rng(303)
    order = rng.permutation(n)
    gaps = rng.integers(1, 16, n).astype(np.uint64)
    off = np.zeros(n, np.uint64)
    pos = np.uint64(3)
    for i in order:  # chunk i placed in shuffled order, misaligned
        off[i] = pos
        pos += np.uint64(lens[i]) + gaps[i]
    total = int(pos) + 16
    host = torch.empty(total, dtype=torch.uint8, pin_memory=pinned)
    # device-side generation of each chunk (8-byte aligned scratch), copied
    # into its misaligned host place
    aoff = np.zeros(n, np.uint64)
    aoff[1:] = np.cumsum((lens.astype(np.uint64) + 7) // 8 * 8)[:-1]
    abytes = int(aoff[-1]) + int(lens[-1]) + 8
    d = torch.empty(abytes, dtype=torch.uint8, device="cuda")
    pkg.synth_fill_ragged_device(d, torch.from_numpy(aoff.astype(np.int64)).cuda(),
                                 torch.from_numpy(lens.astype(np.int32)).cuda(), 0)
    staged = d.cpu().numpy()
    del d
    arr = host.numpy()
    for i in range(n):
        a, o, ln = int(aoff[i]), int(off[i]), int(lens[i])
        arr[o:o + ln] = staged[a:a + ln]
    del staged
    monkeypatch.setenv("SHA1CHUNK_HOST_DEBUG", "1")
    monkeypatch.setenv("SHA1CHUNK_HOST_SLOT_MIB", "256")
    capfd.readouterr()
    got = pkg.hash_batch(arr, off, lens)
    slots = _slots(capfd)
    assert len(slots) >= 12 and all(s[3] == "packed" for s in slots), slots[:4]
    assert sum(s[1] for s in slots) == n
    want = np.fromfile(os.path.join(GOLDEN, "mixed_16384.bin"), np.uint8).reshape(-1, 20)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} mismatching chunks, first {bad[:8]} lens {lens[bad[:8]]}"
    assert oracle.digest_of_digests(got).hex() == golden["config5"]["agg"]
    # and the verify form of the same batch (verify_hash's 0/1 per chunk)
    want_bad = want.copy()
    want_bad[::97, 7] ^= 0x40
    mism = pkg.verify_batch(arr, off, lens, want_bad)
    assert np.array_equal(np.nonzero(mism)[0], np.arange(0, n, 97))
    del arr, host
