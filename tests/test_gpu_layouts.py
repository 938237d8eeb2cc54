"""Chunks scattered over the buffer (offsets permuted at random), through
every shape whose bulk loads are shared across the wave (the split
producers, 8 or 4 lanes per chunk; the mixed kernel's fused tail, 8 lanes per
chunk): each load instruction then reads pieces of 8 or 16 chunks that lie
far apart, and the LDS transpose must hand every lane its own chunk's bytes.
Partial last groups exercise the slots past the batch (they read the
group's first chunk); byte-packed chunks (align 1) the shared loads' any
alignment.  Bit-exact against the oracle."""
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


@pytest.fixture(scope="module")
def cus(dev):
    return dev.cuda.get_device_properties(0).multi_processor_count


def _scattered(rng, n, lens, align=16):
    """Chunks packed in a random order: chunk i at off[i], neighbours in
    caller order are far apart."""
    step = (lens.astype(np.uint64) + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align)
    perm = rng.permutation(n)
    off = np.zeros(n, np.uint64)
    off[perm] = np.concatenate([[0], np.cumsum(step[perm])[:-1]]).astype(np.uint64)
    host = rng.integers(0, 256, int((off + lens).max()) + 64, dtype=np.uint8)
    return host, off


def _run(pkg, torch, host, off, lens, kernel, env, monkeypatch):
    for k in ("SHA1CHUNK_MIXED_PLAN", "SHA1CHUNK_SPLIT_UNIT", "SHA1CHUNK_FORCE_KERNEL"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    n = lens.size
    dig = torch.zeros((n, 20), dtype=torch.uint8, device="cuda")
    pkg.hash_device(torch.from_numpy(host).cuda(), torch.from_numpy(off.astype(np.int64)).cuda(),
                    torch.from_numpy(lens.astype(np.int32)).cuda(), dig, kernel=kernel)
    torch.cuda.synchronize()
    return dig.cpu().numpy()


def _check(got, want, what):
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, f"{what}: {bad.size} bad digests, first {bad[:8]}"


@pytest.mark.parametrize("align", [16, 1])
@pytest.mark.parametrize("unit", ["4", "11", "1"])
def test_split_shapes_scattered(pkg, dev, oracle, monkeypatch, unit, align):
    """Equal-ish 9 KiB chunks (a few ragged tails) in a random order, three
    and a half groups: the one-group (unit 4), 8-wave (unit 11) and 1-block
    (unit 1, lane-per-chunk loads) split shapes."""
    torch = dev
    rng = np.random.default_rng(31 + int(unit))
    n = 64 * 3 + 37
    lens = np.full(n, 9216, np.uint32)
    lens[rng.choice(n, 20, replace=False)] = rng.integers(8000, 9300, 20)
    host, off = _scattered(rng, n, lens, align)
    want = oracle.hash_batch(host, off, lens)
    got = _run(pkg, torch, host, off, lens, "split", {"SHA1CHUNK_SPLIT_UNIT": unit}, monkeypatch)
    _check(got, want, f"split unit {unit} align {align}")


@pytest.mark.parametrize("align", [16, 1])
def test_mixed_plans_scattered(pkg, dev, oracle, cus, monkeypatch, align):
    """A ragged batch of more groups than CUs in a random memory order (so
    every sorted group's chunks lie far apart) through the device plan, the
    all-fused tail at F = 4 and 8, a split head, all-split and the 8-wave
    mode."""
    torch = dev
    rng = np.random.default_rng(47)
    G = cus + 9
    n = 64 * G - 29
    lens = rng.integers(0, 5000, n).astype(np.uint32)
    lens[rng.choice(n, 3 * cus, replace=False)] = rng.integers(9000, 30000, 3 * cus)
    host, off = _scattered(rng, n, lens, align)
    want = oracle.hash_batch(host, off, lens)
    for p in (None, "0,0,4", "0,0,8", "0,17,4", f"0,{G},4", "1,0,0"):
        got = _run(pkg, torch, host, off, lens, "auto", {"SHA1CHUNK_MIXED_PLAN": p} if p else {}, monkeypatch)
        _check(got, want, f"plan {p or 'device'} align {align}")
