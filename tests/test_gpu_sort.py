"""The longest-first order AUTO hashes a ragged batch in (sha1_sort.hip):
descending SHA-1 block counts, ceil((len + 9) / 64) clamped at 65535, ties
in caller order -- numpy's stable argsort of the same keys, position for
position, and the sorted lengths the planner reads.  Tile edges of the
three-kernel radix sort (4096 chunks), all-equal and all-distinct keys,
empty chunks, chunks of 4 MiB and more (clamped keys tie in the sort; the
mixed path then re-ranks up to 4096 of them exactly: s1be_mixed_order_async),
and the scanned
path beyond 1 Mi chunks (hist_scan starts instead of per-workgroup column
sums; rocPRIM's onesweep before round 6).  Through the backend's diagnostics
entry point s1be_sort_order_async (no frontend symbol)."""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "congestion-control-with-bittorren_amd")


@pytest.fixture(scope="module")
def sort_order(pkg):
    import torch
    assert torch.cuda.is_available(), "GPU tests need a device"
    torch.cuda.set_device(0)
    pkg.set_device(0)
    be = C.CDLL(os.path.join(PKG_DIR, "libsha1chunk_hip.so"))
    f = be.s1be_sort_order_async
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p]

    def run(lens):
        n = lens.size
        d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
        d_ord = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        d_srt = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        rc = f(d_len.data_ptr(), n, d_ord.data_ptr(), d_srt.data_ptr(), None)
        assert rc == 0, rc
        torch.cuda.synchronize()
        return d_ord.cpu().numpy().view(np.uint32), d_srt.cpu().numpy().view(np.uint32)

    return run


def keys(lens):
    return np.minimum((lens.astype(np.int64) + 9 + 63) // 64, 65535)


def want(lens):
    return np.argsort(-keys(lens), kind="stable").astype(np.uint32)


def check(sort_order, lens):
    order, srt = sort_order(lens)
    w = want(lens)
    bad = np.flatnonzero(order != w)
    assert bad.size == 0, (lens.size, bad[:8], order[bad[:8]], w[bad[:8]])
    assert np.array_equal(srt, lens[w].astype(np.uint32))


@pytest.mark.parametrize("n", [65, 4095, 4096, 4097, 8192 + 63, 131072, 262144 + 4093, 1 << 20])
def test_config5_law_and_tile_edges(sort_order, n):
    rng = np.random.default_rng(n)  # 1 << 20: 256 tiles, the own sort's largest batch
    lens = np.exp(rng.uniform(np.log(4096), np.log(1 << 20), n)).astype(np.uint32)
    lens[rng.choice(n, min(n, 40), replace=False)] = 0
    lens[rng.choice(n, min(n, 40), replace=False)] = 55   # 1 block
    lens[rng.choice(n, min(n, 40), replace=False)] = 56   # 2 blocks
    check(sort_order, lens)


def test_ties_and_clamp(sort_order):
    """Few distinct keys (long runs of ties across tiles, both digits), and
    chunks of 4 MiB and more whose keys clamp to 65535 (caller order)."""
    rng = np.random.default_rng(5)
    n = 50000
    lens = rng.choice(np.array([0, 64, 119, 120, 183, 184, 4096, 65536 * 64, (1 << 22) - 9, 1 << 22, 1 << 30],
                               dtype=np.uint64), n).astype(np.uint32)
    check(sort_order, lens)
    check(sort_order, np.full(9000, 1000, np.uint32))              # one key
    check(sort_order, np.arange(70000, dtype=np.uint32) * 64)      # every key distinct-ish, ascending
    check(sort_order, (np.arange(70000, dtype=np.uint32)[::-1] * 64).copy())  # already sorted


@pytest.mark.parametrize("n", [(1 << 20) + 1, (1 << 20) + 4097, 3 * (1 << 20) + 12345])
def test_scan_path_beyond_1mi(sort_order, n):
    """Past 256 tiles of 4096 the tile starts come from hist_scan (one
    workgroup per slot) instead of each scatter workgroup's column sums: the
    same stable order, at one chunk past the cut, a partial tile past it, and
    ~3 Mi chunks of the config-5 law with clamped 8 MiB chunks and empties."""
    rng = np.random.default_rng(n)
    if n < (1 << 21):
        lens = rng.integers(0, 300000, n).astype(np.uint32)
    else:
        lens = np.exp(rng.uniform(np.log(4096), np.log(1 << 20), n)).astype(np.uint32)
        lens[rng.choice(n, 500, replace=False)] = 0
    lens[rng.choice(n, 1000, replace=False)] = 1 << 23
    check(sort_order, lens)


@pytest.fixture(scope="module")
def mixed_order(pkg, sort_order):
    """s1be_mixed_order_async: the sort, then the layout kernel's exact
    re-ranking of chunks of 4 MiB and more (BigFix) -- the order the mixed
    path hashes in."""
    import torch
    be = C.CDLL(os.path.join(PKG_DIR, "libsha1chunk_hip.so"))
    f = be.s1be_mixed_order_async
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p]

    def run(lens):
        n = lens.size
        off = np.zeros(n, np.int64)
        off[1:] = np.cumsum(lens.astype(np.int64))[:-1]
        d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
        d_off = torch.from_numpy(off).cuda()
        d_ord = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        d_srt = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        rc = f(d_len.data_ptr(), d_off.data_ptr(), n, d_ord.data_ptr(), d_srt.data_ptr(), None)
        assert rc == 0, rc
        torch.cuda.synchronize()
        return d_ord.cpu().numpy().view(np.uint32), d_srt.cpu().numpy().view(np.uint32)

    return run


def exact_keys(lens):
    return (lens.astype(np.int64) + 9 + 63) // 64


@pytest.mark.parametrize("nbig", [0, 1, 100, 2047, 2049, 4096, 4097, 4200])
def test_mixed_order_exact_for_big_chunks(mixed_order, nbig):
    """Chunks of 4 MiB and more tie at the clamped sort key; the mixed path
    re-ranks up to 4096 of them by their exact block counts (stable), across
    the layout kernel's first two workgroups' positions (2048 each).  Beyond
    4096 they keep the sort's order (caller order among themselves).  Lengths
    near the clamp edge (65534..65536 blocks) and equal exact lengths (ties
    in caller order) included."""
    rng = np.random.default_rng(nbig + 3)
    n = 70000
    lens = rng.integers(0, 1 << 20, n).astype(np.uint64)
    big = rng.choice(n, nbig, replace=False)
    lens[big] = rng.integers(65534 * 64 - 9, 1 << 27, nbig)
    if nbig >= 100:
        lens[big[:20]] = 5 << 20  # ties
        lens[big[20:23]] = [65534 * 64 - 9, 65535 * 64 - 9, 65536 * 64 - 9]  # 65534, 65535, 65536 blocks
    lens = lens.astype(np.uint32)
    order, srt = mixed_order(lens)
    # re-ranked when at most 4096 keys clamp (4097: one of them is the
    # 65534-block chunk, so exactly 4096 clamp; 4200: beyond, caller order)
    exact = int((exact_keys(lens) >= 65535).sum()) <= 4096
    w = np.argsort(-(exact_keys(lens) if exact else keys(lens)), kind="stable").astype(np.uint32)
    bad = np.flatnonzero(order != w)
    assert bad.size == 0, (nbig, bad[:8], order[bad[:8]], w[bad[:8]])
    assert np.array_equal(srt, lens[w])


@pytest.mark.parametrize("pattern", ["sawtooth", "tile_runs", "alternating", "one_long"])
def test_adversarial_patterns(sort_order, pattern):
    """Key patterns that stress the ranking and the per-tile histograms:
    a sawtooth whose period is not the tile's, one key per tile (every
    tile's histogram a single slot), two keys alternating lane by lane
    (every ballot split), and one long chunk among equal short ones."""
    n = 64 * 1111 + 1
    i = np.arange(n, dtype=np.int64)
    if pattern == "sawtooth":
        lens = (i % 777) * 64 + 1
    elif pattern == "tile_runs":
        lens = (i // 4096) * 6400 + 100
    elif pattern == "alternating":
        lens = np.where(i % 2 == 0, 100, 1 << 20)
    else:
        lens = np.full(n, 64)
        lens[n // 2] = 1 << 22
    check(sort_order, lens.astype(np.uint32))
