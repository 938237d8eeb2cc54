"""CPU: the mixed kernel's planner (sha1_kernels.hip plan_mixed_kernel), in
the restatement tests/test_gpu_mixed.py checks the device against, picks the
plans the measurements behind it call for (DESIGN.md section 5,
profiles/mixed_r02.json) on a 256-CU MI355X."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import test_gpu_mixed as M  # noqa: E402  (the restatement; its GPU tests stay GPU-marked)

C = 256
L512 = 524288


def contiguous(lens):
    off = np.zeros(lens.size, np.uint64)
    off[1:] = np.cumsum((lens.astype(np.uint64) + 127) // 128 * 128)[:-1]
    return off


def law(n, seed=0x5EED0001):
    """oracle_mixed_len (oracle/sha1_oracle.c), vectorised."""
    def sm(x):
        with np.errstate(over="ignore"):
            z = x + np.uint64(0x9E3779B97F4A7C15)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            return z ^ (z >> np.uint64(31))
    i = np.arange(n, dtype=np.uint64)
    r = sm(np.uint64(seed + 1) ^ i)
    ln = (np.uint32(4096) + ((r >> np.uint64(8)) & np.uint64(4095)).astype(np.uint32)) << (
        r & np.uint64(7)).astype(np.uint32)
    tail = (sm(np.uint64(seed + 2) ^ i) % np.uint64(63)).astype(np.uint32) + 1
    return np.where(i % 7 == 6, ln + tail, ln).astype(np.uint32)


def test_law_matches_golden_lengths():
    g = np.fromfile(os.path.join(os.path.dirname(__file__), "golden", "mixed_16384_len.bin"), "<u4")
    assert np.array_equal(law(16384), g)


@pytest.mark.parametrize("n,mode", [(32768, 1), (65536, 0), (131072, 0)])
def test_uniform_batches_keep_their_kernels(n, mode):
    """Equal 512 KiB chunks back to back: the 8-wave split at <= 2 groups
    per CU, the fused kernel beyond (F = 4 at one wave per SIMD, F = 8 at
    two) -- AUTO's uniform-batch rule, measured 6.47 / 10.33 / 20.25 ms."""
    lens = np.full(n, L512, np.uint32)
    (est, m, H, F), _ = M.model_plan(lens, C, contiguous(lens))
    assert m == mode and (m == 1 or H == 0)
    if n == 65536:
        assert F == 4
    if n == 131072:
        assert F == 8


@pytest.mark.parametrize("n", [32768, 65536, 131072, 262144])
def test_arrival_order_mixed_batches_go_all_split(n):
    """The config-5 law in arrival order: sorted groups of far-apart chunks,
    so the whole batch runs in the one-group split shape (measured 12.27,
    12.94, 21.86, 43.46 ms against 14.58, 32.38, 38.63, 56.39 before)."""
    lens = law(n)
    (est, m, H, F), (B, _) = M.model_plan(lens, C, contiguous(lens))
    assert (m, H, F) == (0, len(B), 4)


@pytest.mark.parametrize("n,lo,hi", [(65536, 60, 200), (131072, 150, 400), (262144, 60, 400)])
def test_longest_first_layout_gets_a_split_head_and_fused_tail(n, lo, hi):
    """The same lengths laid out longest-first: a split head of the longest
    groups, the rest fused at one wave per SIMD (measured H = 107, 257, 115:
    12.47, 16.45, 19.07 ms against 18.86, 20.11, 25.37 before); the
    estimate is within the longest chain's time of the measurement."""
    lens = np.sort(law(n))[::-1].copy()
    (est, m, H, F), (B, _) = M.model_plan(lens, C, contiguous(lens))
    assert m == 0 and lo <= H <= hi and F == 4, (H, F)
    assert est >= B[0] * M.CHAIN["split4"]  # never below the longest chain


def test_model_rounds_bound_is_exact_for_equal_jobs():
    """(k+1) p_{kC}: 2.4 C equal groups in the 8-wave split shape are
    ceil(1.2 C / C) = 2 rounds of pairs."""
    G = int(2.4 * C)
    B = [1025] * G
    P = [0]
    for b in B:
        P.append(P[-1] + b)
    m = M.model_makespan(B, C, 1, 0, 0, P)
    assert m == pytest.approx(2 * 1025 * M.CHAIN["split8"])


@pytest.mark.parametrize("layout,scattered", [("in_place", False), ("window64", False),
                                              ("runs_of_4", False), ("random", True)])
def test_uniform_layouts_scatter_rule(layout, scattered):
    """65536 x 512 KiB laid out as tools/locality_probe.sh measured them: in
    place, permuted within each 64-chunk window, permuted in 2 MiB runs of
    four (fused 14.8 ms, split 24.6: keep the fused kernel), permuted at
    random (fused 29.3, split 28.9: the split shape)."""
    n = 65536
    lens = np.full(n, L512, np.uint32)
    off = contiguous(lens)
    rng = np.random.default_rng(1)
    if layout == "window64":
        perm = np.concatenate([w + rng.permutation(64) for w in range(0, n, 64)])
    elif layout == "runs_of_4":
        perm = (rng.permutation(n // 4)[:, None] * 4 + np.arange(4)[None, :]).reshape(-1)
    elif layout == "random":
        perm = rng.permutation(n)
    else:
        perm = np.arange(n)
    off = off[perm]
    (est, m, H, F), (B, _) = M.model_plan(lens, C, off)
    assert ((m, H, F) == (0, len(B), 4)) == scattered, (layout, m, H, F)
