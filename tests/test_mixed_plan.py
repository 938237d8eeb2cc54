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
    (est, m, H, F), _ = M.model_plan(lens, C)
    assert m == mode and (m == 1 or H == 0)
    if n == 65536:
        assert F == 4
    if n == 131072:
        assert F == 8


@pytest.mark.parametrize("n,lo,hi", [(65536, 60, 200), (131072, 150, 400), (262144, 60, 400)])
def test_longest_first_layout_gets_a_split_head_and_fused_tail(n, lo, hi):
    """The config-5 law: a split head of the longest groups, the rest fused
    at one wave per SIMD.  Laid out longest-first, measured H = 107, 257,
    115: 12.47, 16.45, 19.07 ms against 18.86, 20.11, 25.37 before the mixed
    kernel; in arrival order (each sorted group's chunks far apart) the same
    plans at 65536 and 262144 chunks took 12.63 and 20.22 ms, against 13.17
    and 43.06 when far-apart groups went all-split (lane-per-chunk fused
    loads); profiles/mixed_r02.json."""
    lens = np.sort(law(n))[::-1].copy()
    (est, m, H, F), (B, _) = M.model_plan(lens, C)
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


def test_plan_ignores_arrival_order():
    """The plan is a function of the multiset of lengths: the device sorts
    before planning, and the fused tail's shared loads make the layout
    irrelevant to the choice (65536 x 512 KiB with permuted offsets: fused
    tail 10.83 ms, in place 10.74; profiles/mixed_r02.json)."""
    lens = law(65536)
    assert M.model_plan(lens, C)[0] == M.model_plan(np.sort(lens)[::-1].copy(), C)[0]
    rng = np.random.default_rng(3)
    assert M.model_plan(lens, C)[0] == M.model_plan(rng.permutation(lens), C)[0]
