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


@pytest.mark.parametrize("n,mode,lo,hi", [(65536, 0, 1024, 1024), (131072, 0, 176, 200), (262144, 0, 60, 200)])
def test_config5_law_plans(n, mode, lo, hi):
    """The config-5 law in arrival order: every group split (65536:
    chain-bound, all-split simulated as fast as a split head + fused tail
    and measured 12.14 ms against 12.50), or a split head of the longest
    groups and the rest fused at one wave per SIMD (131072, 262144).  The
    plan depends on the lengths only (the device sorts first).  Measured
    (profiles/mixed_verify_r04c.jsonl): 131072 H = 187 13.88 ms, 192 13.90,
    the 8-wave mode 14.21 (the pick before the fused share factor and the
    refinement pass), 200 14.96; 262144 H = 115 19.94, 122 19.97, 96 20.39."""
    lens = law(n)
    (est, m, H, F), (B, _, _) = M.model_plan(lens, C)
    assert m == mode and (m == 1 or (lo <= H <= hi and F == 4)), (m, H, F)
    assert est >= B[0] * M.CHAIN["split4"]  # never below the longest chain


def test_simulation_rejects_late_long_fused_jobs():
    """At 131072 chunks a split head of H = 257 (> C: the 257th split group
    and the first long fused jobs start only when a CU frees) -- what the
    bounds alone picked with the round-2 to round-4 constants -- simulates
    above 16 ms (measured 17.36 in round 2, 17.39 with H = 256 in round 4);
    the plan chosen is near 14 ms with no such head.  (With round 5's
    scattered-fused constants the bounds alone pick H = 191.)"""
    lens = law(131072)
    (lb, m0, H0, F0), (B, P, L) = M.model_plan(lens, C, simulate=False)
    assert M.sim_plan(B, C, 0, 257, 4, L) > 16000
    (est, m, H, F), _ = M.model_plan(lens, C)
    assert est < 14500 and (m == 1 or H <= C), (est, m, H, F)


def test_sorted_insertion_sim_is_greedy_list_scheduling():
    """sim_xcd's sorted-array update (start at the earliest free CU, insert
    the end in order) against a heap, on random job lists."""
    import heapq
    rng = np.random.default_rng(5)
    for _ in range(20):
        G = int(rng.integers(40, 900))
        B = sorted(rng.integers(1, 20000, G).tolist(), reverse=True)
        mode, H, F = (1, 0, 0) if rng.integers(0, 4) == 0 else (0, int(rng.integers(0, G + 1)), int(rng.choice([4, 8])))
        if H == G:
            F = 4
        per = int(rng.choice([4, 32]))
        J = [B[2 * j] * M.CHAIN["split8"] for j in range((G + 1) // 2)] if mode == 1 else \
            [B[j] * M.CHAIN["split4"] for j in range(H)] + \
            [B[j] * M.CHAIN[f"fused{F}T"] for j in range(H, G, F)]
        for x in range(8):
            h = [0.0] * per
            for p in J[x::8]:
                heapq.heappush(h, heapq.heappop(h) + p)
            assert float(M.sim_xcd(B, mode, H, F, x, per)) == pytest.approx(max(h), rel=1e-5)


def test_model_rounds_bound_is_exact_for_equal_jobs():
    """(k+1) p_{kC}: 2.4 C equal groups in the 8-wave split shape are
    ceil(1.2 C / C) = 2 rounds of pairs."""
    G = int(2.4 * C)
    B = [1025] * G
    P = [0]
    for b in B:
        P.append(P[-1] + b)
    m = M.model_makespan(B, C, 1, 0, 0, P, M.Layout([True] * G, B))
    assert m == pytest.approx(2 * 1025 * M.CHAIN["split8"])


def test_plan_depends_on_lengths_and_grouping_not_order():
    """The device sorts before planning, so the caller's order of the
    lengths does not matter when every sorted group's chunks lie scattered
    (arrival layouts); what does is whether they lie together (round 4): a
    batch laid out longest-first streams its fused tail lane-per-chunk."""
    lens = law(65536)
    rng = np.random.default_rng(3)
    assert M.model_plan(lens, C)[0] == M.model_plan(rng.permutation(lens), C)[0]
    srt = np.sort(lens)[::-1].copy()
    _, (_, _, L_arr) = M.model_plan(lens, C)
    _, (_, _, L_srt) = M.model_plan(srt, C)
    assert L_arr.ft < 0.1 and L_srt.ft > 0.9


def test_longest_first_layout_takes_split_head_and_fused_tail():
    """the config-5 law at 131072 chunks laid out
    longest-first measured 13.10 ms with a 160-group split head + fused-4
    tail against 13.63-13.82 for the 8-wave mode the layout-blind planner
    picked (profiles/mixed_dispatch_ab_r03.json).  With the fused shapes
    priced by layout and by their share of the chip, and the heads next to
    the best refined (round 4), both layouts take a split head of ~186
    groups: longest-first 12.39-12.40 ms at H = 176-192 against 14.22 for
    the 8-wave mode, arrival order 13.88 at H = 187 against 14.21
    (profiles/mixed_verify_r04c.jsonl)."""
    lens = law(131072)
    (_, m_arr, H_arr, F_arr), _ = M.model_plan(lens, C)
    (_, m_srt, H, F), _ = M.model_plan(np.sort(lens)[::-1].copy(), C)
    assert m_arr == 0 and F_arr == 4 and 176 <= H_arr <= 192, (m_arr, H_arr, F_arr)
    assert m_srt == 0 and F == 4 and 176 <= H <= 192, (m_srt, H, F)


@pytest.mark.parametrize("G", [257, 300, 511, 512, 513, 1024, 1025, 4096, 16384])
def test_candidates_are_valid_plans(G):
    """Every candidate the planner simulates is a plan the mixed kernel runs
    (H <= hcap or H = G, F in {4, 8}, F = 4 when H = G) and they fit its
    128 simulation slots; the bounds' plan is candidate 0, all-split 2."""
    hcap, _ = M.grid_of(G, C)
    for hb in (0, 1, hcap // 2, hcap):
        for fb in (4, 8):
            cands = M.candidates(G, C, hcap, hb, fb)
            assert len(cands) + 16 <= 128  # + the refinement pass's heads
            assert cands[0] == (0, hb, 4 if hb == G else fb) and cands[1] == (1, 0, 0) and cands[2] == (0, G, 4)
            for m, h, f in cands:
                if m == 1:
                    continue
                assert h <= hcap or h == G, (h, hcap, G)
                assert f in (4, 8) and (h < G or f == 4)
