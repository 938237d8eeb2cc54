#!/usr/bin/env python3
"""Mixed-length device batches larger than BASELINE config 5 (which is 16384
chunks): the same length law (4 KiB .. 1 MiB, every 7th length with a
ragged tail; oracle_mixed_len restated with numpy) at N chunks, timed with
several dispatches: auto (the mixed kernel's device plan above 256 groups),
auto_nomixed (AUTO's uniform-batch rule: fused / 8-wave split), x_sorted
(AUTO's longest-first sort, kernel x forced), x (kernel x in caller order);
any mode + "@hw" / "@persistent" selects the mixed kernel's dispatch (one
workgroup per job / the default work queue, one workgroup per CU).
Digests of every mode must agree, and a sample is checked with hashlib.

  python tools/mixed_bench.py --chunks 16384,65536,131072 [--out FILE]
"""
from __future__ import annotations

import argparse
import hashlib
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SEED = 0x5EED0001
M64 = (1 << 64) - 1


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def mixed_lengths(n: int, seed: int = SEED) -> np.ndarray:
    """oracle/sha1_oracle.c oracle_mixed_len, vectorised."""
    i = np.arange(n, dtype=np.uint64)
    r = splitmix64(np.uint64(seed + 1) ^ i)
    octave = (r & np.uint64(7)).astype(np.uint32)
    mant = ((r >> np.uint64(8)) & np.uint64(4095)).astype(np.uint32)
    ln = (np.uint32(4096) + mant) << octave
    tail = (splitmix64(np.uint64(seed + 2) ^ i) % np.uint64(63)).astype(np.uint32) + 1
    ln = np.where(i % 7 == 6, ln + tail, ln)
    return ln.astype(np.uint32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="16384,65536,131072")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--modes", default="auto,auto_nomixed,split4_sorted")
    ap.add_argument("--layout", default="arrival",
                    choices=["arrival", "sorted", "shuffled", "shuffled_blocks4", "shuffled_window64"],
                    help="chunk placement in memory: arrival order, sorted longest-first, "
                         "arrival order with the offsets permuted at random, permuted in runs of 4 "
                         "adjacent chunks (2 MiB for 512 KiB chunks), or permuted only within each "
                         "window of 64 chunks")
    ap.add_argument("--uniform", type=int, default=0, help="every chunk this long instead of the law")
    ap.add_argument("--misalign", action="store_true",
                    help="hash each chunk from 1..15 bytes past its (16-byte aligned) start, 16 bytes "
                         "shorter: no wave has all lanes 16-byte aligned (the per-lane load path)")
    ap.add_argument("--b2b", type=int, default=0,
                    help="after the timed calls, K more enqueued back to back (one sync): ms per call")
    ap.add_argument("--out", default=None)
    ap.add_argument("--lib", default=None, help="A/B: load this libsha1chunk.so (and its backend) instead")
    a = ap.parse_args()
    import torch
    pkg = importlib.import_module("congestion-control-with-bittorren_amd")
    if a.lib:
        pkg.sha1chunk.LIB_PATH = os.path.abspath(a.lib)
    torch.cuda.set_device(0)
    pkg.set_device(0)
    rows = []
    for n in [int(x) for x in a.chunks.split(",")]:
        lens = np.full(n, a.uniform, np.uint32) if a.uniform else mixed_lengths(n)
        if a.layout == "sorted":
            lens = np.sort(lens)[::-1].copy()
        off, total = pkg.sha1chunk.ragged_layout(lens)
        if a.layout.startswith("shuffled"):
            rng = np.random.default_rng(1)
            if a.layout == "shuffled":
                perm = rng.permutation(n)
            elif a.layout == "shuffled_blocks4":
                perm = (rng.permutation(n // 4)[:, None] * 4 + np.arange(4)[None, :]).reshape(-1)
            else:
                perm = np.concatenate([w + rng.permutation(min(64, n - w)) for w in range(0, n, 64)])
            off, lens = off[perm].copy(), lens[perm].copy()
        base = torch.zeros(total + 128, dtype=torch.uint8, device="cuda")
        d_off = torch.from_numpy(off.astype(np.int64)).cuda()
        d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
        pkg.synth_fill_ragged_device(base, d_off, d_len, 0)
        if a.misalign:
            shift = (np.arange(n, dtype=np.uint64) % np.uint64(15)) + np.uint64(1)
            off = off + shift
            lens = np.maximum(lens.astype(np.int64) - 16, 0).astype(np.uint32)
            d_off = torch.from_numpy(off.astype(np.int64)).cuda()
            d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
        nbytes = int(lens.astype(np.uint64).sum())
        ref = None
        for mode in a.modes.split(","):
            # AUTO sorts a ragged batch longest-first; an explicit kernel does
            # not.  "<x>_sorted" keeps AUTO's sort and forces kernel x behind
            # it (SHA1CHUNK_FORCE_KERNEL); split8 = the 8-wave two-pair layout
            # for every group, split4 = one group per CU with 4-block units.
            mode_name = mode
            mode, _, disp = mode.partition("@")  # <mode>@hw / @persistent: the mixed kernel's dispatch
            base_mode, _, srt = mode.partition("_")
            env = {"SHA1CHUNK_MIXED_DISPATCH": disp} if disp else {}
            kernel = base_mode
            if base_mode.startswith("plan"):  # plan<mode>.<H>.<F>: the mixed kernel with a forced plan
                kernel, env = "auto", {"SHA1CHUNK_MIXED_PLAN": base_mode[4:].replace(".", ",")}
            if base_mode in ("split8", "split4"):
                kernel, env = "split", {"SHA1CHUNK_SPLIT_UNIT": "11" if base_mode == "split8" else "4"}
            if srt == "sorted":
                env["SHA1CHUNK_FORCE_KERNEL"] = kernel
                kernel = "auto"
            elif srt == "nomixed":  # AUTO without the mixed kernel (the uniform-batch rule)
                env["SHA1CHUNK_MIXED"] = "0"
            elif srt == "mixedall":  # the mixed kernel even at <= CUs groups
                env["SHA1CHUNK_MIXED"] = "all"
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                dig = torch.zeros((n, 20), dtype=torch.uint8, device="cuda")
                if kernel == "auto" and srt != "nomixed":  # print the device plan (untimed call)
                    os.environ["SHA1CHUNK_MIXED_DEBUG"] = "1"
                    pkg.hash_device(base, d_off, d_len, dig, kernel=kernel)
                    torch.cuda.synchronize()
                    os.environ.pop("SHA1CHUNK_MIXED_DEBUG")
                ts = []
                for r in range(a.reps + 1):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    pkg.hash_device(base, d_off, d_len, dig, kernel=kernel)
                    torch.cuda.synchronize()
                    if r:
                        ts.append(time.perf_counter() - t0)
                b2b = None
                if a.b2b:  # K calls enqueued back to back, one sync: the chip stays busy
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(a.b2b):
                        pkg.hash_device(base, d_off, d_len, dig, kernel=kernel)
                    torch.cuda.synchronize()
                    b2b = round((time.perf_counter() - t0) / a.b2b * 1e3, 3)
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            got = dig.cpu().numpy()
            if ref is None:
                ref = got
                ok = True
                for i in np.unique(np.linspace(0, n - 1, 24).astype(np.int64)):
                    o, L = int(off[i]), int(lens[i])
                    ok &= hashlib.sha1(base[o:o + L].cpu().numpy().tobytes()).digest() == got[i].tobytes()
            else:
                ok = bool(np.array_equal(got, ref))
            sec = float(np.median(ts))
            row = {"chunks": n, "mode": mode_name, "layout": a.layout + ("+misalign" if a.misalign else ""),
                   "uniform": a.uniform, "payload_bytes": nbytes, "ms": round(sec * 1e3, 3),
                   "payload_GiBps": round(nbytes / sec / 2**30, 2), "runs_ms": [round(t * 1e3, 3) for t in ts],
                   "longest_blocks": int(lens.max()) // 64 + 2, "parity": ok}
            if b2b is not None:
                row["back_to_back_ms_per_call"] = b2b
            print(json.dumps(row), flush=True)
            rows.append(row)
        del base
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
