#!/usr/bin/env python3
"""Kernel sweep on one GPU: GiB/s of each hashing kernel vs chunk count, all
kernels interleaved in one process (cdna_hip_programming.md rule 24), on the
same device-resident synthetic chunks.  Prints one JSON line per point and a
summary table; used to tune choose_kernel() in sha1_runtime.hip."""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="1024,4096,16384,65536")
    ap.add_argument("--chunk-len", type=int, default=524288)
    ap.add_argument("--kernels", default="lane,fused,split")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--lib", default=None, help="A/B: load this libsha1chunk.so instead")
    ap.add_argument("--burst", type=int, default=1,
                    help="launches per kernel per round, back to back; the last ceil(burst/2) "
                         "are timed (the chip's clock ramps over the first few ms of a full load)")
    ap.add_argument("--no-check", action="store_true",
                    help="timing only: skip the cross-kernel digest check (diagnostic variants)")
    a = ap.parse_args()
    import torch
    pkg = importlib.import_module("congestion-control-with-bittorren_amd")
    if a.lib:
        import ctypes
        pkg.sha1chunk.LIB_PATH = os.path.abspath(a.lib)
        old = ctypes.CDLL(pkg.sha1chunk.LIB_PATH)  # an older build: bind what it has
        pkg.sha1chunk._SIGNATURES[:] = [sg for sg in pkg.sha1chunk._SIGNATURES if hasattr(old, sg[0])]
    torch.cuda.set_device(0)
    pkg.set_device(0)
    L = a.chunk_len
    kernels = a.kernels.split(",")
    rows = []
    for n in [int(x) for x in a.chunks.split(",")]:
        buf = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        pkg.synth_fill_device(buf, 0, n, L)
        ref = None
        times = {k: [] for k in kernels}
        for _ in range(a.rounds):
            for k in kernels:
                dig = torch.zeros((n, 20), dtype=torch.uint8, device="cuda")
                name = k
                if k.startswith("split") and k[5:].isdigit():  # split<U>: force the unit size
                    os.environ["SHA1CHUNK_SPLIT_UNIT"] = k[5:]
                    name = "split"
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                       for _ in range(max(1, a.burst))]
                for e0, e1 in evs:
                    e0.record()
                    pkg.hash_uniform_device(buf, L, n, dig, kernel=name)
                    e1.record()
                torch.cuda.synchronize()
                os.environ.pop("SHA1CHUNK_SPLIT_UNIT", None)
                timed = evs[len(evs) // 2:]
                times[k].append(float(np.mean([e0.elapsed_time(e1) for e0, e1 in timed])))
                d = dig.cpu().numpy()
                if ref is None:
                    ref = d
                assert a.no_check or np.array_equal(d, ref), f"kernel {k} disagrees at n={n}"
        for k in kernels:
            ms = float(np.median(times[k]))
            row = {"chunks": n, "chunk_bytes": L, "kernel": k, "ms": round(ms, 4),
                   "GiBps": round(n * L / (ms * 1e-3) / 2**30, 2),
                   "hbm_frac": round(n * (L + 20) / (ms * 1e-3) / 8e12, 5),
                   "all_ms": [round(t, 4) for t in times[k]]}
            rows.append(row)
            print(json.dumps(row), flush=True)
        del buf
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
