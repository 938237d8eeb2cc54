#!/usr/bin/env python3
"""Where a split consumer's time goes (round 5): runs the A/B library's probe
shapes (SHA1CHUNK_SPLIT_UNIT 97 / 98 / 99: the 8-wave two-pair shape as the
product launches it, the same with phase-shifted 10-read bursts, and the
config-2 one-group shape), whose consumer waves time their s_barrier waits
and their whole block loop with the shader clock and write the counts over
their group's first digest row.  Prints per shape: kernel ms, mean loop
cycles per block, mean barrier-wait cycles per block (the consumer waiting
for its producers), and the spread over groups.  Usage:
  python tools/split_probe.py --lib congestion-control-with-bittorren_amd/build-ab/libsha1chunk.so
"""
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
    ap.add_argument("--lib", required=True)
    ap.add_argument("--cases", default="97:32768,98:32768,99:4096")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    pkg = importlib.import_module("congestion-control-with-bittorren_amd")
    pkg.sha1chunk.LIB_PATH = os.path.abspath(a.lib)
    torch.cuda.set_device(0)
    pkg.set_device(0)
    L = 524288
    for case in a.cases.split(","):
        unit, n = (int(x) for x in case.split(":"))
        buf = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        pkg.synth_fill_device(buf, 0, n, L)
        dig = torch.zeros((n, 20), dtype=torch.uint8, device="cuda")
        os.environ["SHA1CHUNK_SPLIT_UNIT"] = str(unit)
        ms = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            pkg.hash_uniform_device(buf, L, n, dig, kernel="split")
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        allrows = dig.cpu().numpy().view(np.uint32).reshape(n, 5).astype(np.uint64)
        rec = {"unit": unit, "chunks": n, "kernel_ms": round(float(np.median(ms)), 4)}
        # row 0 of a group: its consumer; rows 1, 2: its producers (U == NPROD
        # shapes only); groups 2w and 2w+1 are the two pairs of workgroup w
        for role, r0 in (("consumer", 0), ("producer0", 1), ("producer1", 2)):
            for par in (0, 1):
                rows = allrows[r0::64][par::2]
                blocks = rows[:, 4].astype(np.float64)
                if not np.all(blocks > 0):
                    continue
                bw = (rows[:, 0] | (rows[:, 1] << 32)).astype(np.float64)
                tot = (rows[:, 2] | (rows[:, 3] << 32)).astype(np.float64)
                rec[f"{role}_pair{par}"] = {
                    "loop_cycles_per_block": round(float(np.mean(tot / blocks)), 1),
                    "barrier_wait_per_block": round(float(np.mean(bw / blocks)), 1),
                    "barrier_wait_min_max": [round(float(np.min(bw / blocks)), 1),
                                             round(float(np.max(bw / blocks)), 1)]}
                if role == "consumer" and par == 0:
                    rec["clock_ghz_est"] = round(float(np.mean(tot)) / (float(np.median(ms)) * 1e6), 3)
        print(json.dumps(rec), flush=True)
        del buf, dig
        torch.cuda.empty_cache()
        os.environ.pop("SHA1CHUNK_SPLIT_UNIT")


if __name__ == "__main__":
    main()
