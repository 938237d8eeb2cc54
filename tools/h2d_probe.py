#!/usr/bin/env python3
"""Diagnostic only: host-to-device copy rate from pinned memory with the
copy split over 1, 2 or 4 HIP streams (does a second SDMA queue raise the
PCIe rate config 3's one-copy-stream pipeline reaches?).  Prints one JSON
line per stream count: GiB/s over `--gib` GiB, best of `--reps`."""
import argparse
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--piece-mib", type=int, default=64)
    a = ap.parse_args()
    n = a.gib << 30
    src = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    src.fill_(7)
    dst = torch.empty(n, dtype=torch.uint8, device="cuda")
    piece = a.piece_mib << 20
    for ns in (1, 2, 4):
        streams = [torch.cuda.Stream() for _ in range(ns)]
        best = 0.0
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i, off in enumerate(range(0, n, piece)):
                with torch.cuda.stream(streams[i % ns]):
                    dst[off:off + piece].copy_(src[off:off + piece], non_blocking=True)
            torch.cuda.synchronize()
            best = max(best, n / (time.perf_counter() - t0) / 2**30)
        print(json.dumps({"streams": ns, "piece_mib": a.piece_mib, "gib": a.gib, "h2d_gibps": round(best, 2)}),
              flush=True)


if __name__ == "__main__":
    main()
