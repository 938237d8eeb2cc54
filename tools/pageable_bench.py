#!/usr/bin/env python3
"""End-to-end rate of sha1chunk_hash_batch from PAGEABLE host memory (a
numpy array, the Python host API's usual input): chunks are packed into
pinned staging by the device's pack pool, copied H2D, hashed, digests D2H.
Spot-checks digests against hashlib (stdlib), nothing from oracle/.

    python3 tools/pageable_bench.py --chunks 16384 --reps 3
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

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    pkg = importlib.import_module("congestion-control-with-bittorren_amd")
    L = pkg.sha1chunk.CHUNK_LEN
    n = a.chunks
    rng = np.random.default_rng(9)
    tile = rng.integers(0, 256, 64 << 20, dtype=np.uint8)
    buf = np.empty(n * L, np.uint8)
    for i in range(0, buf.size, tile.size):
        buf[i:i + tile.size] = tile[: min(tile.size, buf.size - i)]
    buf[::L] = np.arange(n, dtype=np.uint64).astype(np.uint8)  # make chunks differ
    off = np.arange(n, dtype=np.uint64) * L
    ln = np.full(n, L, np.uint32)
    pkg.hash_batch(buf[: 64 * L], off[:64], ln[:64])  # warm-up: device, pools, slots
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        dig = pkg.hash_batch(buf, off, ln)
        ts.append(time.perf_counter() - t0)
    ok = all(dig[i].tobytes() == hashlib.sha1(buf[i * L:(i + 1) * L].tobytes()).digest()
             for i in sorted({0, 1, n // 2, n - 1}))
    row = {"chunks": n, "bytes": n * L, "best_s": round(min(ts), 4), "runs_s": [round(t, 4) for t in ts],
           "GiBps": round(n * L / min(ts) / 2**30, 3),
           "pack_piece_mib": os.environ.get("SHA1CHUNK_PACK_PIECE_MIB", "default"),
           "copy_threads": os.environ.get("SHA1CHUNK_COPY_THREADS", "default"), "digests_ok": ok}
    print(json.dumps(row), flush=True)
    if a.out:
        json.dump(row, open(a.out, "w"), indent=1)
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
