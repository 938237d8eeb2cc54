#!/usr/bin/env python3
"""CPU baseline table (BASELINE.md "CPU baseline on the box"):
the reference sha.c built with its own Makefile flags (-g, no -O) and with
-O2, plus the repo's CPU restatement, each on 1 thread and on the box's CPU
share (16 threads, chunk-strided pthreads), over the same synthetic 512 KiB
chunks bench.py hashes.  Test infrastructure only: it times oracle/, never
the product.

    python3 tools/cpu_baseline_table.py --out profiles/cpu_baseline_r01.json
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402


def cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,16")
    ap.add_argument("--chunks-per-thread", type=int, default=256,
                    help="sample = this many chunks per thread (capped at 4096)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
    L = O.CHUNK_LEN
    rows = []
    for kind, opt in (("reference", "O2"), ("reference", "O0"), ("port", "O2")):
        for t in (int(x) for x in a.threads.split(",")):
            n = min(4096, a.chunks_per_thread * t)
            if kind == "reference":
                r = O.ref_lib(opt)
                if r is None:
                    raise FileNotFoundError(f"oracle/_ref reference build ({opt}) missing")
                import numpy as np
                agg = np.zeros(20, np.uint8)
                secs = float(r.ref_time_synth(0, n, L, O.SEED, t, agg.ctypes.data_as(O._u8p)))
                agg = agg.tobytes()
            else:
                secs, agg = O.time_synth(n, L, threads=t, kind="port")
            row = {"impl": "sha.c" if kind == "reference" else "oracle restatement",
                   "flags": "-g (reference Makefile)" if opt == "O0" else "-O2",
                   "threads": t, "chunks": n, "seconds": round(secs, 4),
                   "GiBps": round(n * L / secs / 2**30, 4),
                   "agg_matches_golden": (agg.hex() == golden["weak4096"][0]) if n == 4096 else None}
            rows.append(row)
            print(json.dumps(row), flush=True)
    res = {"host_cpu": cpu_model(), "os_cpu_count": os.cpu_count(),
           "note": "oracle/_ref/libsharef*.so = the reference sha.c compiled from /root/reference by "
                   "oracle/Makefile; chunks 0..n-1 of the bench corpus (splitmix64, seed 0x5EED0001), "
                   "512 KiB each; threads take chunks by stride",
           "rows": rows}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
