#!/usr/bin/env python3
"""Summarise a tools/profile_bench.sh run (gpurun_out/prof_<tag>) into
profiles/: the rocprofv3 kernel stats CSV as-is, the SQ counter CSV, and a
traffic JSON (FETCH_SIZE x 2 gfx950 correction + WRITE_SIZE, per dispatch of
the dominant kernel) that bench.py reads for roofline.traffic.

The x 2 read correction is measured, not quoted: tools/fetch_calib.hip reads
a known 2 GiB both coalesced and in the hash kernels' own pattern (lane =
chunk, 16-byte loads, 128 bytes per lane per stage) and FETCH_SIZE comes out
at half the bytes in both (read bytes / FETCH_SIZE bytes = 1.99999 and
1.99996), WRITE_SIZE at exactly the bytes written (profiles/fetch_calib_r02.json)."""
import csv
import json
import os
import shutil
import sys

tag, out_tag = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 4096  # chunks per launch (bench --chunks)
name = "bench" if n == 4096 else f"bench_{n}"
src = f"gpurun_out/prof_{tag}"
dst = "profiles"
shutil.copy(f"{src}/trace/run_kernel_stats.csv", f"{dst}/rocprof_{name}_{out_tag}_kernel_stats.csv")
shutil.copy(f"{src}/sq/run_counter_collection.csv", f"{dst}/rocprof_{name}_{out_tag}_sq_counters.csv")


grid = sys.argv[4] if len(sys.argv) > 4 else None  # Grid_Size of the timed launches (other legs in the pass)


def per_kernel(path, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and "sha1_" in r["Kernel_Name"] and "synth" not in r["Kernel_Name"] \
                and (grid is None or r["Grid_Size"] == grid):
            vals.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    (k, v), = [(k, v) for k, v in vals.items()]
    return k, v


k, fetch = per_kernel(f"{src}/fetch/run_counter_collection.csv", "FETCH_SIZE")
_, write = per_kernel(f"{src}/write/run_counter_collection.csv", "WRITE_SIZE")
L = 524288
f_kb, w_kb = sum(fetch) / len(fetch), sum(write) / len(write)
rd, wr = 2 * f_kb * 1024, w_kb * 1024
alg = n * (L + 20)
rec = {
    "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, of `python3 bench.py "
              f"--steps 10 --warmup 2 --no-cpu-baseline{'' if n == 4096 else f' --chunks {n}'}` "
              "(tools/profile_bench.sh)",
    "kernel": k, "chunks": n, "chunk_bytes": L, "dispatches": len(fetch),
    "fetch_size_kb_per_dispatch": f_kb, "write_size_kb_per_dispatch": w_kb,
    "correction": "gfx950 FETCH_SIZE reports half the bytes read in this access pattern "
                  "(calibrated on a known 2 GiB read: profiles/fetch_calib_r02.json): read "
                  "bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024 exact",
    "read_bytes_per_launch": rd, "write_bytes_per_launch": wr, "bytes_per_launch": rd + wr,
    "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": (rd + wr) / alg,
}
json.dump(rec, open(f"{dst}/traffic_{out_tag}.json" if n == 4096 else f"{dst}/traffic_{n}_{out_tag}.json", "w"),
          indent=1)
print(json.dumps(rec, indent=1))
