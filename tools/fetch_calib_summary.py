#!/usr/bin/env python3
"""Summarise tools/fetch_calib.sh: per-dispatch FETCH_SIZE and WRITE_SIZE
(kB, as rocprofv3 reports them) of each calibration kernel against the bytes
it is known to read and write -> profiles/fetch_calib_<tag>.json.  The
read factor is what tools/summarize_prof.py multiplies FETCH_SIZE by."""
import csv
import glob
import json
import sys

out, tag = sys.argv[1], sys.argv[2]
known = json.load(open(f"{out}/bytes.json"))


def per_kernel(counter, sub):
    vals = {}
    for path in glob.glob(f"{out}/{sub}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] != counter:
                continue
            for k in ("stream_read", "lane_read"):
                if k in r["Kernel_Name"]:
                    vals.setdefault(k, []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


fetch, write = per_kernel("FETCH_SIZE", "fetch"), per_kernel("WRITE_SIZE", "write")
rec = {"source": "tools/fetch_calib.hip under rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE "
                 "(separate passes, tools/fetch_calib.sh)",
       "chunks": known["chunks"], "chunk_bytes": known["chunk_bytes"], "kernels": {}}
for k in ("stream_read", "lane_read"):
    rb, wb = known[k]["read_bytes"], known[k]["write_bytes"]
    rec["kernels"][k] = {
        "read_bytes": rb, "write_bytes": wb,
        "fetch_size_kb": fetch.get(k), "write_size_kb": write.get(k),
        "read_bytes_over_fetch_size_bytes": rb / (fetch[k] * 1024) if fetch.get(k) else None,
        "write_size_bytes_over_written": write[k] * 1024 / wb if write.get(k) else None,
    }
json.dump(rec, open(f"profiles/fetch_calib_{tag}.json", "w"), indent=1)
print(json.dumps(rec, indent=1))
