#!/usr/bin/env python3
"""Per (kernel, grid size) dispatch statistics of a rocprofv3 kernel trace
(run_kernel_trace.csv): bench.py runs config 2 and then its other legs
(config 5, config 3, the one-chunk latency, ...) whose launches share kernel
names with config 2's, so the stats CSV's per-name average mixes them; the
timed config-2 launches are the ones with config 2's grid.

  python tools/trace_by_grid.py gpurun_out/prof_<tag>/trace/run_kernel_trace.csv > profiles/...csv
"""
import csv
import statistics
import sys

groups = {}
for r in csv.DictReader(open(sys.argv[1])):
    if r["Kind"] != "KERNEL_DISPATCH":
        continue
    key = (r["Kernel_Name"], int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))
    groups.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
w = csv.writer(sys.stdout)
w.writerow(["Kernel_Name", "Grid_Size", "Workgroup_Size", "Calls", "Average_us", "Median_us", "Min_us", "Max_us"])
for (name, grid, wg), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
    w.writerow([name, grid, wg, len(d), f"{statistics.fmean(d):.2f}", f"{statistics.median(d):.2f}",
                f"{min(d):.2f}", f"{max(d):.2f}"])
