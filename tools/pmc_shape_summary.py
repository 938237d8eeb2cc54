#!/usr/bin/env python3
"""Summarise tools/pmc_shape.sh runs (one directory per chunk count) into a
JSON of mean counters per dispatch of the timed kernel, the clock
(GRBM_GUI_ACTIVE / 8 XCDs / dispatch time) and per-block ratios:
  python tools/pmc_shape_summary.py out.json DIR:N:KERNEL_SUBSTRING:GRID ...
(the bench command also runs its other legs: the timed kernel is picked by
name and grid size)."""
import csv
import glob
import json
import statistics
import sys


def main():
    out, runs = sys.argv[1], sys.argv[2:]
    res = {"what": "rocprofv3 PMC passes over bench.py's device-resident launch of N x 512 KiB (tools/pmc_shape.sh), "
                   "one --pmc pass per counter set; the timed kernel's dispatches (name + grid) of each pass",
           "units": "SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* in quad-cycles (MI355X_MICROARCH.md); "
                    "GRBM_GUI_ACTIVE summed over 8 XCDs", "shapes": {}}
    for spec in runs:
        d, n, sub, grid = spec.split(":")
        n = int(n)
        trace = list(csv.DictReader(open(glob.glob(f"{d}/t/**/run_kernel_trace.csv", recursive=True)[0])))
        mine = [r for r in trace if sub in r["Kernel_Name"] and r["Grid_Size_X"] == grid]
        kern = mine[0]["Kernel_Name"]
        ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in mine]
        ctr = {}
        for path in glob.glob(f"{d}/p*/**/run_counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(path)):
                if r["Kernel_Name"] != kern or r["Grid_Size"] != grid:
                    continue
                ctr.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
                ctr[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        mean = {k: statistics.fmean(v.values()) for k, v in sorted(ctr.items())}
        steady = statistics.median(ms[1:]) if len(ms) > 1 else ms[0]
        ghz = mean.get("GRBM_GUI_ACTIVE", 0) / 8 / (steady * 1e-3) / 1e9 if "GRBM_GUI_ACTIVE" in mean else None
        rec = {"kernel": kern, "dispatch_ms_trace": [round(x, 3) for x in ms], "steady_ms": round(steady, 3),
               "clock_ghz": round(ghz, 3) if ghz else None,
               "cycles_per_block": round(steady * 1e-3 * ghz * 1e9 / 8193, 1) if ghz else None,
               "counters_mean_per_dispatch": {k: round(v) for k, v in mean.items()}}
        wc = mean.get("SQ_WAVE_CYCLES")
        if wc:
            rec["wait_inst_lds_frac_of_wave_cycles"] = round(mean.get("SQ_WAIT_INST_LDS", 0) / wc, 4)
            rec["wait_any_frac"] = round(mean.get("SQ_WAIT_ANY", 0) / wc, 4)
            rec["wait_inst_any_frac"] = round(mean.get("SQ_WAIT_INST_ANY", 0) / wc, 4)
            rec["active_lds_frac"] = round(mean.get("SQ_ACTIVE_INST_LDS", 0) / wc, 4)
        if mean.get("SQ_INSTS_LDS"):
            rec["lds_bank_conflict_per_lds_inst"] = round(mean.get("SQ_LDS_BANK_CONFLICT", 0) / mean["SQ_INSTS_LDS"], 4)
        res["shapes"][str(n)] = rec
    json.dump(res, open(out, "w"), indent=1)
    for n, r in res["shapes"].items():
        print(n, {k: v for k, v in r.items() if k not in ("counters_mean_per_dispatch", "dispatch_ms_trace")})


if __name__ == "__main__":
    main()
