#!/bin/bash
# Is the scattered-layout slowdown (tools/locality_probe.sh) address
# translation?  UTCL1 (per-CU translation cache) hit/miss and stall counters
# and L2 hit/miss for the fused kernel on 65536 x 512 KiB in place vs with
# permuted offsets.  One rocprofv3 --pmc pass per counter set (TCP block: at
# most 4 per pass), each under its own time limit.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/tlb
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for L in arrival shuffled; do
  CMD="python3 $R/tools/mixed_bench.py --reps 1 --chunks 65536 --uniform 524288 --layout $L --modes fused"
  timeout -s KILL 180 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_THRASHING_STALL_sum --output-format csv -d $OUT/${L}_tcp -o run -- $CMD > $OUT/${L}_tcp.log 2>&1 || exit $?
  timeout -s KILL 180 rocprofv3 --pmc TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum --output-format csv -d $OUT/${L}_tcp2 -o run -- $CMD > $OUT/${L}_tcp2.log 2>&1 || exit $?
  timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/${L}_tcc -o run -- $CMD > $OUT/${L}_tcc.log 2>&1 || exit $?
done
python3 - "$OUT" <<'PY'
import csv, glob, json, sys
out = sys.argv[1]
res = {}
for L in ("arrival", "shuffled"):
    for part in ("tcp", "tcp2", "tcc"):
        for path in glob.glob(f"{out}/{L}_{part}/**/run_counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(path)):
                if "sha1_fused" not in r["Kernel_Name"]:
                    continue
                res.setdefault(L, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
summary = {L: {k: sum(v) / len(v) for k, v in d.items()} for L, d in res.items()}
json.dump(summary, open(f"{out}/summary.json", "w"), indent=1)
print(json.dumps(summary, indent=1))
PY
