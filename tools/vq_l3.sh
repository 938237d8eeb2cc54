#!/bin/bash
# The verify-queue bench with the receive threads on the GPU's node as a
# whole (--pin gpu) against one per L3 domain of it (--pin l3), submit and
# zero-copy, PROCS processes of REPS passes each, interleaved; one JSON line
# per pass into $OUT, the box's L3 domains into $OUT.topo.txt.
set -u
OUT=${OUT:-gpurun_out/vq_l3.jsonl}
REPS=${REPS:-5}
PROCS=${PROCS:-2}
DISTINCT=${DISTINCT:-64}
: > "$OUT"
{
  for n in /sys/devices/system/node/node*/cpulist; do echo "# $n $(cat "$n")"; done
  sort -u /sys/devices/system/cpu/cpu*/cache/index3/shared_cpu_list | sed 's/^/# l3 /'
  echo "# cpu.max $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
} > "$OUT.topo.txt"
for p in $(seq 1 "$PROCS"); do
  for pin in gpu l3; do
    for mode in submit reserve; do
      timeout -k 10 120 tools/vq_zc_bench --mode $mode --chunks 16384 --producers 4 --distinct "$DISTINCT" \
        --pieces 1 --pin $pin --reps "$REPS" --golden tests/golden/synth_4096x512k.bin >> "$OUT" \
        || { echo "fail $pin $mode rc=$?"; exit 1; }
    done
  done
done
python3 - "$OUT" <<'PY'
import json, statistics, sys
r = {}
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        r.setdefault((d["placement"]["pin"], d["mode"]), []).append(d["GiBps"])
for k, v in sorted(r.items()):
    print(k, "median", statistics.median(v), "min", min(v), "max", max(v), v)
PY
