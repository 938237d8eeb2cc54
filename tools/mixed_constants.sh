#!/bin/bash
# The mixed planner's per-shape constants, measured with every CU busy
# (VERDICT r3 next #8): one job per CU of each shape on uniform 512 KiB
# chunks (chain time per block = kernel time / 8193), the fused shapes with
# their chunks lying together (arrival layout: lane-per-chunk loads) and
# scattered (shuffled: shared loads), then the config-5 law at 131072 and
# 262144 chunks in both layouts, AUTO against a grid of forced plans.
# JSON rows (tools/mixed_bench.py) appended to $1.
out=${1:-gpurun_out/mixed_const.jsonl}
mkdir -p "$(dirname "$out")"
: > "$out"
mb() { timeout -k 10 240 python -u tools/mixed_bench.py --reps 5 "$@" >> "$out" 2>/dev/null; }
mb --chunks 16384 --uniform 524288 --layout arrival --modes plan0.256.4 || exit 1
mb --chunks 32768 --uniform 524288 --layout arrival --modes plan1.0.0 || exit 1
for lay in arrival shuffled; do
  mb --chunks 65536 --uniform 524288 --layout $lay --modes plan0.0.4 || exit 1
  mb --chunks 131072 --uniform 524288 --layout $lay --modes plan0.0.8 || exit 1
done
grid=auto,plan1.0.0,plan0.96.4,plan0.128.4,plan0.160.4,plan0.192.4,plan0.224.4,plan0.256.4,plan0.128.8,plan0.160.8,plan0.192.8,auto
for lay in arrival sorted; do
  mb --chunks 131072 --layout $lay --modes $grid || exit 1
done
