#!/bin/bash
# The layout-aware planner (round 4) against forced plans around its picks:
# config-5 law at 131072 and 262144 chunks, arrival and longest-first
# layouts.  JSON rows (tools/mixed_bench.py) appended to $1.
out=${1:-gpurun_out/mixed_verify.jsonl}
mkdir -p "$(dirname "$out")"
: > "$out"; : > "${out%.jsonl}.plans.log"
mb() { timeout -k 10 240 python -u tools/mixed_bench.py --reps 5 "$@" >> "$out" 2>> "${out%.jsonl}.plans.log"; }
g131=auto,plan1.0.0,plan0.176.4,plan0.184.4,plan0.186.4,plan0.187.4,plan0.192.4,plan0.200.4,auto
g262=auto,plan0.96.4,plan0.101.4,plan0.105.4,plan0.115.4,plan0.116.4,plan0.122.4,auto
for lay in arrival sorted; do
  mb --chunks 131072 --layout $lay --modes $g131 || exit 1
  mb --chunks 262144 --layout $lay --modes $g262 || exit 1
done
