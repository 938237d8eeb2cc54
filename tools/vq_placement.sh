#!/bin/bash
# Receive-path verify-queue rate against host placement:
# tools/vq_zc_bench in both modes, producers left to the scheduler (--pin
# none) and bound to the GPU's NUMA node (--pin gpu), REPS times each,
# interleaved, plus the library's own placement off (SHA1CHUNK_NUMA=off).
# One JSON line per run into $OUT.  Run from the repo root on the GPU box.
set -u
OUT=${OUT:-gpurun_out/vq_place.jsonl}
REPS=${REPS:-3}
MODES=${MODES:-"reserve submit"}
NUMAS=${NUMAS:-"default"}
: > "$OUT"
{
  echo "# nodes: $(cat /sys/devices/system/node/online 2>/dev/null)"
  for n in /sys/devices/system/node/node*; do echo "# $(basename $n) cpus $(cat $n/cpulist 2>/dev/null)"; done
  echo "# cpu.max $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
  echo "# affinity $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))')"
} >> "${OUT%.jsonl}.topo.txt"
for r in $(seq 1 "$REPS"); do
  for numa in $NUMAS; do
    for pin in none gpu; do
      for mode in $MODES; do
        line=$(VQ_ZC_TRACE=1 SHA1CHUNK_NUMA=$numa timeout -k 10 60 tools/vq_zc_bench --mode "$mode" --chunks 16384 \
               --producers 4 --distinct 4096 --pieces 1 --pin "$pin" \
               --golden tests/golden/synth_4096x512k.bin 2>"${OUT%.jsonl}.last.err") || {
          rc=$?; echo "vq_zc_bench failed rc=$rc (rep $r numa $numa pin $pin mode $mode)" >&2
          cat "${OUT%.jsonl}.last.err" >&2; exit 1; }
        echo "{\"rep\": $r, \"numa\": \"$numa\", $(echo "$line" | sed 's/^{//')" >> "$OUT"
        echo "rep $r numa $numa pin $pin $mode: $(echo "$line" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["GiBps"], d["produce_seconds"], d["placement"]["gpu_node"], d["placement"]["ring_pages"])')"
      done
    done
  done
done
