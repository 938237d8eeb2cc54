#!/bin/bash
# Run-to-run spread of the verify-queue bench with the receive threads on the
# GPU's node: each mode (fill alone, zero-copy, submit) in PROCS processes of
# REPS passes each, interleaved; one JSON line per pass into $OUT.
set -u
OUT=${OUT:-gpurun_out/vq_reps.jsonl}
REPS=${REPS:-7}
PROCS=${PROCS:-2}
DISTINCT=${DISTINCT:-4096}  # distinct source chunks: 4096 = 2 GiB (DRAM), 64 = 32 MiB (cache-resident)
: > "$OUT"
for p in $(seq 1 "$PROCS"); do
  for mode in fill reserve submit; do
    timeout -k 10 120 tools/vq_zc_bench --mode $mode --chunks 16384 --producers 4 --distinct "$DISTINCT" --pieces 1 \
      --pin gpu --reps "$REPS" --golden tests/golden/synth_4096x512k.bin | sed "s/^{/{\"proc\": $p, /" >> "$OUT" \
      || { echo "vq_zc_bench $mode failed"; exit 1; }
  done
done
python3 - "$OUT" <<'PY'
import json, statistics, sys, collections
r = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l)
    r[(d["mode"], d["proc"])].append(d["GiBps"])
for k, v in sorted(r.items()):
    print(k, "median", statistics.median(v), "min", min(v), "max", max(v), v)
PY
