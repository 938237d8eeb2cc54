#!/bin/bash
# The mixed path's fixed cost (sort + layout + planner kernels before the
# hash, tools/fixed_cost.py) at 131072 chunks of the config-5 law, in
# arrival and longest-first layouts, for the build under test against an
# A/B knob (AB_ENV: the round-6 study's SHA1CHUNK_LAYOUT_SORTED=0, in the
# build that had it), alternated REPS times.
# rocprofv3 kernel traces under gpurun_out/$TAG/.
set -u
TAG=${TAG:-fixed_ab}
REPS=${REPS:-2}
CHUNKS=${CHUNKS:-131072}
AB_ENV=${AB_ENV:-SHA1CHUNK_LAYOUT_SORTED=0}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
for r in $(seq 1 "$REPS"); do
  for v in new old; do
    for lay in arrival sorted; do
      d=gpurun_out/$TAG/${v}_${lay}_$r
      if [ $v = old ]; then envs="$AB_ENV"; else envs="SHA1CHUNK_AB_NONE=1"; fi
      env $envs timeout -k 10 200 rocprofv3 --kernel-trace -d $d -o run -- python3 tools/mixed_bench.py --chunks $CHUNKS \
        --modes auto --reps 5 --b2b 5 --layout $lay > $d.log 2>&1 || { echo "fail $d"; exit 1; }
      python3 tools/fixed_cost.py $(find $d -name '*.db' | head -n 1) > $d.jsonl
      python3 - "$d.jsonl" "$v" "$lay" <<'PY'
import json, statistics, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
s = [r["sum_us"] for r in rows]
k = {}
for r in rows:
    for n, v in r["kernels_us"].items():
        k.setdefault(n, []).append(v)
print(sys.argv[2], sys.argv[3], "median sum", statistics.median(s), {n: statistics.median(v) for n, v in k.items()})
PY
    done
  done
done
