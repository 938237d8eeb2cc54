#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on the GPU box (tools/fetch_calib.hip):
# the plain run prints the byte counts, then one rocprofv3 pass per counter
# (never combined with each other or with tracing), summarised by
# tools/fetch_calib_summary.py into profiles/fetch_calib_<tag>.json.
set -u
TAG=${1:-r02}
OUT=gpurun_out/fetch_calib_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 ./tools/fetch_calib 4096 3 > "$OUT/bytes.json" || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- ./tools/fetch_calib 4096 3 > "$OUT/fetch.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- ./tools/fetch_calib 4096 3 > "$OUT/write.log" 2>&1 || exit $?
python3 tools/fetch_calib_summary.py "$OUT" "$TAG"
