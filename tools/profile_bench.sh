#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box): kernel trace + stats
# of the bench command, then FETCH_SIZE and WRITE_SIZE in their own passes
# (never combined with tracing domains), summarised to profiles/.
set -u
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
# the kernel trace covers the whole bench command (config 2, then the strong
# leg and the one-chunk latency child); the counter passes time config 2 alone
BENCH_FULL="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-}"
BENCH="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --strong-total 0 --weak4-chunks 0 --no-latency --no-configs ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $BENCH_FULL > "$OUT/trace.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- $BENCH > "$OUT/fetch.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- $BENCH > "$OUT/write.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d "$OUT/sq" -o run -- $BENCH > "$OUT/sq.log" 2>&1 || exit $?
echo done
