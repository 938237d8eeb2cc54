#!/bin/bash
# Instruction-cache and barrier counters over bench.py's launch of N chunks
# (one rocprofv3 process per pass, each with its own limit).
#   usage: tools/pmc_icache.sh <outdir> <chunks>
set -u
OUT=$1
N=$2
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD="python3 bench.py --chunks $N --steps 6 --warmup 3 --no-cpu-baseline --no-latency --strong-total 0"
i=0
for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH GRBM_GUI_ACTIVE SQ_WAVES" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
    i=$((i + 1))
    timeout -k 10 180 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- $CMD > "$OUT/p$i.log" 2>&1 || exit $?
done
