#!/bin/bash
# PMC comparison of split-kernel variants at config 2 (one process per pass;
# each pass its own time limit; stops at the first failing pass).
#   usage: tools/pmc_variants.sh <outdir> <kernels, e.g. split32,split3>
set -u
OUT=$1
K=$2
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD="python3 tools/sweep.py --chunks 4096 --kernels $K --rounds 2"
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH"; do
    i=$((i + 1))
    timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- $CMD > "$OUT/p$i.log" 2>&1 || exit $?
done
