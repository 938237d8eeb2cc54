#!/bin/bash
# SQ counters for the fused kernel at high occupancy (131072 chunks).
set -u
OUT=$1
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD="python3 tools/sweep.py --chunks 131072 --kernels fused --rounds 2"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d "$OUT/p1" -o run -- $CMD > "$OUT/p1.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM --output-format csv -d "$OUT/p2" -o run -- $CMD > "$OUT/p2.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/t" -o run -- $CMD > "$OUT/t.log" 2>&1 || exit $?
