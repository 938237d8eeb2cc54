#!/bin/bash
# PMC passes over bench.py's device-resident launch of N x 512 KiB chunks
# (the kernel AUTO picks for N): clock (GRBM_GUI_ACTIVE), issue and wait
# counters, LDS.  One rocprofv3 process per pass, each with its own limit;
# stops at the first failing pass.
#   usage: tools/pmc_shape.sh <outdir> <chunks> [extra env assignments for bench.py]
set -u
OUT=$1
N=$2
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD="python3 bench.py --chunks $N --steps 6 --warmup 1 --no-cpu-baseline --no-latency --strong-total 0"
i=0
for set in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM" \
           "SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_IFETCH"; do
    i=$((i + 1))
    timeout -k 10 180 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- $CMD > "$OUT/p$i.log" 2>&1 || exit $?
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/t" -o run -- $CMD > "$OUT/t.log" 2>&1 || exit $?
