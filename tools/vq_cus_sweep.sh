#!/bin/bash
# Verify-queue throughput vs the drain's CU count (SHA1CHUNK_VQ_CUS; the
# budget knob raised so a single queue may take them) with zero-copy
# reservations, 4 receive threads.  One JSON line per run into $1.
out=${1:-gpurun_out/vq_cus.jsonl}
mkdir -p "$(dirname "$out")"
: > "$out"
for cus in 32 64 128 192; do
  for mode in reserve submit; do
    SHA1CHUNK_VQ_CUS=$cus SHA1CHUNK_VQ_CU_BUDGET=256 timeout -k 10 60 tools/vq_zc_bench --mode $mode --producers 4 --chunks 16384 \
      | sed "s/^{/{\"vq_cus\": $cus, /" >> "$out" || exit 1
  done
done
