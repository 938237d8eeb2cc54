#!/bin/bash
# Verify-queue throughput (tools/vq_zc_bench, 16384 x 512 KiB, 4 receive
# threads) vs the drain's CU count (SHA1CHUNK_VQ_CUS, budget raised so one
# queue may take them) and the data path: the drain reading the pinned ring
# over PCIe (DMA=0) or the copy engine staging each group in HBM (DMA=1).
# One JSON line per run into $1.
out=${1:-gpurun_out/vq_cus.jsonl}
mkdir -p "$(dirname "$out")"
: > "$out"
for dma in 0 1; do
  for cus in 64 128; do
    for mode in reserve submit; do
      SHA1CHUNK_VQ_DMA=$dma SHA1CHUNK_VQ_CUS=$cus SHA1CHUNK_VQ_CU_BUDGET=256 timeout -k 10 60 \
        tools/vq_zc_bench --mode $mode --producers 4 --chunks 16384 \
        | sed "s/^{/{\"dma\": $dma, \"vq_cus\": $cus, /" >> "$out" || exit 1
    done
  done
done
for p in 2 8; do
  SHA1CHUNK_VQ_DMA=1 timeout -k 10 60 tools/vq_zc_bench --mode reserve --producers $p --chunks 16384 \
    | sed "s/^{/{\"dma\": 1, \"vq_cus\": 64, /" >> "$out" || exit 1
done
