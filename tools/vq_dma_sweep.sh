#!/bin/bash
# Verify-queue throughput (tools/vq_zc_bench, 512 KiB chunks of config 2's
# corpus) by data path -- the drain reading the pinned ring over PCIe
# (SHA1CHUNK_VQ_DMA=0) or the copy engine staging each group in HBM (=1) --
# mode (reserve / submit / fill alone) and receive-thread count.  One JSON
# line per run into $1.
out=${1:-gpurun_out/vq_dma.jsonl}
mkdir -p "$(dirname "$out")"
: > "$out"
for dma in 0 1; do
  for spec in "fill 4" "reserve 2" "reserve 4" "reserve 8" "submit 4"; do
    set -- $spec
    SHA1CHUNK_VQ_DMA=$dma timeout -k 10 60 tools/vq_zc_bench --mode $1 --producers $2 --chunks 32768 \
      | sed "s/^{/{\"dma\": $dma, /" >> "$out" || exit 1
  done
done
