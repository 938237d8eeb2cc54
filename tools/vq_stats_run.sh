#!/bin/bash
# Verify-queue lock and event counters (SHA1CHUNK_VQ_STATS=1) for the
# zero-copy bench, per data path and receive-thread count: the bench's JSON
# line, then the queue's stats line.  Into $1.
out=${1:-gpurun_out/vq_stats.log}
mkdir -p "$(dirname "$out")"
: > "$out"
for dma in 0 1; do
  for p in 4 8; do
    SHA1CHUNK_VQ_STATS=1 SHA1CHUNK_VQ_DMA=$dma timeout -k 10 60 tools/vq_zc_bench --mode reserve --producers $p \
      --chunks 16384 >> "$out" 2>&1 || exit 1
  done
done
