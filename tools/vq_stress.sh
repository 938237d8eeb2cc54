#!/bin/bash
# Verify-queue stress (tools/vq_zc_bench, results checked chunk by chunk
# against the golden digests, 20 % corrupted): many receive threads, a small
# ring (so reserve/submit keep waiting for space, which they do without the
# queue's lock), both data paths, reserve and submit.  One JSON line per run
# into $1; any wrong result or error fails the script.
out=${1:-gpurun_out/vq_stress.jsonl}
mkdir -p "$(dirname "$out")"
: > "$out"
for dma in 1 0; do
  for ring in 64 1024; do
    for spec in "reserve 16" "submit 16" "reserve 3"; do
      set -- $spec
      SHA1CHUNK_VQ_DMA=$dma SHA1CHUNK_VQ_RING_MIB=$ring timeout -k 10 120 tools/vq_zc_bench --mode $1 \
        --producers $2 --chunks 32768 | sed "s/^{/{\"dma\": $dma, \"ring_mib\": $ring, /" >> "$out" || exit 1
    done
  done
done
