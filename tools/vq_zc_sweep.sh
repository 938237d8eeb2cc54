#!/bin/bash
# Verify-queue throughput sweep on a GPU box (tools/vq_zc_bench): zero-copy
# reservations vs submit copies vs the fill alone, per producer-thread count
# and ring memory type.  One JSON line per run into $1.
out=${1:-gpurun_out/vq_zc.jsonl}
mkdir -p "$(dirname "$out")"
: > "$out"
bench=tools/vq_zc_bench
for mem in uncached coherent; do
  for spec in "submit 1" "submit 4" "fill 1" "fill 4" "fill 8" "reserve 1" "reserve 2" "reserve 4" "reserve 8"; do
    set -- $spec
    SHA1CHUNK_VQ_RING_MEM=$mem timeout -k 10 60 $bench --mode $1 --producers $2 --chunks 16384 >> "$out" || exit 1
  done
done
