#!/bin/bash
# DMA-staged verify queue (SHA1CHUNK_VQ_DMA=1): throughput of the zero-copy
# bench (8 receive threads, 16384 x 512 KiB) against the drain's CU count,
# the ring size and the queue's batch (group) size, with the queue's
# counters (SHA1CHUNK_VQ_STATS).  Into $1.
out=${1:-gpurun_out/vq_dma_knobs.log}
mkdir -p "$(dirname "$out")"
: > "$out"
run() { echo "# $*" >> "$out"; env SHA1CHUNK_VQ_DMA=1 SHA1CHUNK_VQ_STATS=1 "$@" timeout -k 10 60 tools/vq_zc_bench \
  --mode reserve --producers 8 --chunks 16384 $BARGS >> "$out" 2>&1 || exit 1; }
BARGS="" run SHA1CHUNK_VQ_CUS=64
BARGS="" run SHA1CHUNK_VQ_CUS=128 SHA1CHUNK_VQ_CU_BUDGET=256
BARGS="" run SHA1CHUNK_VQ_RING_MIB=4096
BARGS="" run SHA1CHUNK_VQ_CUS=128 SHA1CHUNK_VQ_CU_BUDGET=256 SHA1CHUNK_VQ_RING_MIB=4096
BARGS="--batch 256" run SHA1CHUNK_VQ_CUS=64
BARGS="--producers 16" run SHA1CHUNK_VQ_CUS=64
