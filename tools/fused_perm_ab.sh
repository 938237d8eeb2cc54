#!/bin/bash
# A/B of the byte swap into fresh registers (round 4, bswap_fresh in
# csrc/sha1_device.hpp): the product library against a copy of the previous
# build in abold/, alternating libraries -- the fused kernel at 65536 /
# 131072 / 262144 uniform chunks, and the mixed kernel (config-5 law) at
# 131072 / 262144 chunks in both layouts with the plans forced equal, and
# the 8-wave split shape at 32768 chunks.
out=${1:-gpurun_out/fused_perm_ab}
mkdir -p "$out"
for r in 1 2; do
  for lib in abold/libsha1chunk.so congestion-control-with-bittorren_amd/libsha1chunk.so; do
    tag=$(basename "$(dirname "$lib")")
    timeout -k 10 300 python -u tools/sweep.py --lib "$lib" --chunks 65536,131072,262144 --kernels fused \
      --rounds 5 --burst 3 --out "$out/${tag}_$r.json" > "$out/${tag}_$r.log" 2>&1 || exit 1
    # the 8-wave split shape (two groups per CU, config 4's shard of 8; its
    # lane-per-chunk producers swap the same way)
    timeout -k 10 300 python -u tools/sweep.py --lib "$lib" --chunks 32768 --kernels split11 \
      --rounds 5 --burst 4 --out "$out/${tag}_split_$r.json" > "$out/${tag}_split_$r.log" 2>&1 || exit 1
  done
done
for lay in arrival sorted; do
  for lib in abold congestion-control-with-bittorren_amd; do
    SHA1CHUNK_LIB=$lib/libsha1chunk.so timeout -k 10 300 python -u tools/mixed_bench.py --reps 5 --chunks 131072,262144 \
      --layout $lay --modes plan0.187.4,plan0.116.4 >> "$out/mixed_${lib%%-*}_$lay.jsonl" 2>/dev/null || exit 1
  done
done
