#!/bin/bash
# The strong leg's kernel (fused, 262144 x 512 KiB on one GPU) with the
# fresh-register byte swap (product) against the previous build (abold/),
# three rounds alternating.  Into $1/.
out=${1:-gpurun_out/fused_strong_ab}
mkdir -p "$out"
for r in 1 2 3; do
  for lib in abold/libsha1chunk.so congestion-control-with-bittorren_amd/libsha1chunk.so; do
    tag=$(basename "$(dirname "$lib")")
    timeout -k 10 300 python -u tools/sweep.py --lib "$lib" --chunks 262144 --kernels fused --rounds 5 --burst 3 \
      --out "$out/${tag}_$r.json" > "$out/${tag}_$r.log" 2>&1 || exit 1
  done
done
