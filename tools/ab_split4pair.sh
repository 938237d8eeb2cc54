set -e
mkdir -p gpurun_out/ab
L=congestion-control-with-bittorren_amd/build-ab/libsha1chunk.so
for n in 65536 49152; do
  timeout -k 10 120 python bench.py --chunks $n --kernel fused --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab/f_$n.log 2>&1
  for u in 8 86 87; do
    SHA1CHUNK_LIB=$L SHA1CHUNK_SPLIT_UNIT=$u timeout -k 10 120 python bench.py --chunks $n --kernel split --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab/s${u}_$n.log 2>&1
  done
done
