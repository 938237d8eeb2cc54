set -u
mkdir -p gpurun_out/loc
for L in arrival shuffled shuffled_blocks4 shuffled_window64; do
  timeout -k 10 200 python tools/mixed_bench.py --reps 2 --chunks 65536 --uniform 524288 --layout $L --modes fused,split4,auto > gpurun_out/loc/$L.txt 2>&1 || exit $?
done
grep -h chunks gpurun_out/loc/*.txt
