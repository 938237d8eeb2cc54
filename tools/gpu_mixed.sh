# Mixed-batch evidence (profiles/mixed_r02.json "final"): the mixed-kernel GPU
# tests, then tools/mixed_bench.py on arrival-order, longest-first and uniform
# layouts.  Run on the GPU box: bash tools/gpu_mixed.sh
set -u
mkdir -p gpurun_out/mixed
timeout -k 10 300 python -u -m pytest tests/test_gpu_mixed.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mixed/pytest_mixed.log 2>&1; rc=$?
echo "mixed tests rc=$rc"; tail -18 gpurun_out/mixed/pytest_mixed.log
[ $rc -ne 0 ] && exit $rc
B="timeout -k 10 300 python tools/mixed_bench.py --reps 3"
$B --chunks 16384,32768,65536,131072,262144 --modes auto,auto_nomixed,split4_sorted --out gpurun_out/mixed/arrival.json > gpurun_out/mixed/arrival.txt 2>&1 || exit $?
$B --chunks 65536,131072,262144 --layout sorted --modes auto,auto_nomixed,split4_sorted --out gpurun_out/mixed/sorted.json > gpurun_out/mixed/sorted.txt 2>&1 || exit $?
$B --chunks 32768,65536,131072 --uniform 524288 --modes auto,auto_nomixed --out gpurun_out/mixed/uniform.json > gpurun_out/mixed/uniform.txt 2>&1 || exit $?
grep -h -E "chunks|plan" gpurun_out/mixed/arrival.txt gpurun_out/mixed/sorted.txt gpurun_out/mixed/uniform.txt
