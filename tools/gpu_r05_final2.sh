# round-5 evidence after the fixed-cost work: GPU suite, the driver's bench
# command, rocprofv3 trace + FETCH/WRITE/SQ passes of the bench
set -u
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r05e.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu_r05e.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r05c.log 2>&1 || exit 1
bash tools/profile_bench.sh r05c || exit 1
echo done
