#!/bin/bash
# Round-6 evidence on the final tree: the GPU suite, the driver's bench
# command twice (the verify-queue spread across two lines), the bounds-checked
# runs, and rocprofv3 trace + FETCH/WRITE/SQ passes of the bench.
set -u
TAG=${TAG:-r06}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -n 2 gpurun_out/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${TAG}.log 2>&1 || exit 1
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${TAG}b.log 2>&1 || exit 1
bash tools/gpu_r06_checked.sh || exit 1
BENCH_ARGS="--file-chunks 0" bash tools/profile_bench.sh $TAG || exit 1
echo done
