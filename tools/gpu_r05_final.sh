# round-5 evidence session: GPU suite, the driver's bench command, rocprofv3
# trace + FETCH/WRITE/SQ passes of the bench, LDS/issue PMC passes of the
# one-group (4096) and two-pair (32768) split shapes
set -u
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r05d.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu_r05d.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r05b.log 2>&1 || exit 1
bash tools/profile_bench.sh r05 || exit 1
for n in 4096 32768; do bash tools/pmc_shape.sh gpurun_out/pmc_shape_r05_$n $n || exit 1; done
echo done
