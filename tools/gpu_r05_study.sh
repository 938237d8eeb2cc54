# round-5 study session: LDS-DMA fused loop, tests + A/B against the round-4 build
set -u
timeout -k 10 400 python -u -m pytest tests/test_gpu_mixed.py tests/test_gpu_layouts.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_glds2_r05.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_glds2_r05.log; [ $rc -eq 0 ] || exit $rc
for lib in congestion-control-with-bittorren_amd/libsha1chunk.so congestion-control-with-bittorren_amd/build-old/libsha1chunk.so; do
  for lay in arrival shuffled shuffled_blocks4; do timeout -k 10 300 python tools/mixed_bench.py --lib $lib --chunks 65536 --uniform 524288 --reps 5 --layout $lay --modes plan0.0.4,plan0.0.8 2>&1 | grep "^{" | sed "s|^|$lib |" >> gpurun_out/glds2_ab_r05.log || exit 1; done
  for lay in arrival sorted; do timeout -k 10 300 python tools/mixed_bench.py --lib $lib --chunks 131072 --reps 5 --layout $lay --modes auto,plan0.187.4 2>&1 | grep "^{" | sed "s|^|$lib |" >> gpurun_out/glds2_ab_r05.log || exit 1; done
done
echo done
