# A/B of the fused tail's LDS-DMA depth at F = 4 (nine buffers, eight blocks
# ahead, against the round-5 five): the tests of the mixed kernel, then the
# config-5 law at 131072 chunks (AUTO and the forced all-fused F = 4 plan) in
# arrival and longest-first order and 65536 uniform 512 KiB chunks permuted,
# alternating the libraries
set -u
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mixed.py tests/test_gpu_layouts.py tests/test_gpu_fuzz.py tests/test_gpu_sort.py > gpurun_out/glds_depth_pytest.log 2>&1 || exit 1
for rep in 1 2 3; do
  for lib in congestion-control-with-bittorren_amd/build-base/libsha1chunk.so congestion-control-with-bittorren_amd/libsha1chunk.so; do
    for lay in arrival sorted; do
      timeout -k 10 120 python3 tools/mixed_bench.py --lib $lib --chunks 131072 --modes auto,plan0.0.4 --reps 5 --layout $lay | sed "s|^|$lib |" >> gpurun_out/glds_depth_ab.log || exit 1
    done
    timeout -k 10 120 python3 tools/mixed_bench.py --lib $lib --uniform 524288 --chunks 65536 --modes plan0.0.4,plan0.0.8 --reps 5 --layout shuffled | sed "s|^|$lib |" >> gpurun_out/glds_depth_ab.log || exit 1
  done
done
echo done
