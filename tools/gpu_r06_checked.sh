#!/bin/bash
# Round 6: the bounds-checked backend over the layout, mixed and fuzz GPU
# tests (must be green), then the negative control -- round 5's fallback
# clamp reverted -- on test_mixed_plans_scattered (must fail, by the
# checked counter, not by a fault).  Logs under gpurun_out/.
set -u
B=$PWD/congestion-control-with-bittorren_amd
SHA1CHUNK_CHECKED=1 SHA1CHUNK_LIB=$B/build-checked/libsha1chunk.so timeout -k 10 400 \
  python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_gpu_layouts.py tests/test_gpu_mixed.py \
  tests/test_gpu_fuzz.py -m gpu > gpurun_out/pytest_checked_r06.log 2>&1 || { echo "checked run rc=$?"; exit 1; }
tail -1 gpurun_out/pytest_checked_r06.log
SHA1CHUNK_CHECKED=1 SHA1CHUNK_LIB=$B/build-checked-unclamped/libsha1chunk.so timeout -k 10 200 \
  python -u -m pytest -v --timeout 150 --timeout-method thread "tests/test_gpu_layouts.py::test_mixed_plans_scattered" \
  -m gpu > gpurun_out/pytest_checked_unclamped_r06.log 2>&1
rc=$?
echo "unclamped rc=$rc" | tee -a gpurun_out/pytest_checked_unclamped_r06.log
[ $rc -eq 1 ]
