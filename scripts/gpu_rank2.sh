#!/bin/bash
# decode-path tests, then one C2 document and the per-op loop
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_wave_decode.py tests/test_gpu_decode_paths.py tests/test_gpu_corrupt.py tests/test_gpu_anyform.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/rank_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 5 gpurun_out/rank_tests.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/rank_tests.log; exit $rc; }
bash scripts/gpu_small.sh
