#!/bin/bash
# decode-path tests (ranked small updates), then the per-op probe
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_wave_decode.py tests/test_gpu_decode_paths.py tests/test_gpu_corrupt.py tests/test_gpu_anyform.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/rank_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 25 gpurun_out/rank_tests.log
[ $rc -eq 0 ] || exit $rc
PEROP_N=${PEROP_N:-2000} timeout -k 10 300 python3 scripts/probe_perop.py > gpurun_out/perop.log 2>&1
rc=$?; echo "[perop] rc=$rc"; cut -c1-900 gpurun_out/perop.log
exit $rc
