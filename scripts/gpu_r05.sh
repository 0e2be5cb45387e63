#!/bin/bash
# Round-5 GPU step (edited per call)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_mapyata.py tests/test_gpu_corrupt.py > gpurun_out/r05_tests.log 2>&1 || { grep -E "^E |FAIL|Error" gpurun_out/r05_tests.log | head -40; tail -5 gpurun_out/r05_tests.log; exit 1; }
tail -2 gpurun_out/r05_tests.log
