#!/bin/bash
# Round-5 GPU step (edited per call)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_large_ds.py tests/test_gpu_fastwalk.py tests/test_gpu_corrupt.py tests/test_gpu_chunk_path.py tests/test_gpu_configs.py > gpurun_out/r05_tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r05_tests.log | head -30; tail -5 gpurun_out/r05_tests.log; exit 1; }
tail -2 gpurun_out/r05_tests.log
bash scripts/gpu_c3trace.sh
