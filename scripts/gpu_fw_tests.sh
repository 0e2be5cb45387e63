#!/bin/bash
# decode / config / shard tests, then C3 and C4 phases
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/fw_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 4 gpurun_out/fw_tests.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/fw_tests.log; exit $rc; }
bash scripts/gpu_chunks.sh
