#!/bin/bash
# full GPU tests, then C4 / C3 phases with the decode statistics
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/final_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 3 gpurun_out/final_tests.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/final_tests.log; exit $rc; }
bash scripts/gpu_fwm.sh && bash scripts/gpu_chunks.sh
