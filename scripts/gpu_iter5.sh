#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_chunk_path.py tests/test_gpu_decode_paths.py tests/test_gpu_windows.py tests/test_gpu_parity.py tests/test_gpu_pending.py tests/test_gpu_compat135.py -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/t5.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/t5.log | tail -8
case $rc in 0|1) ;; *) exit $rc;; esac
for cs in 256 512 1024; do
  YCRDT_SCHUNK=$cs timeout -k 10 120 python3 scripts/probe_single.py 10 > gpurun_out/s5_$cs.log 2>&1
  echo "== single schunk $cs"; grep -E "wall" gpurun_out/s5_$cs.log; grep -o "'decode.direct': [0-9.]*" gpurun_out/s5_$cs.log
done
timeout -k 10 300 python3 scripts/probe_c4full.py 2 > gpurun_out/c4full.log 2>&1 || { echo "c4 rc=$?"; tail -3 gpurun_out/c4full.log; exit 1; }
grep "merge ms" gpurun_out/c4full.log | cut -c1-400
