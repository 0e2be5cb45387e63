#!/bin/bash
# YATA / array tests, then C3 and C4 merge phases (sibling-loop changes)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_yata.py tests/test_gpu_arrays.py tests/test_gpu_view.py tests/test_gpu_configs.py -x -q --timeout 280 --timeout-method thread > gpurun_out/sib_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "passed|failed" gpurun_out/sib_tests.log | tail -2; [ $rc -eq 0 ] || { tail -30 gpurun_out/sib_tests.log; exit $rc; }
timeout -k 10 300 python3 scripts/probe_c3.py 10000000 256 16 > gpurun_out/sib_c3.log 2>&1
rc=$?; echo "[c3] rc=$rc"; grep -E "device ms" gpurun_out/sib_c3.log | head -2 | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/probe_c4full.py 2 > gpurun_out/sib_c4.log 2>&1
rc=$?; echo "[c4] rc=$rc"; grep "merge ms" gpurun_out/sib_c4.log | cut -c1-600
exit $rc
