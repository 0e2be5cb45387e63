#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r03e_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r03e_tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 scripts/probe_single.py 10 > gpurun_out/r03e_single.log 2>&1 && grep wall gpurun_out/r03e_single.log
