#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/t19.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/t19.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/probe_e2e.py 112 > gpurun_out/e2e19.log 2>&1 || { echo "e2e rc=$?"; tail -3 gpurun_out/e2e19.log; exit 1; }
cat gpurun_out/e2e19.log
