#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r03e_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r03e_tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/r03e_bench.log 2>&1
rc=$?; echo "[bench] rc=$rc"
[ $rc -eq 0 ] || { tail -5 gpurun_out/r03e_bench.log; exit $rc; }
tail -1 gpurun_out/r03e_bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_r03e_single -o run -- python3 scripts/probe_single.py 5 > gpurun_out/r03e_single.log 2>&1 || { echo "prof rc=$?"; exit 1; }
rm -f gpurun_out/p_r03e_single/run_kernel_trace.csv
grep wall gpurun_out/r03e_single.log
