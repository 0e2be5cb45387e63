#!/bin/bash
# round-3 final: every GPU test, the default bench line, then the headline kernel stats + PMC passes
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r03d_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r03d_tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/r03d_bench.log 2>&1
rc=$?; echo "[bench] rc=$rc"
[ $rc -eq 0 ] || { tail -5 gpurun_out/r03d_bench.log; exit $rc; }
tail -1 gpurun_out/r03d_bench.log | cut -c1-300
bash scripts/pmc.sh r03d || { echo "pmc failed"; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc_r03d gpurun_out/pmc_r03d/summary.csv > /dev/null
echo "pmc ok"
