#!/bin/bash
# the per-call GPU step (edited per experiment): every -m gpu test, then the C2 PMC / stats passes
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/step_tests.log 2>&1 || { grep -E "^E |FAIL|Error" gpurun_out/step_tests.log | head -30; tail -5 gpurun_out/step_tests.log; exit 1; }
tail -1 gpurun_out/step_tests.log
bash scripts/pmc.sh r05a && python3 scripts/pmc_summary.py gpurun_out/pmc_r05a gpurun_out/pmc_r05a/c2_pmc.csv > gpurun_out/pmc_r05a/summary.txt 2>&1; tail -30 gpurun_out/pmc_r05a/summary.txt; python3 scripts/prof_summary.py gpurun_out/pmc_r05a/stats 2>/dev/null | head -5 || true
