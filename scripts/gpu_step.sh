#!/bin/bash
# the per-call GPU step (edited per experiment)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/step_tests.log 2>&1 || { grep -E "^E |FAIL|Error" gpurun_out/step_tests.log | head -30; tail -5 gpurun_out/step_tests.log; exit 1; }
tail -1 gpurun_out/step_tests.log
timeout -k 10 900 python bench.py --no-cpu-baseline --no-per-op --fleet-docs 0 --fleet-pairs 0 --profile-phases --steps 10 --warmup 3 > gpurun_out/s_h.json 2> gpurun_out/s_h.err || { tail -20 gpurun_out/s_h.err; exit 1; }
python3 scripts/bench_summary.py gpurun_out/s_h.json || true
