#!/bin/bash
# the per-call GPU step (edited per experiment)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/step_tests.log 2>&1 || { grep -E "^E |FAIL|Error" gpurun_out/step_tests.log | head -30; tail -5 gpurun_out/step_tests.log; exit 1; }
tail -1 gpurun_out/step_tests.log
timeout -k 10 300 python -u scripts/probe_fullstate.py 2>&1 | grep -E "ycrdt decode|merge|chunk_wait" | head -3
timeout -k 10 600 python -u bench.py --only-headline --steps 10 > gpurun_out/step_h.json 2> gpurun_out/step_h.err || { tail -5 gpurun_out/step_h.err; exit 1; }
python3 scripts/bench_summary.py gpurun_out/step_h.json
