#!/bin/bash
# Round-end rehearsal on one GPU: every -m gpu test, smoke(), then the full default bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/final_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 3 gpurun_out/final_tests.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/final_tests.log; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 1000 python -u bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { tail -20 gpurun_out/final_bench.err; exit 1; }
python3 scripts/bench_summary.py gpurun_out/final_bench.json
