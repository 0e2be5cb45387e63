#!/bin/bash
# the per-call GPU step (edited per experiment): GPU tests, small A/B, per-op trace, bench
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_f.log 2>&1; rc=$?
tail -3 gpurun_out/t_f.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python3 scripts/probe_small_ab.py 2 > gpurun_out/ab_small4.log 2>&1 || exit 1
tail -5 gpurun_out/ab_small4.log
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trp -- python3 scripts/probe_trace.py perop > gpurun_out/trp.log 2>&1 || exit 1
python3 scripts/trace_last.py gpurun_out/trp 0 > gpurun_out/tr_perop6.txt; rm -rf gpurun_out/trp
timeout -k 10 400 python3 bench.py > gpurun_out/b_f.json 2> gpurun_out/b_f.err || exit 1
python3 scripts/bench_summary.py gpurun_out/b_f.json 2>/dev/null | head -6
