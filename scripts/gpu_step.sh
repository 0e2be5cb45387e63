#!/bin/bash
# the per-call GPU step (edited per experiment)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
YCRDT_DEBUG_DECODE=1 timeout -k 10 300 python3 scripts/probe_trace.py c2x112 > gpurun_out/dbg_c2.log 2>&1 || { tail -20 gpurun_out/dbg_c2.log; exit 1; }
grep "direct split" gpurun_out/dbg_c2.log | tail -2; tail -1 gpurun_out/dbg_c2.log
rm -rf gpurun_out/tr_c2full
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_c2full -o tr -- python3 scripts/probe_trace.py c2full > gpurun_out/tr_c2full.log 2>&1 || { tail -20 gpurun_out/tr_c2full.log; exit 1; }
python3 scripts/trace_last.py gpurun_out/tr_c2full 100 > gpurun_out/tr_c2full.txt; head -30 gpurun_out/tr_c2full.txt
rm -rf gpurun_out/tr_c2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_c2 -o tr -- python3 scripts/probe_trace.py c2x112 > gpurun_out/tr_c2.log 2>&1 || { tail -20 gpurun_out/tr_c2.log; exit 1; }
python3 scripts/trace_last.py gpurun_out/tr_c2 300 > gpurun_out/tr_c2.txt; head -8 gpurun_out/tr_c2.txt
