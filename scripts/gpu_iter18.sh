#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/probe_e2e.py 112 > gpurun_out/e2e18.log 2>&1 || { echo "e2e rc=$?"; tail -3 gpurun_out/e2e18.log; exit 1; }
cat gpurun_out/e2e18.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p18_c3 -o run -- python3 scripts/probe_c3.py 10000000 256 16 > gpurun_out/c3_18.log 2>&1 || { echo "c3 rc=$?"; tail -3 gpurun_out/c3_18.log; exit 1; }
rm -f gpurun_out/p18_c3/run_kernel_trace.csv
grep -E "best|merge" gpurun_out/c3_18.log | tail -3 | cut -c1-600
python3 scripts/prof_top.py gpurun_out/p18_c3/run_kernel_stats.csv 30 | grep -E "k_t|yata|k_y|climb|sib|huge"
