#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
YCRDT_DEBUG_DECODE=1 timeout -k 10 120 python3 scripts/probe_single.py 1 > gpurun_out/d29.log 2>&1 && grep fastwalk gpurun_out/d29.log | tail -1
timeout -k 10 120 python3 scripts/probe_single.py 10 > gpurun_out/s29.log 2>&1 || { echo "single rc=$?"; exit 1; }
echo "== single"; grep -E "wall" gpurun_out/s29.log; grep -o "'decode.direct': [0-9.]*" gpurun_out/s29.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p29 -o run -- python3 scripts/probe_single.py 5 > gpurun_out/s29p.log 2>&1 || { echo "prof rc=$?"; exit 1; }
rm -f gpurun_out/p29/run_kernel_trace.csv
python3 scripts/prof_top.py gpurun_out/p29/run_kernel_stats.csv 8
