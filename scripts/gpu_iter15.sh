#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for h in 2 0; do
  YCRDT_SPEC_HINT=$h YCRDT_DEBUG_DECODE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p15_$h -o run -- python3 scripts/probe_c4full.py 1 > gpurun_out/c15_$h.log 2>&1 || { echo "c4 rc=$?"; tail -3 gpurun_out/c15_$h.log; exit 1; }
  rm -f gpurun_out/p15_$h/run_kernel_trace.csv
  echo "== hint $h"; grep "merge ms" gpurun_out/c15_$h.log | cut -c1-120; grep fastwalk gpurun_out/c15_$h.log | tail -2
  python3 scripts/prof_top.py gpurun_out/p15_$h/run_kernel_stats.csv 8
done
