#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for x in 0 1; do
  YCRDT_SPEC_NOEXACT=$x timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p13_$x -o run -- python3 bench.py --steps 3 --warmup 1 --only-headline > gpurun_out/b13_$x.log 2>&1 || { echo "prof rc=$?"; exit 1; }
  rm -f gpurun_out/p13_$x/run_kernel_trace.csv
  echo "== noexact $x"; python3 scripts/prof_top.py gpurun_out/p13_$x/run_kernel_stats.csv 40 | grep -E "k_spec|k_sync|k_walk|k_direct|k_fastwalk|k_xtab"
  YCRDT_DEBUG_DECODE=1 YCRDT_SPEC_NOEXACT=$x timeout -k 10 200 python3 bench.py --steps 1 --warmup 0 --only-headline > gpurun_out/db13_$x.log 2>&1 || { echo "dbg rc=$?"; exit 1; }
  grep "fastwalk" gpurun_out/db13_$x.log | tail -1
done
