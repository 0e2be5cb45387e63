#!/bin/bash
# headline kernel stats + single doc with the chunk-start hint on
set -u
mkdir -p gpurun_out
for h in 0 1; do YCRDT_DEBUG_DECODE=1 YCRDT_SPEC_HINT=$h timeout -k 10 120 python3 scripts/probe_single.py 1 > gpurun_out/d9_$h.log 2>&1 || { echo "dbg rc=$?"; tail -3 gpurun_out/d9_$h.log; exit 1; }; echo "== hint $h"; grep "fastwalk" gpurun_out/d9_$h.log | tail -1; done
export TMPDIR=/tmp
YCRDT_SPEC_HINT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p9_single -o run -- python3 scripts/probe_single.py 5 > gpurun_out/s9.log 2>&1 || { echo "single rc=$?"; tail -3 gpurun_out/s9.log; exit 1; }
rm -f gpurun_out/p9_single/run_kernel_trace.csv
echo "== single hint"; grep -E "wall" gpurun_out/s9.log; grep -o "'decode.direct': [0-9.]*" gpurun_out/s9.log
python3 scripts/prof_top.py gpurun_out/p9_single/run_kernel_stats.csv 8
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p9_head -o run -- python3 bench.py --steps 3 --warmup 1 --only-headline > gpurun_out/b9.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/b9.log; exit 1; }
rm -f gpurun_out/p9_head/run_kernel_trace.csv
echo "== head"; python3 scripts/prof_top.py gpurun_out/p9_head/run_kernel_stats.csv 16
