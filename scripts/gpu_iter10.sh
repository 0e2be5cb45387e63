#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_chunk_path.py tests/test_gpu_decode_paths.py tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/t10.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/t10.log | tail -5
[ $rc -eq 0 ] || exit $rc
for h in 0 1; do YCRDT_DEBUG_DECODE=1 YCRDT_SPEC_HINT=$h timeout -k 10 120 python3 scripts/probe_single.py 1 > gpurun_out/d10_$h.log 2>&1 || { echo "dbg rc=$?"; tail -3 gpurun_out/d10_$h.log; exit 1; }; echo "== hint $h"; grep "fastwalk" gpurun_out/d10_$h.log | tail -1; grep wall gpurun_out/d10_$h.log; done
YCRDT_DEBUG_DECODE=1 timeout -k 10 200 python3 bench.py --steps 1 --warmup 0 --only-headline > gpurun_out/db10.log 2>&1 || { echo "dbg bench rc=$?"; exit 1; }
echo "== head dbg"; grep "fastwalk" gpurun_out/db10.log | tail -1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p10_head -o run -- python3 bench.py --steps 3 --warmup 1 --only-headline > gpurun_out/b10.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/b10.log; exit 1; }
rm -f gpurun_out/p10_head/run_kernel_trace.csv
echo "== head"; python3 scripts/prof_top.py gpurun_out/p10_head/run_kernel_stats.csv 12
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p10_single -o run -- python3 scripts/probe_single.py 5 > gpurun_out/s10.log 2>&1 || { echo "single rc=$?"; tail -3 gpurun_out/s10.log; exit 1; }
rm -f gpurun_out/p10_single/run_kernel_trace.csv
echo "== single"; python3 scripts/prof_top.py gpurun_out/p10_single/run_kernel_stats.csv 6
