#!/bin/bash
# Per-op loop (bench per_op_leg shape): phase times of the last merges, then a kernel trace
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
PEROP_N=${PEROP_N:-2000} timeout -k 10 300 python3 scripts/probe_perop.py > gpurun_out/perop.log 2>&1 || exit 1
cat gpurun_out/perop.log
PEROP_N=${PEROP_N:-2000} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/perop_trace -o perop -- python3 scripts/probe_perop.py > gpurun_out/perop_trace.log 2>&1 || exit 1
echo "trace ok"
