#!/bin/bash
# one C2 document and the per-op loop (small-merge latency)
set -u
mkdir -p gpurun_out
timeout -k 10 200 python3 scripts/probe_single.py 10 > gpurun_out/single.log 2>&1 || exit 1
cut -c1-700 gpurun_out/single.log
PEROP_N=${PEROP_N:-2000} timeout -k 10 300 python3 scripts/probe_perop.py > gpurun_out/perop.log 2>&1 || exit 1
grep "ms/op" gpurun_out/perop.log
