#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
YCRDT_DEBUG_DECODE=1 timeout -k 10 120 python3 scripts/probe_single.py 1 > gpurun_out/d23.log 2>&1 || { echo "dbg rc=$?"; tail -3 gpurun_out/d23.log; exit 1; }
grep "fastwalk" gpurun_out/d23.log | tail -1
YCRDT_DEBUG_DECODE=1 timeout -k 10 200 python3 bench.py --steps 1 --warmup 0 --only-headline > gpurun_out/db23.log 2>&1 || { echo "dbg bench rc=$?"; exit 1; }
grep "fastwalk" gpurun_out/db23.log | tail -1
timeout -k 10 120 python3 scripts/probe_single.py 10 > gpurun_out/s23.log 2>&1 || { echo "single rc=$?"; exit 1; }
