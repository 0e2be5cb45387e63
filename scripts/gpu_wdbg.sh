#!/bin/bash
# k_wdecode outcome counters (YCRDT_DEBUG_DECODE=1) on the per-op loop's merges
set -u
mkdir -p gpurun_out
PEROP_N=${PEROP_N:-300} YCRDT_DEBUG_DECODE=1 timeout -k 10 300 python3 scripts/probe_perop.py > gpurun_out/wdbg.log 2>&1 || exit 1
grep -c "wave: done 1 " gpurun_out/wdbg.log; grep -c "unsettled 1" gpurun_out/wdbg.log; grep -c "other 1" gpurun_out/wdbg.log
tail -4 gpurun_out/wdbg.log | cut -c1-300
