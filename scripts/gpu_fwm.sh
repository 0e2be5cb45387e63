#!/bin/bash
# C4 with the decode statistics (multi-section fast walk)
set -u
mkdir -p gpurun_out
YCRDT_DEBUG_DECODE=1 timeout -k 10 300 python3 scripts/probe_c4full.py 1 > gpurun_out/fwm_c4.log 2>&1
rc=$?; echo "[c4] rc=$rc"; grep -E "ycrdt decode|merge ms" gpurun_out/fwm_c4.log | head -6 | cut -c1-250
exit $rc
