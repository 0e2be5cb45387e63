#!/bin/bash
# C3 with the YATA loop statistics (YCRDT_DEBUG_YATA=1)
set -u
mkdir -p gpurun_out
YCRDT_DEBUG_YATA=1 timeout -k 10 300 python3 scripts/probe_c3.py 10000000 256 16 > gpurun_out/c3dbg.log 2>&1
rc=$?; echo "[c3dbg] rc=$rc"; grep -E "huge sibling|device ms" gpurun_out/c3dbg.log | head -4 | cut -c1-400
exit $rc
