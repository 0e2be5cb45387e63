#!/bin/bash
# C3 and C4 merge phases (chunk-path changes)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python3 scripts/probe_c3.py 10000000 256 16 > gpurun_out/ch_c3.log 2>&1
rc=$?; echo "[c3] rc=$rc"; grep -E "device ms" gpurun_out/ch_c3.log | head -2 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/probe_c4full.py 2 > gpurun_out/ch_c4.log 2>&1
rc=$?; echo "[c4] rc=$rc"; grep "merge ms" gpurun_out/ch_c4.log | cut -c1-300
exit $rc
