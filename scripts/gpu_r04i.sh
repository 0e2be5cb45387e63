#!/bin/bash
# C3 at full size (10 M values) under kernel tracing: the YATA breakdown
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- python3 scripts/probe_c3.py 10000000 256 16 > gpurun_out/prof_c3.log 2>&1
rc=$?; echo "[c3] rc=$rc"; grep -E "merge|phases|ms" gpurun_out/prof_c3.log | tail -6 | cut -c1-600
exit $rc
