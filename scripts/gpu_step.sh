#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/probe_fullstate.py 2>&1 | grep -E "ycrdt decode|merge|chunk_wait" | head -3
timeout -k 10 300 python -u scripts/probe_c4.py > gpurun_out/r05_c4.log 2>&1; grep -E "ms wall" gpurun_out/r05_c4.log | head -5
