#!/bin/bash
# the per-call GPU step (edited per experiment): small-batch kernels A/B in one process
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/probe_small_ab.py 3 > gpurun_out/ab_small.log 2>&1 || exit 1
tail -4 gpurun_out/ab_small.log
