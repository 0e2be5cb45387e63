#!/bin/bash
# the per-call GPU step (edited per experiment): GPU tests, small-batch kernels A/B in one process
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_sec.log 2>&1; rc=$?
tail -3 gpurun_out/t_sec.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python3 scripts/probe_small_ab.py 3 > gpurun_out/ab_small.log 2>&1 || exit 1
tail -4 gpurun_out/ab_small.log
