#!/bin/bash
# window-path tests, then the >= 1 B-item leg (opt-in bench flag)
set -u
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/windows.log 2>&1
rc=$?; echo "[windows] rc=$rc"; tail -n 8 gpurun_out/windows.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 900 python -u bench.py --steps 3 --warmup 1 --billion 1120 --no-per-op > gpurun_out/billion.log 2>&1
rc=$?; echo "[billion] rc=$rc"; tail -c 3000 gpurun_out/billion.log
