#!/bin/bash
# selected GPU tests, then the full default bench line (all legs)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/full_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 15 gpurun_out/full_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/full_bench.log 2>&1
rc=$?; echo "[bench] rc=$rc"; tail -c 6000 gpurun_out/full_bench.log
