#!/bin/bash
# the GPU suite (optionally a -k / file selection in $@), one process, per-test timeout
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 25 gpurun_out/tests.log
exit $rc
