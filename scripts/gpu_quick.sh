#!/bin/bash
# Quick GPU iteration: parity tests, the single-document probe at several chunk sizes, the
# headline merge alone. Stops at the first fault / abort / timeout.
set -u
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -n 3 "gpurun_out/$name.log"
  case $rc in 124|134|137|139) echo "fatal rc in $name, stopping"; exit $rc;; esac
  return 0
}
step gpu_tests 420 python -u -m pytest tests -x -q --timeout 240 --timeout-method thread -m gpu
for cs in ${SCHUNKS:-}; do YCRDT_SCHUNK=$cs step single_$cs 120 python3 scripts/probe_single.py 10; done
step single 120 python3 scripts/probe_single.py 10
step headline 300 python -u bench.py --steps 10 --warmup 2 --only-headline
