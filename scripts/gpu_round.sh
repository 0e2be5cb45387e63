#!/bin/bash
# GPU-box routine: parity tests, bench, rocprofv3 kernel stats. Stops at the first step that
# ends in a fault/abort/timeout (134, 139, 124, 137); ordinary test failures (rc 1) continue.
set -u
mkdir -p gpurun_out
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  tail -n 4 "gpurun_out/$name.log"
  case $rc in 124|134|137|139) echo "fatal rc in $name, stopping"; exit $rc;; esac
  return 0
}
what=${1:-all}
if [[ $what == all || $what == tests ]]; then
  step gpu_tests 420 python -u -m pytest tests -v --timeout 240 --timeout-method thread -m gpu
fi
if [[ $what == all || $what == bench ]]; then
  step bench 300 python -u bench.py --steps 10 --warmup 2
fi
if [[ $what == all || $what == prof ]]; then
  export TMPDIR=/tmp
  step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --fleet-pairs 0
  rm -f gpurun_out/prof/run_kernel_trace.csv
fi
