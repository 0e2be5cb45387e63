#!/bin/bash
# iteration loop: GPU tests (stop at first failure), headline merge phases, single-document probe
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/iter_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 3 gpurun_out/iter_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --only-headline > gpurun_out/iter_head.log 2>&1 || { echo "head rc=$?"; tail -5 gpurun_out/iter_head.log; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/iter_head.log').read().strip().splitlines()[-1]);print('ms_per_step',d['ms_per_step'], 'roof', d['roofline']['frac']);print(d['phases_ms'])"
for m in ${DECODE_MODES:-default}; do
  if [ $m = default ]; then timeout -k 10 120 python3 scripts/probe_single.py 10 > gpurun_out/iter_single_$m.log 2>&1
  else YCRDT_DECODE=$m timeout -k 10 120 python3 scripts/probe_single.py 10 > gpurun_out/iter_single_$m.log 2>&1; fi
  echo "== single $m"; cat gpurun_out/iter_single_$m.log | cut -c1-400
done
