#!/bin/bash
# headline phases + single-document probe at several chunk sizes (after the GPU tests)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/iter_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 3 gpurun_out/iter_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --only-headline > gpurun_out/iter_head.log 2>&1 || { echo "head rc=$?"; tail -5 gpurun_out/iter_head.log; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/iter_head.log').read().strip().splitlines()[-1]);print('ms_per_step',d['ms_per_step'], 'roof', d['roofline']['frac']);print(d['phases_ms'])"
for cs in ${SCHUNKS:-}; do
  YCRDT_SCHUNK=$cs timeout -k 10 120 python3 scripts/probe_single.py 10 > gpurun_out/iter_single_$cs.log 2>&1
  echo "== single schunk $cs"; grep -E "wall" gpurun_out/iter_single_$cs.log; grep -o "'decode.direct': [0-9.]*" gpurun_out/iter_single_$cs.log
  YCRDT_SCHUNK=$cs timeout -k 10 120 python3 scripts/probe_single.py 10 base > gpurun_out/iter_single_base_$cs.log 2>&1
  echo "   base:"; grep -E "wall" gpurun_out/iter_single_base_$cs.log; grep -o "'decode.direct': [0-9.]*" gpurun_out/iter_single_base_$cs.log
done
