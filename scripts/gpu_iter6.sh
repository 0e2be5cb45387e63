#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_chunk_path.py tests/test_gpu_decode_paths.py tests/test_gpu_parity.py tests/test_gpu_multidoc.py tests/test_gpu_merge.py tests/test_gpu_edges.py -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/t6.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/t6.log | tail -8
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 120 python3 scripts/probe_single.py 10 > gpurun_out/s6.log 2>&1; echo "== single"; grep -E "wall" gpurun_out/s6.log; grep -o "'decode.direct': [0-9.]*" gpurun_out/s6.log
for hint in 1 0; do
  YCRDT_SPEC_HINT=$hint timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4h$hint -o run -- python3 scripts/probe_c4full.py 1 > gpurun_out/c4h$hint.log 2>&1 || { echo "c4 rc=$?"; tail -3 gpurun_out/c4h$hint.log; exit 1; }
  rm -f gpurun_out/prof_c4h$hint/run_kernel_trace.csv
  echo "== c4 hint $hint"; grep "merge ms" gpurun_out/c4h$hint.log | cut -c1-200
  python3 - "$hint" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"gpurun_out/prof_c4h{sys.argv[1]}/run_kernel_stats.csv")))
for r in rows[:8]:
    print("%-50s %5s %10.1f us" % (r['Name'][:50], r['Calls'], float(r['AverageNs']) / 1e3))
PY
done
