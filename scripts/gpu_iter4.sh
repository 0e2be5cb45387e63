#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_yata.py tests/test_gpu_arrays.py tests/test_gpu_exchange.py tests/test_gpu_chunk_path.py tests/test_gpu_decode_paths.py tests/test_gpu_view.py tests/test_gpu_view_reads.py -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/t4.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/t4.log | tail -8
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_single -o run -- python3 scripts/probe_single.py 10 > gpurun_out/prof_single.log 2>&1 || { echo "prof rc=$?"; tail -3 gpurun_out/prof_single.log; exit 1; }
rm -f gpurun_out/prof_single/run_kernel_trace.csv
grep -E "wall" gpurun_out/prof_single.log
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_single/run_kernel_stats.csv")))
for r in rows[:14]:
    print("%-50s %5s %9.1f us" % (r['Name'][:50], r['Calls'], float(r['AverageNs']) / 1e3))
PY
for se in 0 1; do
  YCRDT_SPEC_EXACT=$se timeout -k 10 120 python3 scripts/probe_single.py 10 > gpurun_out/single_se$se.log 2>&1
  echo "== spec_exact $se"; grep -E "wall" gpurun_out/single_se$se.log; grep -o "'decode.direct': [0-9.]*" gpurun_out/single_se$se.log
  YCRDT_SPEC_EXACT=$se timeout -k 10 120 python3 scripts/probe_single.py 10 base > gpurun_out/single_base_se$se.log 2>&1
  echo "   base"; grep -E "wall" gpurun_out/single_base_se$se.log; grep -o "'decode.direct': [0-9.]*" gpurun_out/single_base_se$se.log
done
