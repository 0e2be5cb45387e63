#!/bin/bash
# kernel stats of the C4 (BASELINE scale) and C3 legs, one rocprof run each
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4full -o run -- python3 scripts/probe_c4full.py 2 > gpurun_out/prof_c4full.log 2>&1 || { echo "c4 rc=$?"; tail -5 gpurun_out/prof_c4full.log; exit 1; }
rm -f gpurun_out/prof_c4full/run_kernel_trace.csv
grep "merge ms" gpurun_out/prof_c4full.log | cut -c1-600
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_c4full/run_kernel_stats.csv")))
for r in rows[:25]:
    print("%-60s %5s %10.1f us %6.1f%%" % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3, float(r['Percentage'])))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python3 scripts/probe_c3.py 10000000 > gpurun_out/prof_c3.log 2>&1 || { echo "c3 rc=$?"; tail -5 gpurun_out/prof_c3.log; exit 1; }
rm -f gpurun_out/prof_c3/run_kernel_trace.csv
tail -3 gpurun_out/prof_c3.log | cut -c1-600
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_c3/run_kernel_stats.csv")))
for r in rows[:25]:
    print("%-60s %5s %10.1f us %6.1f%%" % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3, float(r['Percentage'])))
PY
