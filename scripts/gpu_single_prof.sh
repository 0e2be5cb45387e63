#!/bin/bash
# kernel stats of one C2 document merged alone
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_single -o run -- python3 scripts/probe_single.py 5 > gpurun_out/prof_single.log 2>&1 || exit 1
rm -f gpurun_out/prof_single/run_kernel_trace.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_single/run_kernel_stats.csv")))
for r in rows[:14]:
    print("%-50s %5s %9.1f us" % (r['Name'][:50], r['Calls'], float(r['AverageNs']) / 1e3))
PY
