#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/t17.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/t17.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --only-headline > gpurun_out/b17.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/b17.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/b17.log").read().strip().splitlines()[-1])
print("bench", d["ms_per_step"], d.get("phases_ms"))
PY
timeout -k 10 120 python3 scripts/probe_single.py 10 > gpurun_out/s17.log 2>&1 || { echo "single rc=$?"; exit 1; }; echo "== single"; grep -E "wall" gpurun_out/s17.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p17_head -o run -- python3 bench.py --steps 3 --warmup 1 --only-headline > gpurun_out/b17p.log 2>&1 || { echo "prof rc=$?"; exit 1; }
rm -f gpurun_out/p17_head/run_kernel_trace.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/p17_head/run_kernel_stats.csv")))
print("launches per merge", sum(int(r["Calls"]) for r in rows) / 4)
for r in rows:
    if "scan_lb" in r["Name"] or "rocprim" in r["Name"]:
        print(r["Calls"], r["Name"][:80], round(float(r["AverageNs"]) / 1e3, 1))
PY
