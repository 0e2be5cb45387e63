#!/bin/bash
# register-window sizer: decode/parity tests, single doc, headline step
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_chunk_path.py tests/test_gpu_decode_paths.py tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_configs.py -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/t8.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/t8.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p8_single -o run -- python3 scripts/probe_single.py 5 > gpurun_out/s8.log 2>&1 || { echo "single rc=$?"; tail -3 gpurun_out/s8.log; exit 1; }
rm -f gpurun_out/p8_single/run_kernel_trace.csv
echo "== single"; grep -E "wall" gpurun_out/s8.log; grep -o "'decode.direct': [0-9.]*" gpurun_out/s8.log
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/p8_single/run_kernel_stats.csv")))
for r in rows[:8]:
    print("%-50s %5s %10.1f us" % (r['Name'][:50], r['Calls'], float(r['AverageNs']) / 1e3))
PY
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --only-headline > gpurun_out/b8.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/b8.log; exit 1; }
echo "== bench"; tail -1 gpurun_out/b8.log | cut -c1-400
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/b8.log").read().strip().splitlines()[-1])
print({k: d.get(k) for k in ("value", "ms_per_step")}, d.get("phases_ms") or d.get("config", {}).get("phases_ms"))
PY
