#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/t22.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/t22.log | tail -5
[ $rc -eq 0 ] || exit $rc
for x in 0 1; do
  YCRDT_DIRECT_WAVE=$x timeout -k 10 120 python3 scripts/probe_single.py 10 > gpurun_out/s22_$x.log 2>&1 || { echo "single rc=$?"; exit 1; }
  echo "== lane=$x single"; grep -E "wall" gpurun_out/s22_$x.log; grep -o "'decode.direct': [0-9.]*" gpurun_out/s22_$x.log
  YCRDT_DIRECT_WAVE=$x timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --only-headline > gpurun_out/b22_$x.log 2>&1 || { echo "bench rc=$?"; exit 1; }
  python3 - "$x" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/b22_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print("bench", d["ms_per_step"], {k: v for k, v in d["phases_ms"].items() if k.startswith("decode")})
PY
done
