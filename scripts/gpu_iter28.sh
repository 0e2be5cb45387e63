#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode_paths.py -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/t28.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/t28.log | tail -3
[ $rc -eq 0 ] || exit $rc
# default policy (wave for few small updates)
YCRDT_DEBUG_DECODE=1 timeout -k 10 120 python3 scripts/probe_single.py 1 > gpurun_out/d28.log 2>&1 || { echo "dbg rc=$?"; tail -3 gpurun_out/d28.log; exit 1; }
grep "fastwalk" gpurun_out/d28.log | tail -1
timeout -k 10 120 python3 scripts/probe_single.py 10 > gpurun_out/s28.log 2>&1 || { echo "single rc=$?"; exit 1; }
echo "== single"; grep -E "wall" gpurun_out/s28.log; grep -o "'decode.direct': [0-9.]*" gpurun_out/s28.log
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --only-headline > gpurun_out/b28.log 2>&1 || { echo "bench rc=$?"; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/b28.log").read().strip().splitlines()[-1])
print("bench", d["ms_per_step"], {k: v for k, v in d["phases_ms"].items() if k.startswith("decode")})
PY
