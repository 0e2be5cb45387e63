#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
YCRDT_DEBUG_DECODE=1 timeout -k 10 120 python3 scripts/probe_single.py 1 > gpurun_out/d23.log 2>&1 || { echo "dbg rc=$?"; tail -3 gpurun_out/d23.log; exit 1; }
grep "fastwalk" gpurun_out/d23.log | tail -1
YCRDT_DEBUG_DECODE=1 timeout -k 10 200 python3 bench.py --steps 1 --warmup 0 --only-headline > gpurun_out/db23.log 2>&1 || { echo "dbg bench rc=$?"; exit 1; }
grep "fastwalk" gpurun_out/db23.log | tail -1
timeout -k 10 120 python3 scripts/probe_single.py 10 > gpurun_out/s23.log 2>&1 || { echo "single rc=$?"; exit 1; }
echo "== single"; grep -E "wall" gpurun_out/s23.log; grep -o "'decode.direct': [0-9.]*" gpurun_out/s23.log
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --only-headline > gpurun_out/b23.log 2>&1 || { echo "bench rc=$?"; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/b23.log").read().strip().splitlines()[-1])
print("bench", d["ms_per_step"], {k: v for k, v in d["phases_ms"].items() if k.startswith("decode")})
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p23_c4 -o run -- python3 scripts/probe_c4full.py 2 > gpurun_out/c4_23.log 2>&1 || { echo "c4 rc=$?"; tail -3 gpurun_out/c4_23.log; exit 1; }
rm -f gpurun_out/p23_c4/run_kernel_trace.csv
grep "merge ms" gpurun_out/c4_23.log | tail -1 | cut -c1-400
python3 scripts/prof_top.py gpurun_out/p23_c4/run_kernel_stats.csv 40 | grep -E "k_t|yata|k_y|climb|sib|huge|wdecode|k_direct"
