#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_chunk_path.py tests/test_gpu_decode_paths.py tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_multidoc.py tests/test_gpu_merge.py -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/t16.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/t16.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --only-headline > gpurun_out/b16.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/b16.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/b16.log").read().strip().splitlines()[-1])
print("bench", d["ms_per_step"], d.get("phases_ms", {}).get("decode.direct"))
PY
timeout -k 10 120 python3 scripts/probe_single.py 10 > gpurun_out/s16.log 2>&1 || { echo "single rc=$?"; exit 1; }; echo "== single"; grep -E "wall" gpurun_out/s16.log
for h in 2 0; do
  YCRDT_SPEC_HINT=$h YCRDT_DEBUG_DECODE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p16_$h -o run -- python3 scripts/probe_c4full.py 1 > gpurun_out/c16_$h.log 2>&1 || { echo "c4 rc=$?"; tail -3 gpurun_out/c16_$h.log; exit 1; }
  rm -f gpurun_out/p16_$h/run_kernel_trace.csv
  echo "== c4 hint $h"; grep "merge ms" gpurun_out/c16_$h.log | cut -c1-120; grep fastwalk gpurun_out/c16_$h.log | tail -1
  python3 scripts/prof_top.py gpurun_out/p16_$h/run_kernel_stats.csv 6
done
