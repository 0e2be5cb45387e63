#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_chunk_path.py tests/test_gpu_decode_paths.py tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/t12.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/t12.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --only-headline > gpurun_out/b12.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/b12.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/b12.log").read().strip().splitlines()[-1])
print("bench", d["ms_per_step"], d.get("phases_ms"))
PY
for h in 0 1; do YCRDT_SPEC_HINT=$h timeout -k 10 120 python3 scripts/probe_single.py 10 > gpurun_out/s12_$h.log 2>&1 || { echo "single rc=$?"; exit 1; }; echo "== single hint $h"; grep wall gpurun_out/s12_$h.log; done
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/p12_sq -o run -- python3 bench.py --steps 1 --warmup 0 --only-headline > gpurun_out/p12.log 2>&1 || { echo "pmc rc=$?"; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/p12_sq/*counter_collection.csv")[0]
agg = {}
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:30]
    if not any(x in k for x in ("k_direct", "k_spec", "k_sync", "k_walk<false")):
        continue
    agg.setdefault(k, {})
    agg[k][r["Counter_Name"][3:]] = agg[k].get(r["Counter_Name"][3:], 0.0) + float(r["Counter_Value"])
for k, d in agg.items():
    print(k, {c: "%.3g" % v for c, v in sorted(d.items())})
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p12_head -o run -- python3 bench.py --steps 3 --warmup 1 --only-headline > gpurun_out/b12p.log 2>&1 || { echo "prof rc=$?"; exit 1; }
rm -f gpurun_out/p12_head/run_kernel_trace.csv
python3 scripts/prof_top.py gpurun_out/p12_head/run_kernel_stats.csv 10
