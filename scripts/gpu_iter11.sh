#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/p11_sq -o run -- python3 bench.py --steps 1 --warmup 0 --only-headline > gpurun_out/p11.log 2>&1 || { echo "pmc rc=$?"; tail -5 gpurun_out/p11.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/p11_sq/*counter_collection.csv")[0]
rows = list(csv.DictReader(open(f)))
agg = {}
for r in rows:
    k = r["Kernel_Name"][:40]
    if not any(x in k for x in ("k_direct", "k_spec", "k_sync", "k_walk", "k_struct_decode", "k_seg_props", "k_resolve", "k_out_sizes")):
        continue
    agg.setdefault(k, {})
    agg[k][r["Counter_Name"]] = agg[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k, d in agg.items():
    print(k, {c: "%.3g" % v for c, v in sorted(d.items())})
PY
