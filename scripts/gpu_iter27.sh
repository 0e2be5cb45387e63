#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
YCRDT_DIRECT_WAVE=1 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/p27 -o run -- python3 scripts/probe_single.py 1 > gpurun_out/p27.log 2>&1 || { echo "pmc rc=$?"; tail -3 gpurun_out/p27.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/p27/*counter_collection.csv")[0]
agg, disp = {}, {}
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:24]
    if not any(x in k for x in ("k_wdecode", "k_spec", "k_sync", "k_fastwalk", "k_direct")):
        continue
    agg.setdefault(k, {})
    agg[k][r["Counter_Name"][3:]] = agg[k].get(r["Counter_Name"][3:], 0.0) + float(r["Counter_Value"])
    disp.setdefault(k, set()).add(r["Dispatch_Id"])
for k, d in agg.items():
    n = len(disp[k])
    print(k, n, {c: "%.3g" % (v / n) for c, v in sorted(d.items())})
f = glob.glob("gpurun_out/p27/*kernel_trace.csv")[0]
for r in csv.DictReader(open(f)):
    if "wdecode" in r["Kernel_Name"] or "k_spec" in r["Kernel_Name"]:
        print(r["Kernel_Name"][:20], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, "us")
PY
