#!/bin/bash
# round-3 profiles: headline kernel stats + PMC passes, then the FETCH_SIZE calibration
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/pmc.sh r03c || { echo "pmc failed"; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc_r03c gpurun_out/pmc_r03c/summary.csv > gpurun_out/pmc_r03c/summary.txt
head -20 gpurun_out/pmc_r03c/summary.txt
(rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1 || true)
grep -oE "TCC_EA0?_[A-Z0-9_]+|TCC_BUBBLE[A-Z0-9_]*|TCC_REQ[A-Z0-9_]*" gpurun_out/avail.txt | sort -u | tr '\n' ' '; echo
cd scripts/calib
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c --kernel-trace --output-format csv -d ../../gpurun_out/calib_$c -o run -- ./calib_fetch > ../../gpurun_out/calib_$c.log 2>&1 || { echo "calib $c failed"; exit 1; }
done
cd ../..
python3 - <<'PY'
import csv, glob
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"gpurun_out/calib_{c}/*counter_collection.csv")[0]
    acc = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        acc[k] = acc.get(k, 0.0) + float(r["Counter_Value"])
    for k, v in acc.items():
        print(c, k, "KiB %.0f" % v, "bytes per request (64 Mi) %.2f" % (v * 1024 / (64 << 20)), "per streamed byte %.3f" % (v * 1024 / (1 << 30)))
PY
