#!/bin/bash
# single-document decode: per-kernel times for the replica updates alone at several chunk sizes
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "all 256 1" "all 512 1" "all 1024 1" "all 512 0" "base 512 1"; do
  set -- $cfg
  tag="p7_$1_$2_$3"
  YCRDT_SCHUNK=$2 YCRDT_SPEC_EXACT=$3 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag -o run -- python3 scripts/probe_single.py 5 $1 > gpurun_out/$tag.log 2>&1 || { echo "$tag rc=$?"; tail -3 gpurun_out/$tag.log; exit 1; }
  rm -f gpurun_out/$tag/run_kernel_trace.csv
  echo "== $tag"; grep -E "wall" gpurun_out/$tag.log; grep -o "'decode.direct': [0-9.]*" gpurun_out/$tag.log
  python3 - "$tag" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"gpurun_out/{sys.argv[1]}/run_kernel_stats.csv")))
for r in rows[:7]:
    print("%-50s %5s %10.1f us" % (r['Name'][:50], r['Calls'], float(r['AverageNs']) / 1e3))
PY
done
