#!/bin/bash
# one C2 document: ranked vs settled small-update decode
set -u
mkdir -p gpurun_out
for m in rank settle; do
  YCRDT_WDECODE=$m timeout -k 10 200 python3 scripts/probe_single.py 10 > gpurun_out/single_$m.log 2>&1 || exit 1
  echo "== $m"; cut -c1-600 gpurun_out/single_$m.log
done
