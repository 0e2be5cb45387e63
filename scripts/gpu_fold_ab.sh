#!/bin/bash
# per-op loop: copies folded into the merge's last synchronisation, or after it
set -u
mkdir -p gpurun_out
for r in 1 2; do
for f in 0 1; do
  YCRDT_NO_FOLD=$f PEROP_N=2000 timeout -k 10 300 python3 scripts/probe_perop.py > gpurun_out/fold_$f.log 2>&1 || exit 1
  echo "nofold=$f $(grep 'ms/op' gpurun_out/fold_$f.log)"
done
done
