#!/bin/bash
# one C2 document: chunk size of the base snapshot's chunk path
set -u
mkdir -p gpurun_out
for c in 256 512 1024; do
  YCRDT_SCHUNK=$c timeout -k 10 200 python3 scripts/probe_single.py 10 > gpurun_out/schunk_$c.log 2>&1 || exit 1
  echo "== $c"; grep -E "wall" gpurun_out/schunk_$c.log; grep -o "'decode.direct': [0-9.]*, 'decode.chunk_wait': [0-9.]*" gpurun_out/schunk_$c.log
done
