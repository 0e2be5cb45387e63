#!/bin/bash
# the per-call GPU step (edited per experiment)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for sp in 2 1 8 0; do
  YCRDT_DIRECT_SPLIT=$sp timeout -k 10 300 python bench.py --only-headline --profile-phases --steps 6 --warmup 2 > gpurun_out/s_sp$sp.json 2> gpurun_out/s_sp$sp.err || { tail -20 gpurun_out/s_sp$sp.err; exit 1; }
  echo "split $sp"; python3 scripts/bench_summary.py gpurun_out/s_sp$sp.json | head -2 | cut -c1-200 || true
done
