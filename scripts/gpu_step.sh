#!/bin/bash
# the per-call GPU step (edited per experiment): the round-end rehearsal, then the C2 PMC passes
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_final.sh || exit 1
rm -rf gpurun_out/pmc_r05c
bash scripts/pmc.sh r05c && python3 scripts/pmc_summary.py gpurun_out/pmc_r05c gpurun_out/pmc_r05c/c2_pmc.csv > gpurun_out/pmc_r05c/summary.txt 2>&1; tail -3 gpurun_out/pmc_r05c/summary.txt
