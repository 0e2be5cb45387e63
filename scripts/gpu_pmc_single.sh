#!/bin/bash
# headline PMC passes (scripts/pmc.sh) + the single-document probe under rocprof (scripts/probe_single.sh)
set -u
mkdir -p gpurun_out
tag=${1:-r03}
bash scripts/pmc.sh $tag > gpurun_out/pmc_$tag.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_$tag.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc_$tag gpurun_out/pmc_$tag/summary.csv && head -25 gpurun_out/pmc_$tag/summary.csv
bash scripts/probe_single.sh
