#!/bin/bash
# the per-call GPU step: the round-end rehearsal (tests, smoke, bench), the small-batch A/B and a
# per-op kernel trace
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_final.sh || exit 1
timeout -k 10 300 python3 scripts/probe_small_ab.py 2 > gpurun_out/ab_small5.log 2>&1 || exit 1
tail -5 gpurun_out/ab_small5.log
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trp -- python3 scripts/probe_trace.py perop > gpurun_out/trp.log 2>&1 || exit 1
python3 scripts/trace_last.py gpurun_out/trp 0 > gpurun_out/tr_perop7.txt; rm -rf gpurun_out/trp
