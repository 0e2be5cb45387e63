#!/bin/bash
# observer modes (Node facade), kernel stats of C4 (YATA) and of the per-op loop, PMC passes of the headline
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_napi.py -x -v --timeout 280 -k observer > gpurun_out/r04d_napi.log 2>&1
rc=$?; echo "[napi] rc=$rc"; tail -3 gpurun_out/r04d_napi.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- python3 scripts/probe_c4full.py 2 > gpurun_out/prof_c4.log 2>&1
rc=$?; echo "[c4] rc=$rc"; tail -3 gpurun_out/prof_c4.log; [ $rc -eq 0 ] || exit $rc
PEROP_N=300 timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_perop -o perop -- python3 scripts/probe_perop.py > gpurun_out/prof_perop.log 2>&1
rc=$?; echo "[perop] rc=$rc"; tail -4 gpurun_out/prof_perop.log; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc.sh r04d > gpurun_out/pmc_r04d.log 2>&1
rc=$?; echo "[pmc] rc=$rc"; tail -5 gpurun_out/pmc_r04d.log
exit $rc
