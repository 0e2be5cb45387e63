#!/bin/bash
# YATA / view / array tests, then C4 kernel stats (YATA changes)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_yata.py tests/test_gpu_arrays.py tests/test_gpu_view.py tests/test_gpu_view_reads.py tests/test_gpu_shard.py tests/test_gpu_configs.py -x -v --timeout 280 --timeout-method thread > gpurun_out/r04f_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "passed|failed" gpurun_out/r04f_tests.log | tail -2; [ $rc -eq 0 ] || { tail -30 gpurun_out/r04f_tests.log; exit $rc; }
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4f -o c4 -- python3 scripts/probe_c4full.py 2 > gpurun_out/prof_c4f.log 2>&1
rc=$?; echo "[c4] rc=$rc"; grep "merge ms" gpurun_out/prof_c4f.log | cut -c1-400
exit $rc
