#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_yata.py tests/test_gpu_arrays.py tests/test_gpu_multidoc.py -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/t20.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/t20.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p20_c3 -o run -- python3 scripts/probe_c3.py 10000000 256 16 > gpurun_out/c3_20.log 2>&1 || { echo "c3 rc=$?"; tail -3 gpurun_out/c3_20.log; exit 1; }
rm -f gpurun_out/p20_c3/run_kernel_trace.csv
grep -E "device ms" gpurun_out/c3_20.log | tail -1 | cut -c1-400
python3 scripts/prof_top.py gpurun_out/p20_c3/run_kernel_stats.csv 40 | grep -E "k_t|yata|k_y|climb|sib|huge"
