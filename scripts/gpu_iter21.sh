#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_yata.py tests/test_gpu_arrays.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_multidoc.py -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/t21.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/t21.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p21_c4 -o run -- python3 scripts/probe_c4full.py 2 > gpurun_out/c4_21.log 2>&1 || { echo "c4 rc=$?"; tail -3 gpurun_out/c4_21.log; exit 1; }
rm -f gpurun_out/p21_c4/run_kernel_trace.csv
grep "merge ms" gpurun_out/c4_21.log | tail -1 | cut -c1-500
python3 scripts/prof_top.py gpurun_out/p21_c4/run_kernel_stats.csv 40 | grep -E "k_t|yata|k_y|climb|sib|huge"
