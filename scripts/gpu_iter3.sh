#!/bin/bash
# YATA / array / config / shard GPU tests, the C3 probe at 10 M values, the headline merge
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_yata.py tests/test_gpu_arrays.py tests/test_gpu_configs.py tests/test_gpu_shard.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/yata.log 2>&1
rc=$?; echo "yata rc=$rc"; tail -4 gpurun_out/yata.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 200 python3 scripts/probe_c3.py 10000000 > gpurun_out/c3.log 2>&1 || { echo "c3 rc=$?"; tail -5 gpurun_out/c3.log; exit 1; }
tail -6 gpurun_out/c3.log | cut -c1-900
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --only-headline > gpurun_out/iter_head.log 2>&1 || { echo "head rc=$?"; tail -5 gpurun_out/iter_head.log; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/iter_head.log').read().strip().splitlines()[-1]);print('ms_per_step',d['ms_per_step'], 'roof', d['roofline']['frac']);print(d['phases_ms'])"
