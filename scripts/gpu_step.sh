#!/bin/bash
# the per-call GPU step: GPU tests, the small-batch A/B, a per-op kernel trace
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_nf.log 2>&1; rc=$?
tail -3 gpurun_out/t_nf.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python3 scripts/probe_small_ab.py 2 > gpurun_out/ab_small6.log 2>&1 || exit 1
tail -5 gpurun_out/ab_small6.log
timeout -k 10 200 python3 -c "
import sys; sys.path.insert(0, '.')
import bench, crdt_amd
bench._yjs_perop = lambda n: None
r = bench.per_op_leg(crdt_amd.Engine(), (500, 2000))
print({k: (v['ops_per_s'], v['breakdown']['device_ms_per_op'], v['breakdown']['host_ms_per_op']) for k, v in r.items()})
" > gpurun_out/perop_nf.log 2>&1 || exit 1
cat gpurun_out/perop_nf.log
