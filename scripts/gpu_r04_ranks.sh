#!/bin/bash
# headline check, lazy / parity tests, then bench.py --gpus 2 (two ranks on the one device)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --only-headline --steps 5 --warmup 2 > gpurun_out/r04_head.json 2> gpurun_out/r04_head.err
rc=$?; echo "[head] rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/r04_head.json'));print(d['ms_per_step'],d['phases_ms'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_merge.py tests/test_gpu_diff_batch.py tests/test_gpu_exchange.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_t.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 5 gpurun_out/r04_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --gpus 2 --steps 3 --warmup 1 --fleet-docs 200000 > gpurun_out/r04_g2.json 2> gpurun_out/r04_g2.err
rc=$?; echo "[gpus2] rc=$rc"; tail -n 5 gpurun_out/r04_g2.err; python -c "
import json;d=json.load(open('gpurun_out/r04_g2.json'));print(d['n_gpus'],d['value'],d['ms_per_step']);[print(r['rank'],r['ms_per_step'],r['phases_ms']) for r in d['ranks']];print(d['c4_sharded']);print(d['fleet_ranks'])"
exit $rc
