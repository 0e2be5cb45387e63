#!/bin/bash
# Round-5 GPU step (edited per call)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_corrupt.py tests/test_gpu_yata.py tests/test_gpu_arrays.py tests/test_gpu_edges.py tests/test_gpu_edges_fixtures.py tests/test_gpu_configs.py tests/test_gpu_exchange.py > gpurun_out/r05_tests.log 2>&1 || { grep -E "^E |FAIL|Error" gpurun_out/r05_tests.log | head -40; tail -5 gpurun_out/r05_tests.log; exit 1; }
tail -2 gpurun_out/r05_tests.log
timeout -k 10 400 python -u bench.py --gpus 2 --steps 3 --warmup 1 --only-headline --docs 8 > gpurun_out/r05_g2.json 2> gpurun_out/r05_g2.err || { tail -20 gpurun_out/r05_g2.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r05_g2.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['value'], d['config']['transport'], d['torch_loaded'])"
