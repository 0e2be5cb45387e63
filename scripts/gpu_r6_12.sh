set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_anyform.py tests/test_gpu_json_rewrite.py tests/test_gpu_shard.py tests/test_gpu_edges_fixtures.py tests/test_gpu_parity.py > gpurun_out/r6_t12.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 3 gpurun_out/r6_t12.log; [ $rc -eq 0 ] || { grep -n "FAILED\|Error\|assert" gpurun_out/r6_t12.log | head -30; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-per-op > gpurun_out/r6_b12.json 2> gpurun_out/r6_b12.err
rc=$?; echo "[bench] rc=$rc"; python3 -c "
import json;d=json.loads(open('gpurun_out/r6_b12.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d.get('device_ms_per_step'), [(k['kernel'], k['avg_launch_ms']) for k in d['roofline']['kernels']][:4])"
