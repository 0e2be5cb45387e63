set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_corrupt.py tests/test_gpu_pending.py tests/test_gpu_ds_edges.py tests/test_gpu_edges.py tests/test_gpu_large_ds.py > gpurun_out/r6_t25.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 2 gpurun_out/r6_t25.log; [ $rc -eq 0 ] || { grep -n "FAILED\|Error\|assert" gpurun_out/r6_t25.log | head -30; exit $rc; }
timeout -k 10 300 python -u scripts/probe_small_large.py 30 > gpurun_out/r6_sl.log 2>&1 || { tail -5 gpurun_out/r6_sl.log; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/r6_sl.log').read().strip().splitlines()[-1]);print(d.get('small_into_large'))"
