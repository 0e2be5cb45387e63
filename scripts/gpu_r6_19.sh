set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/probe_small_large3.py > gpurun_out/r6_sl3.log 2>&1 || { tail -20 gpurun_out/r6_sl3.log; exit 1; }
grep -v "^W2026\|^E2026" gpurun_out/r6_sl3.log | cut -c1-1500
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ds_edges.py tests/test_gpu_large_ds.py tests/test_gpu_predecode.py tests/test_gpu_fastwalk.py tests/test_gpu_pending.py tests/test_gpu_parity.py tests/test_gpu_corrupt.py tests/test_gpu_json_rewrite.py tests/test_gpu_edges_fixtures.py > gpurun_out/r6_t19.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 3 gpurun_out/r6_t19.log; [ $rc -eq 0 ] || { grep -n "FAILED\|Error\|assert" gpurun_out/r6_t19.log | head -30; exit $rc; }
