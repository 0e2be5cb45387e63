set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_json_rewrite.py tests/test_gpu_edges_fixtures.py tests/test_gpu_corrupt.py tests/test_gpu_anyform.py > gpurun_out/r6_t9.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 3 gpurun_out/r6_t9.log; [ $rc -eq 0 ] || { grep -n "FAILED\|Error\|assert" gpurun_out/r6_t9.log | head -30; exit $rc; }
