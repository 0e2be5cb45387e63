set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wave_decode.py > gpurun_out/r6_t32.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "passed|failed|PASSED|FAILED" gpurun_out/r6_t32.log | tail -n 20; exit $rc
