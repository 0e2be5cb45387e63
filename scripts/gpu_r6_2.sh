set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/probe_fullstate.py > gpurun_out/r6_fs.log 2>&1; rc=$?
cat gpurun_out/r6_fs.log | tail -14; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fastwalk.py tests/test_gpu_large_ds.py tests/test_gpu_chunk_path.py > gpurun_out/r6_t2.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 5 gpurun_out/r6_t2.log; [ $rc -eq 0 ] || { grep -n "FAILED\|Error\|assert" gpurun_out/r6_t2.log | head -30; exit $rc; }
