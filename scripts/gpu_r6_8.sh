set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/probe_fullstate.py nr:YCRDT_RANK_LAST=0 > gpurun_out/r6_fs5.log 2>&1 || { tail -20 gpurun_out/r6_fs5.log; exit 1; }
grep -v "^W2026\|^E2026" gpurun_out/r6_fs5.log | grep "ms, device\|{\|equal\|record mode" | cut -c1-300
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fastwalk.py tests/test_gpu_large_ds.py tests/test_gpu_chunk_path.py tests/test_gpu_predecode.py > gpurun_out/r6_t8.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 3 gpurun_out/r6_t8.log; [ $rc -eq 0 ] || { grep -n "FAILED\|Error\|assert" gpurun_out/r6_t8.log | head -30; exit $rc; }
