set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_predecode.py tests/test_gpu_view_reads.py tests/test_gpu_edges.py > gpurun_out/r6_t4.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 3 gpurun_out/r6_t4.log; [ $rc -eq 0 ] || { grep -n "FAILED\|Error\|assert" gpurun_out/r6_t4.log | head -30; exit $rc; }
timeout -k 10 400 python3 scripts/probe_small_large.py 30 > gpurun_out/r6_sl2.json 2> gpurun_out/r6_sl2.err || { tail -5 gpurun_out/r6_sl2.err; exit 1; }
cat gpurun_out/r6_sl2.json
