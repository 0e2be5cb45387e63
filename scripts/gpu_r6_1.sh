set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ds_edges.py tests/test_gpu_large_ds.py tests/test_gpu_edges.py tests/test_gpu_pending.py > gpurun_out/r6_t1.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 5 gpurun_out/r6_t1.log; [ $rc -eq 0 ] || { grep -n "FAILED\|Error" gpurun_out/r6_t1.log | head -30; exit $rc; }
timeout -k 10 300 python -u bench.py --only-headline --steps 10 --warmup 2 --profile-phases > gpurun_out/r6_b1.json 2> gpurun_out/r6_b1.err || { tail -20 gpurun_out/r6_b1.err; exit 1; }
python3 scripts/bench_summary.py gpurun_out/r6_b1.json
