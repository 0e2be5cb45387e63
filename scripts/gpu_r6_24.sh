set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  env "$@" timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --only-headline > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]);print('$*', d['ms_per_step'], [(k['kernel'][4:], k['avg_launch_ms']) for k in d['roofline']['kernels']][:4])"
}
for i in 1 2; do
  run YCRDT_LIB=$PWD/abtest/libycrdt_r6start.so
  run YCRDT_LIB=$PWD/crdt_amd/libycrdt.so
done
timeout -k 10 300 python -u scripts/probe_small_large3.py > gpurun_out/r6_sl3.log 2>&1 || { tail -20 gpurun_out/r6_sl3.log; exit 1; }
grep -v "^W2026\|^E2026" gpurun_out/r6_sl3.log | head -1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ds_edges.py tests/test_gpu_large_ds.py tests/test_gpu_pending.py tests/test_gpu_parity.py > gpurun_out/r6_t24.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 2 gpurun_out/r6_t24.log; [ $rc -eq 0 ] || { grep -n "FAILED\|Error\|assert" gpurun_out/r6_t24.log | head -30; exit $rc; }
