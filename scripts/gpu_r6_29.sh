set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wave_decode.py tests/test_gpu_decode_paths.py tests/test_gpu_ds_edges.py tests/test_gpu_json_rewrite.py tests/test_gpu_anyform.py > gpurun_out/r6_t29.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 2 gpurun_out/r6_t29.log; [ $rc -eq 0 ] || { grep -n "FAILED\|Error\|assert" gpurun_out/r6_t29.log | head -30; exit $rc; }
for lib in ab_prev/libycrdt_prev.so crdt_amd/libycrdt.so ab_prev/libycrdt_prev.so crdt_amd/libycrdt.so; do
  echo "== $lib"
  YCRDT_LIB=$PWD/$lib timeout -k 10 200 python -u scripts/probe_single.py 40 > gpurun_out/r6_s29.log 2>&1 || { tail -5 gpurun_out/r6_s29.log; exit 1; }
  grep -E "wall|parity" gpurun_out/r6_s29.log; grep -o "'decode.direct': [0-9.]*, 'decode.chunk_wait': [0-9.]*" gpurun_out/r6_s29.log
done
PEROP_N=2000 timeout -k 10 300 python -u scripts/probe_perop.py > gpurun_out/r6_perop29.log 2>&1 || { tail -5 gpurun_out/r6_perop29.log; exit 1; }
grep "ms/op" gpurun_out/r6_perop29.log
