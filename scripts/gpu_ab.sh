#!/bin/bash
# A/B of library builds on the C2 headline (bisect/<name>/libycrdt.so via YCRDT_LIB), alternated
set -u
mkdir -p gpurun_out
for v in ${AB_VARIANTS:-current nodeep current nodeep}; do
  if [ $v = current ]; then unset YCRDT_LIB; else export YCRDT_LIB=$PWD/bisect/$v/libycrdt.so; fi
  timeout -k 10 300 python -u bench.py --only-headline --steps 5 --warmup 2 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "[$v] rc=$rc"; tail -5 gpurun_out/ab_$v.err; exit $rc; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/ab_$v.json').read().splitlines()[-1]);p=d['phases_ms'];print('[$v]',d['ms_per_step'],{k:p[k] for k in ('decode.structs','decode.direct','merge.segment_props','encode.write','encode.sizes') if k in p})"
done
if [ -n "${AB_TESTS:-tests/test_gpu_yata.py tests/test_gpu_arrays.py tests/test_gpu_view.py}" ]; then
  unset YCRDT_LIB
  timeout -k 10 400 python -u -m pytest ${AB_TESTS:-tests/test_gpu_yata.py tests/test_gpu_arrays.py tests/test_gpu_view.py} -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; echo "[tests] rc=$rc $(grep -E 'passed|failed' gpurun_out/ab_tests.log | tail -1)"; exit $rc
fi
