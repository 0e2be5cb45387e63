#!/bin/bash
# A/B of library builds (bisect/<name>/libycrdt.so, via YCRDT_LIB) on one failing test
set -u
mkdir -p gpurun_out
T="tests/test_gpu_yata.py::test_gpu_yata_large_sibling_group"
for v in current climb small wave tk current; do
  if [ $v = current ]; then unset YCRDT_LIB; else export YCRDT_LIB=$PWD/bisect/$v/libycrdt.so; fi
  timeout -k 10 200 python -u -m pytest "$T" -x -q --timeout 180 > gpurun_out/bisect_$v.log 2>&1
  rc=$?; echo "[$v] rc=$rc $(grep -E 'passed|failed' gpurun_out/bisect_$v.log | tail -1)"
  [ $rc -le 1 ] || exit $rc
done
exit 0
