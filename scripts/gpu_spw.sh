#!/bin/bash
# k_spec LDS window size variants (YCRDT_LIB), C4 and C3 phases
set -u
mkdir -p gpurun_out
for v in 64 96; do
  YCRDT_LIB=$PWD/crdt_amd/libycrdt_spw$v.so timeout -k 10 300 python3 scripts/probe_c4full.py 2 > gpurun_out/spw_c4_$v.log 2>&1 || exit 1
  echo "== $v"; grep "merge ms" gpurun_out/spw_c4_$v.log | cut -c1-120
  YCRDT_LIB=$PWD/crdt_amd/libycrdt_spw$v.so timeout -k 10 300 python3 scripts/probe_c3.py 10000000 256 16 > gpurun_out/spw_c3_$v.log 2>&1 || exit 1
  grep -E "device ms" gpurun_out/spw_c3_$v.log | head -1 | cut -c1-80
done
