set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
YCRDT_DEBUG_DECODE=1 timeout -k 10 300 python -u scripts/probe_small_large3.py > gpurun_out/r6_sl3d.log 2>&1 || { tail -20 gpurun_out/r6_sl3d.log; exit 1; }
grep "ds headers" gpurun_out/r6_sl3d.log | tail -3
