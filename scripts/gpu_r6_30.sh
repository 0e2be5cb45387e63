set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for cs in 512 256 128 512 256 128; do
  echo "== YCRDT_SCHUNK=$cs"
  YCRDT_SCHUNK=$cs timeout -k 10 200 python -u scripts/probe_single.py 40 > gpurun_out/r6_sc.log 2>&1 || { tail -5 gpurun_out/r6_sc.log; exit 1; }
  grep -E "wall" gpurun_out/r6_sc.log; grep -o "'decode.direct': [0-9.]*, 'decode.chunk_wait': [0-9.]*, 'decode.bitmap': [0-9.]*" gpurun_out/r6_sc.log
done
