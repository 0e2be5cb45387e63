set -u
mkdir -p gpurun_out
for cs in 1024 512 256 128; do
  YCRDT_SCHUNK=$cs timeout -k 10 120 python3 scripts/probe_single.py 10 > gpurun_out/single_$cs.log 2>&1 || exit 1
  echo "== schunk $cs"; cat gpurun_out/single_$cs.log
done
