set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in ab_prev/libycrdt_prev.so crdt_amd/libycrdt.so ab_prev/libycrdt_prev.so crdt_amd/libycrdt.so; do
  YCRDT_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --only-headline > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]);print('$lib', d['ms_per_step'], [(k['kernel'][4:], k['avg_launch_ms']) for k in d['roofline']['kernels']][:6])"
done
