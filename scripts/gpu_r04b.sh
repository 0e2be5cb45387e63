#!/bin/bash
# corrupt diag, the whole GPU suite, headline bench, kernel stats of the headline
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
[ -n "${DIAG:-}" ] && { timeout -k 10 300 python scripts/diag_corrupt.py || exit 1; }
bash scripts/gpu_tests.sh || exit 1
timeout -k 10 300 python -u bench.py --only-headline --steps 5 --warmup 2 > gpurun_out/r04_head.json 2> gpurun_out/r04_head.err
rc=$?; echo "[head] rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.loads(open('gpurun_out/r04_head.json').read().splitlines()[-1]);print(d['ms_per_step'],d['device_ms_per_step']);print(d['phases_ms'])"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG:-r04b} -o stats -- python3 bench.py --steps 3 --warmup 1 --only-headline > gpurun_out/prof_${TAG:-r04b}.log 2>&1
rc=$?; echo "[prof] rc=$rc"
f=$(ls gpurun_out/prof_${TAG:-r04b}/*/stats_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && head -30 "$f" | cut -c1-160
exit 0
