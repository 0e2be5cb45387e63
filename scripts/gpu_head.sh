#!/bin/bash
# headline merge only, phases printed
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --only-headline > gpurun_out/headline.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/headline.log; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/headline.log').read().strip().splitlines()[-1]);print('ms_per_step',d['ms_per_step']);print(d['phases_ms'])"
