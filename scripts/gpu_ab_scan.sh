#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for x in 1 0 1 0; do
  YCRDT_ROCPRIM_SCAN=$x timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --only-headline > gpurun_out/ab_$x.log 2>&1 || { echo "bench rc=$?"; exit 1; }
  python3 - "$x" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.log").read().strip().splitlines()[-1])
p = d.get("phases_ms")
print("rocprim" if sys.argv[1] == "1" else "lb     ", d["ms_per_step"], {k: p[k] for k in ("decode.structs", "merge.segment_props", "encode.sizes", "decode.direct")})
PY
done
