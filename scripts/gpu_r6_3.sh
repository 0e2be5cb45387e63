set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 scripts/probe_fullstate.py a:YCRDT_FWC_WALK=256 b:YCRDT_FWC_WALK=128 e:YCRDT_FWC_WALK=96 c:YCRDT_FWC_WALK=256,YCRDT_SCHUNK=256 d:YCRDT_FWC_WALK=256,YCRDT_SPEC_HINT=0,YCRDT_SCHUNK=256 f:YCRDT_FWC_WALK=128,YCRDT_SCHUNK=256 > gpurun_out/r6_fs4.log 2>&1 || { tail -20 gpurun_out/r6_fs4.log; exit 1; }
grep -v "^W2026\|^E2026" gpurun_out/r6_fs4.log | grep "merge 1\|merge 2\|{\|record mode\|equal" | cut -c1-80,380-520
