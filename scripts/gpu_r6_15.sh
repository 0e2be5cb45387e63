set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/probe_small_large3.py > gpurun_out/r6_sl3.log 2>&1 || { tail -20 gpurun_out/r6_sl3.log; exit 1; }
grep -v "^W2026\|^E2026" gpurun_out/r6_sl3.log | cut -c1-1500
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_sl3 -o sl3 -- python3 $GRAFT_REPO_ROOT/scripts/probe_small_large3.py > $GRAFT_REPO_ROOT/gpurun_out/r6_sl3_prof.log 2>&1; echo "[prof] rc=$?"
