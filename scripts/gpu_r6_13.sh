set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/probe_single.py 20 > gpurun_out/r6_single.log 2>&1 || { tail -20 gpurun_out/r6_single.log; exit 1; }
grep -v "^W2026\|^E2026" gpurun_out/r6_single.log | cut -c1-1500
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_single -o single -- python3 $GRAFT_REPO_ROOT/scripts/probe_single.py 10 > $GRAFT_REPO_ROOT/gpurun_out/r6_single_prof.log 2>&1; echo "[prof] rc=$?"
