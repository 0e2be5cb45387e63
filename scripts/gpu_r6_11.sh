set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
PEROP_N=500,2000 timeout -k 10 300 python -u scripts/probe_perop.py > gpurun_out/r6_perop.log 2>&1 || { tail -20 gpurun_out/r6_perop.log; exit 1; }
grep -v "^W2026\|^E2026" gpurun_out/r6_perop.log | cut -c1-600
cd /tmp && PEROP_N=300 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_perop -o perop -- python3 $GRAFT_REPO_ROOT/scripts/probe_perop.py > $GRAFT_REPO_ROOT/gpurun_out/r6_perop_prof.log 2>&1; echo "[prof] rc=$?"
