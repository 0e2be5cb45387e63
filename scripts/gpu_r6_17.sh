set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_sl3
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_sl3 -o sl3 -- python3 $GRAFT_REPO_ROOT/scripts/probe_small_large3.py > $GRAFT_REPO_ROOT/gpurun_out/r6_sl3_prof.log 2>&1; echo "[prof] rc=$?"
