set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
PEROP_N=2000 timeout -k 10 300 python -u scripts/probe_perop.py > gpurun_out/r6_perop.log 2>&1 || { tail -5 gpurun_out/r6_perop.log; exit 1; }
cat gpurun_out/r6_perop.log | cut -c1-600
PEROP_N=300 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6_perop_prof -o perop -- python3 scripts/probe_perop.py > gpurun_out/r6_perop_prof.log 2>&1 || { tail -5 gpurun_out/r6_perop_prof.log; exit 1; }
python3 scripts/trace_last.py gpurun_out/r6_perop_prof 0
