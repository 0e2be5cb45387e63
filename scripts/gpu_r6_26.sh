set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/probe_single.py 30 > gpurun_out/r6_single.log 2>&1 || { tail -5 gpurun_out/r6_single.log; exit 1; }
cat gpurun_out/r6_single.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_single_prof -o single -- python3 scripts/probe_single.py 30 > gpurun_out/r6_single_prof.log 2>&1 || { tail -5 gpurun_out/r6_single_prof.log; exit 1; }
f=$(ls gpurun_out/r6_single_prof/*/single_kernel_stats.csv gpurun_out/r6_single_prof/single_kernel_stats.csv 2>/dev/null | head -1); echo "$f"; head -30 "$f" | cut -c1-150
