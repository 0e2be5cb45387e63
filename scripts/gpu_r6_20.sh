export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_r06i
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_r06i/stats -o stats -- python3 bench.py --steps 3 --warmup 1 --only-headline > gpurun_out/pmc_r06i/stats.log 2>&1 || exit 1
echo "stats ok"
