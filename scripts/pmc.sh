#!/bin/bash
# Kernel stats + PMC passes over a short bench run (one counter group per rocprofv3 run, kernel
# trace only; never combined with sys/runtime traces).
# Usage: scripts/pmc.sh <tag> [extra bench args]  → gpurun_out/pmc_<tag>/{stats,sq,fetch,write}/...
export TMPDIR=/tmp
tag=${1:-run}
shift
out=gpurun_out/pmc_$tag
mkdir -p $out
B="bench.py --steps 3 --warmup 1 --only-headline $*"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o stats -- python3 $B > $out/stats.log 2>&1 || exit 1
echo "stats ok"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $out/sq -o sq -- python3 $B > $out/sq.log 2>&1 || exit 1
echo "sq ok"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o fetch -- python3 $B > $out/fetch.log 2>&1 || exit 1
echo "fetch ok"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o write -- python3 $B > $out/write.log 2>&1 || exit 1
echo "write ok"
