#!/bin/bash
# PMC passes over a short bench run (one counter group per rocprofv3 run, kernel-trace only).
# Usage: scripts/pmc.sh <tag>   → gpurun_out/pmc_<tag>/{sq,mem}/...
export TMPDIR=/tmp
tag=${1:-run}
out=gpurun_out/pmc_$tag
mkdir -p $out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $out/sq -o sq -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --fleet-pairs 0 > $out/sq.log 2>&1
echo "sq rc=$?"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o fetch -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --fleet-pairs 0 > $out/fetch.log 2>&1
echo "fetch rc=$?"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o write -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --fleet-pairs 0 > $out/write.log 2>&1
echo "write rc=$?"
find $out -name "*.csv" | head
