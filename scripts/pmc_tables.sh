#!/bin/bash
# PMC pass over the bench (kernel-trace style collection only; no sys/runtime tracing)
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc -o sq -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc/sq.log 2>&1
echo "rc=$?"
ls -R gpurun_out/pmc | head
