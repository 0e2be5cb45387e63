#!/bin/bash
# read-request sizes at the L2's memory side (TCC_EA0_RDREQ by size) for the calibration kernels
# and the headline merge: true fetched bytes = 32 * n32 + 64 * n64 + 128 * n128
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
(cd scripts/calib && timeout -s KILL 60 rocprofv3 --pmc $C --kernel-trace --output-format csv -d ../../gpurun_out/rdreq_calib -o run -- ./calib_fetch > ../../gpurun_out/rdreq_calib.log 2>&1) || { echo "calib failed"; tail -5 gpurun_out/rdreq_calib.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/rdreq_head -o run -- python3 bench.py --steps 3 --warmup 1 --only-headline > gpurun_out/rdreq_head.log 2>&1 || { echo "head failed"; tail -5 gpurun_out/rdreq_head.log; exit 1; }
python3 scripts/rdreq_summary.py gpurun_out/rdreq_calib gpurun_out/rdreq_calib/summary.csv
python3 scripts/rdreq_summary.py gpurun_out/rdreq_head gpurun_out/rdreq_head/summary.csv | head -25
