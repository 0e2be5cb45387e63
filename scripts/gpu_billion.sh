#!/bin/bash
# the >= 1 B-item single-pass leg (opt-in bench flag); progress lines on stderr every ~100 documents
set -u
mkdir -p gpurun_out
timeout -k 10 1000 python -u bench.py --steps 3 --warmup 1 --billion 1120 --no-per-op > gpurun_out/billion.json 2> gpurun_out/billion.err
rc=$?; echo "[billion] rc=$rc"; tail -n 30 gpurun_out/billion.err; tail -c 3000 gpurun_out/billion.json
exit $rc
