#!/bin/bash
# the per-call GPU step: the round-end rehearsal (every -m gpu test, smoke, the default bench)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_final.sh || exit 1
