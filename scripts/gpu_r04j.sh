#!/bin/bash
# YATA tests, C4 and C3 kernel traces
set -u
bash scripts/gpu_r04f.sh || exit $?
bash scripts/gpu_r04i.sh
