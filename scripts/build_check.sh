#!/bin/bash
# local (CPU) gate before any GPU call: build every native piece, then the CPU test suite
set -e
cd "$(dirname "$0")/.."
make -s -j8 -C crdt_amd/csrc 2>&1 | grep -E "error" || true
test -f crdt_amd/libycrdt.so
make -s -C crdt_amd/workload >/dev/null
make -s -C crdt_amd/js >/dev/null
make -s -C oracle >/dev/null
timeout 900 python -m pytest tests -x -q -m "not gpu" 2>&1 | tail -1 | tee /tmp/cpu_tests.txt
grep -q " passed" /tmp/cpu_tests.txt && ! grep -q "failed" /tmp/cpu_tests.txt
