set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r6_full.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 3 gpurun_out/r6_full.log; [ $rc -eq 0 ] || { grep -n "FAILED\|Error" gpurun_out/r6_full.log | head -20; exit $rc; }
