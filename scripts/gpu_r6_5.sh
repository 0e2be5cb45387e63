set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu "tests/test_gpu_predecode.py::test_predecode_pending" > gpurun_out/r6_t5.log 2>&1
grep -n "differ\|Error" gpurun_out/r6_t5.log | head -5; tail -3 gpurun_out/r6_t5.log
