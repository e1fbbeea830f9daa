#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_closed_loop.py tests/test_runner.py tests/test_gpu_step.py -m gpu -v -rP --timeout 300 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
rc=$?
grep -E "homes follow|PASS|FAIL|Error|assert" gpurun_out/pytest_new.log | head -40
tail -3 gpurun_out/pytest_new.log
exit $rc
