#!/bin/bash
# Run selected GPU test files: tools/gpu_tests.sh TAG test_file...
set -o pipefail
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -q -rP --timeout 600 --timeout-method thread > gpurun_out/pytest_sel_$TAG.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_sel_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_sel_$TAG.log
