#!/bin/bash
# Iteration run: dump the fixture objectives (tag $1), the GPU tests, the default bench line.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-cur}
timeout -k 10 300 python -u tools/dump_gpu_obj.py $TAG round > gpurun_out/dump.log 2>&1 || { echo DUMP_FAIL; tail -30 gpurun_out/dump.log; exit 1; }
timeout -k 10 200 python -u bench.py --cpu-seconds 0 > gpurun_out/bench_$TAG.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-400
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
