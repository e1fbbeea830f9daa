#!/bin/bash
# exactness tests + path counts + bench for a kernel change
set -o pipefail
mkdir -p gpurun_out
TAG=$1
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_proven.py tests/test_gpu_parity.py -m gpu -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/pytest_ex_$TAG.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_ex_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_ex_$TAG.log
timeout -k 10 200 python tools/count_paths.py 10000 12 24 7 > gpurun_out/paths_$TAG.log 2>&1 && timeout -k 10 200 python tools/count_paths.py 10000 12 24 7 rl >> gpurun_out/paths_$TAG.log 2>&1 || { echo PATHS_FAIL; tail -20 gpurun_out/paths_$TAG.log; exit 1; }
grep int_path gpurun_out/paths_$TAG.log
timeout -k 10 200 python -u bench.py --cpu-seconds 0 > gpurun_out/bench_$TAG.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-300
