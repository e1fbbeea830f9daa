#!/bin/bash
# RL reward-price path on the GPU: tests, the configs[4] bench line, a configs[3]-sized step.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rl.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_rl.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_rl.log; exit 1; }
tail -3 gpurun_out/pytest_rl.log
timeout -k 10 300 python -u bench.py --workload rl --cpu-seconds 0 --steps 48 > gpurun_out/bench_rl.log 2>&1 || { tail -20 gpurun_out/bench_rl.log; exit 1; }
tail -1 gpurun_out/bench_rl.log
timeout -k 10 300 python -u bench.py --homes 100000 --horizon-hours 6 --steps 24 --cpu-seconds 0 > gpurun_out/bench_100k.log 2>&1 || { tail -20 gpurun_out/bench_100k.log; exit 1; }
tail -1 gpurun_out/bench_100k.log
