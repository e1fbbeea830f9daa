#!/bin/bash
# Fast GPU iteration: smoke, parity tests, bench default and H=24 without the CPU baseline.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 200 python -u bench.py --cpu-seconds 0 > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --cpu-seconds 0 --homes 10000 --horizon-hours 6 > gpurun_out/bench_h24.log 2>&1 || exit 1
tail -1 gpurun_out/smoke.log; tail -1 gpurun_out/pytest_gpu.log
echo quick-done
