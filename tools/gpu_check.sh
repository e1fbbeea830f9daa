#!/bin/bash
# One GPU session: parity tests, phase breakdown, the default bench line (with CPU baseline)
# and a few variants.  Every GPU step under its own time limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 200 python -u tools/phase_breakdown.py --homes 10000 --horizon-hours 12 --month 7 --steps 6 --out gpurun_out/phase_jul_h48_direct.json > gpurun_out/phase2.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --cpu-seconds 0 --month 1 > gpurun_out/bench_jan.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --cpu-seconds 0 --homes 1000 --horizon-hours 6 --month 1 > gpurun_out/bench_cfg2.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --cpu-seconds 0 --homes 10000 --horizon-hours 6 > gpurun_out/bench_h24.log 2>&1 || exit 1
echo check-done
