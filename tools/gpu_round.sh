#!/bin/bash
# Round check: smoke, every GPU test, the default bench line (with the CPU baseline), the RL
# bench line and its rocprofv3 kernel trace.  Each GPU step under its own limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out/prof_rl
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rl -o rl -- python3 bench.py --workload rl --steps 24 --cpu-seconds 0 > gpurun_out/prof_rl/bench_rl.log 2>&1 || { tail -20 gpurun_out/prof_rl/bench_rl.log; exit 1; }
tail -1 gpurun_out/prof_rl/bench_rl.log
echo round-done
