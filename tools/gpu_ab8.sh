#!/bin/bash
# Round-6 A/B of the cell kernel's launch bounds on the RL action (cur = 4 blocks per CU at 128 VGPRs with
# spills; cell_lb3 / cell_lb2: 3 / 2 blocks per CU without), then the RL phase split of the mid launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab8
TAG=ab8r ROUNDS=${ROUNDS:-2} ABARGS="--workload rl --steps 6 --warmup 1" bash tools/gpu_ab6.sh "$@" || exit 1
timeout -k 10 300 python3 -u tools/phase_breakdown.py --rl --homes 10000 --horizon-hours 12 --month 7 --steps 4 --out gpurun_out/ab8/phase_rl.json > gpurun_out/ab8/phase_rl.log 2>&1 || { tail -5 gpurun_out/ab8/phase_rl.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ab8/phase_rl.json')); print(d['kernel_ms_mean'], d['phase_share'], d['phase_mean_cycles'])"
echo ab8-done
