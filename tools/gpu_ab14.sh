#!/bin/bash
# Round-6 A/B: the later launches' regular front DP (the RL tank chain, deferred TOU chains) with two 64-child
# chunks per pass, none held (tankilp3), order rotated: GPU tests on tankilp3, the RL action (3 rounds), the full day
# (2 rounds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab14
DRAGG_LIB=$PWD/abl/tankilp3.so timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab14/tests_tankilp3.log 2>&1 || { tail -30 gpurun_out/ab14/tests_tankilp3.log; exit 1; }
tail -1 gpurun_out/ab14/tests_tankilp3.log
export ROTATE=1
TAG=ab14r ROUNDS=3 ABARGS="--workload rl --steps 6 --warmup 1" bash tools/gpu_ab6.sh cur tankilp3 || exit 1
TAG=ab14f ROUNDS=2 ABARGS="--steps 96 --warmup 4" bash tools/gpu_ab6.sh cur tankilp3 || exit 1
echo ab14-done
