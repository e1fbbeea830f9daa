#!/bin/bash
# Round-6 A/B: BEAM_K 24 / 36 against 32 on the RL action now that the beam caches every child's cost + bound
# (order rotated, 3 rounds); GPU tests on the better variant are run before adopting it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab15
ROTATE=1 TAG=ab15r ROUNDS=3 ABARGS="--workload rl --steps 6 --warmup 1" bash tools/gpu_ab6.sh cur beam24 beam36 || exit 1
echo ab15-done
