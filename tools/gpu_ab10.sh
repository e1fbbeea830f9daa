#!/bin/bash
# Round-6 A/B with the order rotated every round (tools/gpu_ab6.sh ROTATE=1): base (before the dense
# back-pointer rows), dense2 (dense rows), cur (dense rows + no zero stores of unread slots) on the driver
# window and on the full day of the 8-way shard holding home 7519; cur against beamcache on the RL action.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab10
export ROTATE=1
TAG=ab10d ROUNDS=3 bash tools/gpu_ab6.sh base dense2 cur || exit 1
TAG=ab10s ROUNDS=3 ABARGS="--steps 96 --warmup 4 --shard-of 8 --shard-rank 7" bash tools/gpu_ab6.sh base dense2 cur || exit 1
TAG=ab10r ROUNDS=2 ABARGS="--workload rl --steps 6 --warmup 1" bash tools/gpu_ab6.sh cur beamcache || exit 1
echo ab10-done
