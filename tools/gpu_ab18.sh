#!/bin/bash
# Round-6 A/B: the cell kernel's duty minimum by three v_min3_f32 instead of seven v_min_f32 (min3) against the
# in-tree build on the RL action, order rotated; GPU tests on min3 first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab18
DRAGG_LIB=$PWD/abl/min3.so timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab18/tests_min3.log 2>&1 || { tail -30 gpurun_out/ab18/tests_min3.log; exit 1; }
tail -1 gpurun_out/ab18/tests_min3.log
ROTATE=1 TAG=ab18r ROUNDS=3 ABARGS="--workload rl --steps 6 --warmup 1" bash tools/gpu_ab6.sh cur min3 || exit 1
echo ab18-done
