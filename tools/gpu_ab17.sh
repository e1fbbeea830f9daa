#!/bin/bash
# Round-6 A/B: the cell kernel with one v_cvt_flr_i32_f32 per image index instead of v_floor + v_cvt (flr)
# against the in-tree build on the RL action, order rotated; GPU tests on flr first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab17
DRAGG_LIB=$PWD/abl/flr.so timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab17/tests_flr.log 2>&1 || { tail -30 gpurun_out/ab17/tests_flr.log; exit 1; }
tail -1 gpurun_out/ab17/tests_flr.log
ROTATE=1 TAG=ab17r ROUNDS=3 ABARGS="--workload rl --steps 6 --warmup 1" bash tools/gpu_ab6.sh cur flr || exit 1
echo ab17-done
