#!/bin/bash
# Round-6 A/B: the mid launch's cell-bound passes with 64 key/cost buckets instead of 128 -- the beam pass
# (beam64), the exact pass (exact64), both (cell64) -- on the RL action, order rotated; GPU tests on cell64.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab13
DRAGG_LIB=$PWD/abl/cell64.so timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab13/tests_cell64.log 2>&1 || { tail -30 gpurun_out/ab13/tests_cell64.log; exit 1; }
tail -1 gpurun_out/ab13/tests_cell64.log
ROTATE=1 TAG=ab13r ROUNDS=2 ABARGS="--workload rl --steps 6 --warmup 1" bash tools/gpu_ab6.sh cur cell64 beam64 exact64 || exit 1
echo ab13-done
