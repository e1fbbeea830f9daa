#!/bin/bash
# Round-6 A/B: the cell kernel's pair-minimum row with +inf pads (no range test per duty lookup: cellpad) against
# the in-tree build on the RL action, order rotated; GPU tests on cellpad first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab16
DRAGG_LIB=$PWD/abl/cellpad.so timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab16/tests_cellpad.log 2>&1 || { tail -30 gpurun_out/ab16/tests_cellpad.log; exit 1; }
tail -1 gpurun_out/ab16/tests_cellpad.log
ROTATE=1 TAG=ab16r ROUNDS=3 ABARGS="--workload rl --steps 6 --warmup 1" bash tools/gpu_ab6.sh cur cellpad || exit 1
echo ab16-done
