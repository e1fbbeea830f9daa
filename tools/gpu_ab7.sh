#!/bin/bash
# Round-6 A/B of the dense back-pointer rows (+ the one-barrier cell rows): the GPU tests on the
# variant, then the driver window and the RL action, cur against the variants (tools/gpu_ab6.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab7
V=${VARIANT:-dense_cellb}
DRAGG_LIB=$PWD/abl/$V.so timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab7/tests_$V.log 2>&1 || { tail -30 gpurun_out/ab7/tests_$V.log; exit 1; }
tail -2 gpurun_out/ab7/tests_$V.log
TAG=ab7d ROUNDS=${ROUNDS:-2} bash tools/gpu_ab6.sh "$@" || exit 1
TAG=ab7r ROUNDS=${ROUNDS:-2} ABARGS="--workload rl --steps 6 --warmup 1" bash tools/gpu_ab6.sh "$@" || exit 1
echo ab7-done
