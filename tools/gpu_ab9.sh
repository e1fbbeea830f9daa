#!/bin/bash
# Round-6 A/B: the in-tree build (dense back-pointers + no zero stores of unread slots) against dense2 (dense
# only) and base (before the dense rows) on the driver window and the full day of the 8-way shard holding
# home 7519; the RL action against beamcache (the beam's cost + bound cached for all its children) and
# cellrow (that + the cell row staged in LDS per stage).  GPU tests on the in-tree build and on cellrow first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab9
( while sleep 60; do echo "tick $(date +%T)" >> gpurun_out/ab9/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab9/tests.log 2>&1 || { tail -30 gpurun_out/ab9/tests.log; exit 1; }
tail -1 gpurun_out/ab9/tests.log
DRAGG_LIB=$PWD/abl/cellrow.so timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab9/tests_cellrow.log 2>&1 || { tail -30 gpurun_out/ab9/tests_cellrow.log; exit 1; }
tail -1 gpurun_out/ab9/tests_cellrow.log
TAG=ab9r ROUNDS=2 ABARGS="--workload rl --steps 6 --warmup 1" bash tools/gpu_ab6.sh cur beamcache cellrow || exit 1
TAG=ab9d ROUNDS=2 bash tools/gpu_ab6.sh cur dense2 base || exit 1
TAG=ab9s ROUNDS=2 ABARGS="--steps 96 --warmup 4 --shard-of 8 --shard-rank 7" bash tools/gpu_ab6.sh cur dense2 base || exit 1
echo ab9-done
