#!/bin/bash
# The committed CPU baseline (BASELINE.md CPU-baseline plan): bench.py --cpu-only on the GPU box's host
# cores (one worker process per core this job may use), >= 1,000 home-steps of a workload, HiGHS limit
# 300 s per solve (solves reaching it or the wall budget are counted separately).  No GPU use.
# A heartbeat line every 50 s (the CPU leg prints nothing until it ends).
# Usage: bash tools/gpu_cpu_baseline.sh TAG WALL_S [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; WALL=$2; shift 2
OUT=gpurun_out/cpu_$TAG
mkdir -p $OUT
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
timeout -k 10 $((WALL + 120)) python3 -u bench.py --cpu-only --cpu-seconds $WALL --cpu-home-steps ${HOME_STEPS:-1000} --cpu-milp-limit 300 "$@" > $OUT/cpu_baseline_full.json 2> $OUT/cpu.err
rc=$?
kill $HB
cut -c1-400 $OUT/cpu_baseline_full.json
exit $rc
