#!/bin/bash
# CPU baseline on >= 1,000 home-steps of the bench workload (BASELINE.md CPU-baseline plan), on the
# GPU box's host cores (16 workers).  A heartbeat line every minute: the CPU leg prints nothing.
set -o pipefail
mkdir -p gpurun_out/cpu1000
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
timeout -k 10 900 python -u bench.py --cpu-seconds 700 --cpu-home-steps 1000 --steps 8 --warmup 2 > gpurun_out/cpu1000/bench.log 2>&1
rc=$?
kill $HB
tail -1 gpurun_out/cpu1000/bench.log | cut -c1-300
exit $rc
