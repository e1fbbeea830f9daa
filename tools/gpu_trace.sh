#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run.  Usage: bash tools/gpu_trace.sh TAG [bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
OUT=gpurun_out/trace_$TAG
mkdir -p $OUT
ARGS=${@:-"--homes 10000 --horizon-hours 12 --month 7 --steps 6 --warmup 1 --cpu-seconds 0"}
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o trace -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
find $OUT -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200
