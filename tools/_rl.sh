#!/bin/bash
set -o pipefail
OUT=gpurun_out/${T:-rl}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/rl_paths.py --steps 3 > $OUT/rl_paths.txt 2>&1 || { echo rl_paths failed; tail -5 $OUT/rl_paths.txt; exit 1; }
tail -3 $OUT/rl_paths.txt
TAG=$T TESTS=none LINES="rl" TRACE=rl bash tools/gpu_r05.sh
