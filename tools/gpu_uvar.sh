#!/bin/bash
# step-function DP first-bound variants: stage profile + full day per variant library (varlib/)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-uvar}
mkdir -p $OUT
( while sleep 60; do echo "tick $(date +%T)" >> $OUT/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
for v in ${VARS:-060 065}; do
  DRAGG_LIB=varlib/sp$v.so timeout -k 10 200 python -u tools/step_prof.py --steps 50 > $OUT/sp$v.log 2>&1 || { echo SP_FAIL $v; tail -5 $OUT/sp$v.log; exit 1; }
  echo "sp$v $(tail -1 $OUT/sp$v.log | cut -c1-300)"
  DRAGG_LIB=varlib/u$v.so timeout -k 10 300 python3 bench.py --steps 96 --warmup 4 --cpu-seconds 0 > $OUT/u$v.json 2> $OUT/u$v.err || { echo BENCH_FAIL $v; tail -5 $OUT/u$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/u$v.json')); print('u$v', round(d['ms_per_step'],4), 'ms/step')"
done
