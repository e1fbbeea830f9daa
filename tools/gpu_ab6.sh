#!/bin/bash
# Round-6 A/B of library builds on one box: abl/<name>.so via DRAGG_LIB ("cur" = the in-tree build), each
# for the bench args in ABARGS, ROUNDS rounds interleaved.  Usage: bash tools/gpu_ab6.sh cur nobits ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-ab6}
mkdir -p $OUT
( while sleep 60; do echo "tick $(date +%T)" >> $OUT/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
LIBS=("$@")
n=${#LIBS[@]}
for r in $(seq 1 ${ROUNDS:-2}); do
  # ROTATE=1: round r starts at the (r-1)-th build, so that no build always runs first (a box's first runs
  # of a session were measured slower)
  order=()
  for i in $(seq 0 $((n - 1))); do
    if [ -n "$ROTATE" ]; then order+=("${LIBS[$(( (i + r - 1) % n ))]}"); else order+=("${LIBS[$i]}"); fi
  done
  for lib in "${order[@]}"; do
    if [ "$lib" = cur ]; then unset DRAGG_LIB; else export DRAGG_LIB=$PWD/abl/$lib.so; fi
    timeout -k 10 ${AB_LIMIT:-240} python3 -u bench.py --cpu-seconds 0 ${ABARGS:---steps 20 --warmup 5} > $OUT/$lib.$r.out 2> $OUT/$lib.$r.err || { echo "AB_FAIL $lib"; tail -5 $OUT/$lib.$r.err; exit 1; }
    grep '^{' $OUT/$lib.$r.out | tail -1 > $OUT/$lib.$r.json
    python3 -c "
import json; d=json.load(open('$OUT/$lib.$r.json')); print('$lib', $r, round(d['ms_per_step'],4), 'ms/step kern', round(d['roofline']['kernel_ms'],4), {k: v for k, v in d['status_counts'].items() if v and k != 'optimal'})"
  done
done
unset DRAGG_LIB
echo ab-done
