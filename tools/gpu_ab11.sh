#!/bin/bash
# Round-6 A/B of the steps modes (lag / adaptive / serial) with the adaptive start's flag reduced on a stream
# of its own, the order rotated every round: the driver window (3 rounds) and the full day (2 rounds, lag and
# adaptive).  The overlap tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab11
mkdir -p $OUT
( while sleep 60; do echo "tick $(date +%T)" >> $OUT/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_overlap.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
run() { name=$1; shift
  timeout -k 10 300 python3 bench.py --cpu-seconds 0 "$@" > $OUT/$name.out 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 1; }
  grep '^{' $OUT/$name.out | tail -1 > $OUT/$name.json
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', round(d['ms_per_step'],4), d.get('steps_mode'), d.get('lag_from_step'))"
}
M=(lag adaptive serial)
for r in 1 2 3; do
  for i in 0 1 2; do m=${M[$(( (i + r - 1) % 3 ))]}; run d_${m}.$r --steps 20 --warmup 5 --steps-mode $m || exit 1; done
done
for r in 1 2; do
  if [ $r = 1 ]; then o="lag adaptive"; else o="adaptive lag"; fi
  for m in $o; do run f_${m}.$r --steps 96 --warmup 4 --steps-mode $m || exit 1; done
done
echo ab11-done
