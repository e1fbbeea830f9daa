#!/bin/bash
# Round-4 session: selected GPU tests (TESTS, default the step / edges / parity / proven-loop files),
# the driver's bench command, the full day (default and DRAGG_FLAG_EXACT), the 8-way shard, and the
# two-rank rehearsal of `bench.py --gpus 2` on one GPU (gloo).  Each step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04}
mkdir -p $OUT
( while sleep 60; do echo "tick $(date +%T)" >> $OUT/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
TESTS=${TESTS:-tests}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
run() { name=$1; shift; timeout -k 10 400 python3 bench.py "$@" > $OUT/$name.out 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 1; }
  grep '^{' $OUT/$name.out | tail -1 > $OUT/$name.json
  python3 -c "
import json; d=json.load(open('$OUT/$name.json')); print('$name', round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],4), 'ms/step', 'n_gpus', d['n_gpus'], d['config'].get('homes_per_rank'), {k: v for k, v in d['status_counts'].items() if v and k != 'optimal'})"; }
for spec in ${LINES:-driver full96 shard8 shard4 gloo2}; do
  case $spec in
    driver) run driver --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 ;;
    full96) run full96 --steps 96 --warmup 4 --cpu-seconds 0 ;;
    exact96) run exact96 --steps 96 --warmup 4 --cpu-seconds 0 --exact ;;
    shard8) run shard8 --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 8 ;;
    shard4) run shard4 --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 4 ;;
    rl) run rl --workload rl --steps 6 --warmup 1 --cpu-seconds 0 ;;
    gloo2) DRAGG_BENCH_BACKEND=gloo run gloo2 --gpus 2 --steps 20 --warmup 5 ;;
  esac
done
echo session-done
