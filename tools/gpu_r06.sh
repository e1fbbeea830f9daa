#!/bin/bash
# Round-6 session: selected GPU tests (TESTS, "none" to skip), bench lines (LINES), optional
# kernel traces of lines (TRACE=<line names>), end-to-end runs (E2E=h24 h48: tools/e2e.py).  Each step under its own limit; results under
# gpurun_out/$TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r06}
mkdir -p $OUT
( while sleep 60; do echo "tick $(date +%T)" >> $OUT/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
TESTS=${TESTS:-tests}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest $TESTS -m gpu -x -v -s --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $OUT/smoke.log; exit 1; }
  tail -2 $OUT/smoke.log
fi
args_of() {
  case $1 in
    driver) echo --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 ;;
    drivers) echo --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-overlap ;;
    drivera) echo --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --steps-mode adaptive ;;
    full96a) echo --steps 96 --warmup 4 --cpu-seconds 0 --steps-mode adaptive ;;
    shard8r7a) echo --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 8 --shard-rank 7 --steps-mode adaptive ;;
    cfg3a) echo --homes 100000 --horizon-hours 6 --steps 24 --warmup 2 --cpu-seconds 0 --no-history ;;
    shard8r7) echo --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 8 --shard-rank 7 ;;
    shard8r7d) echo --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 8 --shard-rank 7 ;;
    shard8r0d) echo --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 8 --shard-rank 0 ;;
    shard8m7) echo --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 8 --shard-rank 7 ;;
    shard8m7s) echo --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 8 --shard-rank 7 --no-overlap ;;
    full96) echo --steps 96 --warmup 4 --cpu-seconds 0 ;;
    full96s) echo --steps 96 --warmup 4 --cpu-seconds 0 --no-overlap ;;
    shard8maxs) echo --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 8 --shard-max --no-overlap ;;
    exact96) echo --steps 96 --warmup 4 --cpu-seconds 0 --exact ;;
    shard8) echo --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 8 ;;
    shard8max) echo --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 8 --shard-max ;;
    shard4max) echo --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 4 --shard-max ;;
    shard8maxd) echo --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 8 --shard-max ;;
    shard4maxd) echo --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 4 --shard-max ;;
    shard2maxd) echo --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 2 --shard-max ;;
    shard2max) echo --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 2 --shard-max ;;
    rl) echo --workload rl --steps 6 --warmup 1 --cpu-seconds 0 ;;
    cfg1) echo --homes 1000 --horizon-hours 6 --month 1 --steps 96 --warmup 4 --cpu-seconds 0 ;;
    h24) echo --horizon-hours 6 --steps 96 --warmup 4 --cpu-seconds 0 ;;
    cfg3) echo --homes 100000 --horizon-hours 6 --steps 24 --warmup 2 --cpu-seconds 0 ;;
    gloo2) echo --gpus 2 --steps 20 --warmup 5 --cpu-seconds 0 ;;
    gloo2full) echo --gpus 2 --steps 96 --warmup 4 --cpu-seconds 0 ;;
  esac
}
run() { name=$1
  if [ "${name#gloo2}" != "$name" ]; then export DRAGG_BENCH_BACKEND=gloo; else unset DRAGG_BENCH_BACKEND; fi
  timeout -k 10 ${LINE_LIMIT:-400} python3 bench.py $(args_of $name) > $OUT/$name.out 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 1; }
  grep '^{' $OUT/$name.out | tail -1 > $OUT/$name.json
  python3 -c "
import json; d=json.load(open('$OUT/$name.json')); print('$name', round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],4), 'ms/step', 'kern', round(d['roofline']['kernel_ms'],4), (d.get('shard_emulation') or {}).get('max_over_shards'), {k: v for k, v in d['status_counts'].items() if v and k != 'optimal'})"; }
for spec in ${LINES:-full96}; do [ "$spec" = none ] || run $spec; done
for E in $E2E; do
  ref=""
  case $E in h24) hh=6; mo=1 ;; h48) hh=12; mo=7 ;; h24ref) hh=6; mo=1; ref=--reference-writer ;; h48ref) hh=12; mo=7; ref=--reference-writer ;; esac
  timeout -k 10 ${E2E_LIMIT:-600} python3 -u tools/e2e.py --homes ${E2E_HOMES:-10000} --horizon-hours $hh --month $mo $ref --out $OUT/e2e_$E.json > $OUT/e2e_$E.log 2>&1 || { echo "e2e $E failed"; tail -5 $OUT/e2e_$E.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/e2e_$E.json')); print('e2e $E', round(d['value'],3), 's', {k: round(v,3) for k, v in d['phases_s'].items()})"
done
for TR in $TRACE; do
  timeout -k 10 ${LINE_LIMIT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$TR -o run -- python3 bench.py $(args_of $TR) > $OUT/trace_$TR.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace_$TR.log; exit 1; }
  f=$(find $OUT/trace_$TR -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && head -8 "$f"
done
echo session-done
