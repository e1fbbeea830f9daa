#!/bin/bash
# exact step-function DP iteration: its stage profile (DRAGG_STEP_PROF variant), the exactness tests
# that take it, the full day
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-narrow}
mkdir -p $OUT
( while sleep 60; do echo "tick $(date +%T)" >> $OUT/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
if [ -f varlib/stprof.so ]; then
  DRAGG_LIB=varlib/stprof.so timeout -k 10 300 python -u tools/step_prof.py --steps 50 > $OUT/step_prof.log 2>&1 || { echo STEPPROF_FAIL; tail -20 $OUT/step_prof.log; exit 1; }
  tail -2 $OUT/step_prof.log
fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_joint.py tests/test_gpu_exact.py tests/test_gpu_edges.py tests/test_gpu_configs.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
grep -E "step-function|narrow-set" $OUT/pytest.log | head -4
timeout -k 10 300 python3 bench.py --steps 96 --warmup 4 --cpu-seconds 0 > $OUT/full96.json 2> $OUT/full96.err || { echo BENCH_FAIL; tail -5 $OUT/full96.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/full96.json')); print('full96', round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],4), 'ms/step')"
for v in ${EXTRA:-shard8}; do
  case $v in
    shard8) timeout -k 10 300 python3 bench.py --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 8 > $OUT/$v.json 2> $OUT/$v.err || { echo BENCH_FAIL $v; tail -5 $OUT/$v.err; exit 1; } ;;
  esac
  python3 -c "import json; d=json.load(open('$OUT/$v.json')); print('$v', round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],4), 'ms/step')"
done
