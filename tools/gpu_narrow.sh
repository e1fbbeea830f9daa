#!/bin/bash
# exact step-function DP: focused GPU tests, then the full suite and the default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03b
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_exact.py -x -v --timeout 300 --timeout-method thread -k step_function > $OUT/pytest_steps.txt 2>&1 || { echo "step tests failed"; tail -30 $OUT/pytest_steps.txt; exit 1; }
grep -E "passed|failed|records solved" $OUT/pytest_steps.txt | tail -8
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -2 $OUT/pytest_gpu.txt
grep -E "exact step-function|ROUND_FAIL solves" $OUT/pytest_gpu.txt
timeout -k 10 300 python3 bench.py --steps 96 --warmup 0 --cpu-seconds 0 > $OUT/full96.json 2> $OUT/full96.err || { echo "full96 failed"; exit 1; }
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/driver20.json 2> $OUT/driver20.err || { echo "bench failed"; exit 1; }
for nw in 1 2 4; do
  DRAGG_WAVES_PER_HOME=$nw timeout -k 10 300 python3 bench.py --steps 96 --warmup 0 --cpu-seconds 0 --shard-of 8 > $OUT/shard8_nw$nw.json 2> $OUT/shard8_nw$nw.err || { echo "shard8 nw$nw failed"; exit 1; }
done
timeout -k 10 300 python3 bench.py --workload rl --steps 6 --warmup 1 --cpu-seconds 0 > $OUT/rl_smooth.json 2> $OUT/rl_smooth.err || { echo "rl failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_rl -o trace -- python3 bench.py --workload rl --steps 6 --warmup 1 --cpu-seconds 0 > $OUT/prof_rl.log 2>&1 || { echo "rl trace failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof96 -o trace -- python3 bench.py --steps 96 --warmup 0 --cpu-seconds 0 > $OUT/prof96.log 2>&1 || { echo "trace failed"; exit 1; }
python3 - <<'PY'
import json
for f in ["full96", "driver20", "shard8_nw1", "shard8_nw2", "shard8_nw4", "rl_smooth"]:
    d = json.load(open(f"gpurun_out/r03b/{f}.json"))
    print(f, round(d["value"] / 1e6, 3), "M/s", round(d["ms_per_step"], 4), "ms/step", d["status_counts"])
PY
DRAGG_LIB=varlib/sprof.so DRAGG_WAVES_PER_HOME=1 timeout -k 10 200 python3 tools/stage_prof.py --world 8 --steps 48 --out $OUT/stage_1250.json > /dev/null 2>&1 || { echo "stage prof failed"; exit 1; }
DRAGG_LIB=varlib/sprof.so timeout -k 10 200 python3 tools/stage_prof.py --world 1 --steps 48 --out $OUT/stage_10k.json > /dev/null 2>&1 || { echo "stage prof 10k failed"; exit 1; }
cat $OUT/stage_1250.json $OUT/stage_10k.json
echo narrow-done
