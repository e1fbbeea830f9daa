#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03c
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_exact.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread -k "step_function or narrow or round_fail or config4" > $OUT/pytest_focus.txt 2>&1 || { echo "focus tests failed"; tail -30 $OUT/pytest_focus.txt; exit 1; }
grep -E "passed|failed|step-function|configs\[4\]|ROUND_FAIL" $OUT/pytest_focus.txt | tail -12
timeout -k 10 300 python3 tools/launch_counts.py --steps 96 > $OUT/counts_rbo.txt 2>&1 || { echo "counts failed"; exit 1; }
tail -1 $OUT/counts_rbo.txt
timeout -k 10 300 python3 tools/launch_counts.py --steps 6 --rl > $OUT/counts_rl.txt 2>&1 || { echo "counts rl failed"; exit 1; }
tail -1 $OUT/counts_rl.txt
for lib in cache nocache; do
  DRAGG_LIB=$PWD/varlib/$lib.so timeout -k 10 300 python3 bench.py --steps 96 --warmup 0 --cpu-seconds 0 > $OUT/full96_$lib.json 2> $OUT/full96_$lib.err || { echo "full96 $lib failed"; exit 1; }
  DRAGG_LIB=$PWD/varlib/$lib.so timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/driver_$lib.json 2> $OUT/driver_$lib.err || { echo "driver $lib failed"; exit 1; }
  DRAGG_LIB=$PWD/varlib/$lib.so timeout -k 10 300 python3 bench.py --steps 96 --warmup 0 --cpu-seconds 0 --shard-of 8 > $OUT/shard8_$lib.json 2> $OUT/shard8_$lib.err || { echo "shard8 $lib failed"; exit 1; }
done
timeout -k 10 300 python3 bench.py --workload rl --steps 6 --warmup 1 --cpu-seconds 0 > $OUT/rl_smooth.json 2> $OUT/rl_smooth.err || { echo "rl failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof96 -o trace -- python3 bench.py --steps 96 --warmup 0 --cpu-seconds 0 > $OUT/prof96.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_rl -o trace -- python3 bench.py --workload rl --steps 6 --warmup 1 --cpu-seconds 0 > $OUT/prof_rl.log 2>&1 || { echo "rl trace failed"; exit 1; }
DRAGG_LIB=varlib/sprof.so DRAGG_WAVES_PER_HOME=1 timeout -k 10 200 python3 tools/stage_prof.py --world 8 --steps 48 --out $OUT/stage_1250.json > /dev/null 2>&1 || { echo "stage prof failed"; exit 1; }
python3 - <<'PY'
import json, csv
for f in ["full96_cache", "full96_nocache", "driver_cache", "driver_nocache", "shard8_cache", "shard8_nocache", "rl_smooth"]:
    d = json.load(open(f"gpurun_out/r03c/{f}.json"))
    print(f, round(d["value"] / 1e6, 3), "M/s", round(d["ms_per_step"], 4), "ms/step", d["status_counts"])
for f in ["prof96", "prof_rl"]:
    for r in list(csv.DictReader(open(f"gpurun_out/r03c/{f}/trace_kernel_stats.csv")))[:5]:
        print(f, r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us avg", round(float(r["MaxNs"]) / 1e3, 1), "max")
print(json.load(open("gpurun_out/r03c/stage_1250.json"))["cycles_per_stage_mean"])
PY
echo r03c-done
