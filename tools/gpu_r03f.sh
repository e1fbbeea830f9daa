#!/bin/bash
# step-DP profile in exact mode + the default path's bench lines after the narrow-policy change
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03f
mkdir -p $OUT
DRAGG_LIB=varlib/stprof.so timeout -k 10 300 python3 tools/step_prof.py --exact --steps 24 > $OUT/step_prof.txt 2>&1 || { echo "step prof failed"; tail -5 $OUT/step_prof.txt; exit 1; }
tail -1 $OUT/step_prof.txt
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
timeout -k 10 300 python3 bench.py --steps 96 --warmup 0 --cpu-seconds 0 > $OUT/full96.json 2> $OUT/full96.err || { echo "full96 failed"; exit 1; }
timeout -k 10 300 python3 bench.py --workload rl --steps 6 --warmup 1 --cpu-seconds 0 > $OUT/rl.json 2> $OUT/rl.err || { echo "rl failed"; exit 1; }
timeout -k 10 300 python3 tools/launch_counts.py --steps 96 > $OUT/launch_counts.txt 2>&1 || { echo "launch counts failed"; exit 1; }
tail -3 $OUT/launch_counts.txt
for f in bench full96 rl; do python3 -c "
import json; d=json.load(open('$OUT/$f.json')); print('$f', round(d['value'],1), d['unit'], round(d['ms_per_step'],4), 'ms/step')"; done
echo r03f-done
