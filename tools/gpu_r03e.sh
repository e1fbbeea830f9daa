#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03e
mkdir -p $OUT
DRAGG_LIB=varlib/stprof.so timeout -k 10 300 python3 tools/step_prof.py --steps 96 > $OUT/step_prof.txt 2>&1 || { echo "step prof failed"; tail -5 $OUT/step_prof.txt; exit 1; }
tail -2 $OUT/step_prof.txt
timeout -k 10 300 python3 bench.py --steps 96 --warmup 0 --cpu-seconds 0 > $OUT/full96.json 2> $OUT/full96.err || { echo "full96 failed"; exit 1; }
DRAGG_NO_STEP_DP=1 timeout -k 10 300 python3 tools/rl_paths.py --steps 4 > $OUT/rl_paths_nostep.txt 2>&1 || { echo "rl paths failed"; exit 1; }
tail -1 $OUT/rl_paths_nostep.txt
timeout -k 10 300 python3 tools/rl_paths.py --steps 4 > $OUT/rl_paths.txt 2>&1 || { echo "rl paths failed"; exit 1; }
cat $OUT/rl_paths.txt
python3 -c "
import json; d=json.load(open('$OUT/full96.json')); print('full96', round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],4), 'ms/step')"
echo r03e-done
