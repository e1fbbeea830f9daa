#!/bin/bash
# A/B of RL-path variants (bench --workload rl, smooth price): varlib/*.so vs the in-tree build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-rlab}
mkdir -p $OUT
for lib in cur $(cd varlib && ls *.so | sed 's/\.so$//'); do
  L=""; [ $lib != cur ] && L=$PWD/varlib/$lib.so
  DRAGG_LIB=$L timeout -k 10 300 python3 bench.py --workload rl --steps 6 --warmup 1 --cpu-seconds 0 > $OUT/rl_$lib.json 2> $OUT/rl_$lib.err || { echo "rl $lib failed"; tail -3 $OUT/rl_$lib.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/rl_$lib.json')); print('$lib', round(d['ms_per_step'],2), 'ms/action', {k: v for k, v in d['status_counts'].items() if v})"
done
