#!/bin/bash
# Bench experimental library variants (varlib/NAME.so), then the iteration run of the in-tree
# library: tools/gpu_var.sh TAG NAME...
set -o pipefail
mkdir -p gpurun_out
TAG=$1; shift
for v in "$@"; do
  DRAGG_LIB=varlib/$v.so timeout -k 10 200 python -u bench.py --cpu-seconds 0 > gpurun_out/bench_var_$v.log 2>&1 || { echo VAR_FAIL $v; tail -20 gpurun_out/bench_var_$v.log; exit 1; }
  echo "variant $v: $(tail -1 gpurun_out/bench_var_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["status_counts"])')"
done
bash tools/gpu_iter.sh $TAG
