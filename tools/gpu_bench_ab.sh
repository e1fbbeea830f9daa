#!/bin/bash
# Bench A/B of library builds under varlib/ (DRAGG_LIB), two rounds each.  Usage: gpu_bench_ab.sh a b c ...
# Extra bench arguments via BENCH_ARGS.
set -o pipefail
mkdir -p gpurun_out/ab
for r in 1 2; do
  for lib in "$@"; do
    DRAGG_LIB=$PWD/varlib/$lib.so timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps 48 $BENCH_ARGS > gpurun_out/ab/bench_$lib.log 2>&1 || { echo BENCH_FAIL $lib; tail -20 gpurun_out/ab/bench_$lib.log; exit 1; }
    echo "$lib $(tail -1 gpurun_out/ab/bench_$lib.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"], 4), d["status_counts"])')"
  done
done
