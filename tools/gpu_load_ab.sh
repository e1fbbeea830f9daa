#!/bin/bash
# Per-GPU load sweep (the strong-scaling shard sizes) for alternative builds under explib/.
# Usage: bash tools/gpu_load_ab.sh libA.so libB.so ...
set -o pipefail
mkdir -p gpurun_out/load
for homes in ${LOAD_HOMES:-1250 2500 10000}; do
    for lib in "$@"; do
        n=$(basename $lib .so)
        DRAGG_LIB=$PWD/explib/$lib timeout -k 10 120 python -u bench.py --cpu-seconds 0 --homes $homes --steps 48 --warmup 2 > gpurun_out/load/${n}_h${homes}.log 2>&1 || exit 1
        echo "$n $homes $(tail -1 gpurun_out/load/${n}_h${homes}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"], 4), round(d["value"]))')"
    done
done
echo sweep-done
