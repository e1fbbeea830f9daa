#!/bin/bash
# Per-GPU load of the strong-scaling runs (10k homes over N = 8, 4, 2, 1 GPUs: a strided
# shard has the community's type mix, so it is the same workload at 10k/N homes).
set -o pipefail
mkdir -p gpurun_out/load
for homes in 1250 2500 5000 10000; do
    timeout -k 10 120 python -u bench.py --cpu-seconds 0 --homes $homes --steps 48 --warmup 2 > gpurun_out/load/h${homes}.log 2>&1 || exit 1
    echo "$homes $(tail -1 gpurun_out/load/h${homes}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"], 4), round(d["value"]))')"
done
echo sweep-done
