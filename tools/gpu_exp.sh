#!/bin/bash
# Kernel experiments: phase breakdown + bench for each alternative library build under explib/
# (DRAGG_LIB selects it).  Usage: bash tools/gpu_exp.sh lib1.so lib2.so ...
set -o pipefail
mkdir -p gpurun_out/exp
for lib in "$@"; do
    n=$(basename $lib .so)
    DRAGG_LIB=$PWD/explib/$lib timeout -k 10 200 python -u tools/phase_breakdown.py --homes 10000 --horizon-hours 12 --month 7 --steps 6 --out gpurun_out/exp/phase_$n.json > gpurun_out/exp/phase_$n.log 2>&1 || { echo "phase $n failed"; tail -20 gpurun_out/exp/phase_$n.log; exit 1; }
    DRAGG_LIB=$PWD/explib/$lib timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps 48 > gpurun_out/exp/bench_$n.log 2>&1 || { echo "bench $n failed"; tail -20 gpurun_out/exp/bench_$n.log; exit 1; }
    echo "$n $(tail -1 gpurun_out/exp/bench_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["status_counts"])')"
done
echo exp-done
