#!/bin/bash
# Bit-for-bit A/B of two library builds under explib/ on two workloads.  Usage: gpu_ab.sh libA.so libB.so
set -o pipefail
mkdir -p gpurun_out/ab
WL=${AB_WORKLOADS:-"--month 7|--month 4 --horizon-hours 6 --homes 4000"}
IFS='|' read -ra WS <<< "$WL"
for w in "${WS[@]}"; do
    tag=$(echo $w | tr -d ' -')
    for lib in $1 $2; do
        DRAGG_LIB=$PWD/explib/$lib timeout -k 10 200 python -u tools/ab_equal.py --dump gpurun_out/ab/${lib%.so}_$tag.npz $w > gpurun_out/ab/${lib%.so}_$tag.log 2>&1 || { tail -5 gpurun_out/ab/${lib%.so}_$tag.log; exit 1; }
    done
    python tools/ab_equal.py --compare gpurun_out/ab/${1%.so}_$tag.npz gpurun_out/ab/${2%.so}_$tag.npz | tail -4
    rm -f gpurun_out/ab/*.npz
done
