#!/bin/bash
# threads-per-home sweep at the per-GPU load of the strong-scaling runs (10k homes / N GPUs)
set -o pipefail
mkdir -p gpurun_out/nt
for homes in 1250 2500 5000 10000; do
  for nt in 64 128 256; do
    DRAGG_DIRECT_THREADS=$nt timeout -k 10 120 python -u bench.py --cpu-seconds 0 --homes $homes --steps 24 --warmup 2 > gpurun_out/nt/h${homes}_nt${nt}.log 2>&1 || exit 1
  done
done
echo sweep-done
