#!/bin/bash
# session 1: exactness suite on the in-tree build, A/B bench, front statistics (NB_CAP 2048 build)
set -o pipefail
mkdir -p gpurun_out/s1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/s1/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/s1/pytest.log; exit 1; }
tail -1 gpurun_out/s1/pytest.log
for lib in head front128 head front128; do
  DRAGG_LIB=$PWD/varlib/$lib.so timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps 48 > gpurun_out/s1/bench_$lib.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/s1/bench_$lib.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/s1/bench_$lib.log | cut -c1-200)"
done
for a in "10000 12 7" "10000 12 7 rl" "10000 6 1" "10000 12 4"; do
  NB_CAP=2048 DRAGG_LIB=$PWD/varlib/stats.so timeout -k 10 200 python -u tools/front_stats.py $a > gpurun_out/s1/stats.log 2>&1 || { echo STATS_FAIL; tail -20 gpurun_out/s1/stats.log; exit 1; }
  cat gpurun_out/s1/stats.log
done
