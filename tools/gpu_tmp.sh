set -o pipefail
for c in q56 q72; do
DRAGG_LIB=$PWD/varlib/$c.so timeout -k 10 200 python tools/count_paths.py 10000 12 96 7 2>&1 | grep -v amdgpu.ids || exit 1
done
BENCH_ARGS="--steps 96" bash tools/gpu_bench_ab.sh c17 q56 q72 || exit 1
