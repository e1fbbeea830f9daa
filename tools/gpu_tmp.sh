set -o pipefail
for c in nb128 nb192; do
DRAGG_LIB=$PWD/varlib/$c.so timeout -k 10 200 python tools/count_paths.py 10000 12 16 7 rl 2>&1 | grep -v amdgpu.ids || exit 1
done
BENCH_ARGS="--workload rl --steps 16" bash tools/gpu_bench_ab.sh c17 nb128 nb192 || exit 1
