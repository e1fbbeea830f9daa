set -o pipefail
BENCH_ARGS="--steps 96" bash tools/gpu_bench_ab.sh head c11 c11n128 c11n256 || exit 1
BENCH_ARGS="--steps 96 --homes 1250" bash tools/gpu_bench_ab.sh head c11 c8 || exit 1
