set -o pipefail
for c in h168p64 h160p48 h160p80 h128p32; do
DRAGG_LIB=$PWD/varlib/$c.so timeout -k 10 200 python tools/count_paths.py 10000 12 96 7 2>&1 | grep -v amdgpu.ids || exit 1
done
BENCH_ARGS="--steps 96" bash tools/gpu_bench_ab.sh h160p64 h168p64 h160p48 h160p80 h128p32 || exit 1
BENCH_ARGS="--steps 96 --homes 1250" bash tools/gpu_bench_ab.sh c13 h160p64 h160p48 || exit 1
