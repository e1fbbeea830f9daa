set -o pipefail
mkdir -p gpurun_out/s11
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/s11/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/s11/pytest.log; exit 1; }
tail -1 gpurun_out/s11/pytest.log
timeout -k 10 200 python tools/count_paths.py 10000 12 96 7 2>&1 | grep -v amdgpu.ids || exit 1

timeout -k 10 200 python tools/count_paths.py 10000 12 16 7 rl 2>&1 | grep -v amdgpu.ids || exit 1
BENCH_ARGS="--steps 96 --homes 1250" bash tools/gpu_bench_ab.sh c14 c16 || exit 1
BENCH_ARGS="--workload rl --steps 8" bash tools/gpu_bench_ab.sh c14 c16 || exit 1
BENCH_ARGS="--steps 96" bash tools/gpu_bench_ab.sh c14 c16 || exit 1
