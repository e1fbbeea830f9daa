set -o pipefail
mkdir -p gpurun_out/s10
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/s10/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/s10/pytest.log; exit 1; }
tail -1 gpurun_out/s10/pytest.log
BENCH_ARGS="--steps 96" bash tools/gpu_bench_ab.sh h168p64 c14 || exit 1
