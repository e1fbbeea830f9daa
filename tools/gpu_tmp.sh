set -o pipefail
mkdir -p gpurun_out/s8
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_proven.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/s8/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/s8/pytest.log; exit 1; }
tail -1 gpurun_out/s8/pytest.log
BENCH_ARGS="--steps 96" bash tools/gpu_bench_ab.sh c11 pa64 pa96 pa160 || exit 1
BENCH_ARGS="--steps 96 --homes 1250" bash tools/gpu_bench_ab.sh c11 pa64 pa96 pa160 || exit 1
