set -o pipefail
mkdir -p gpurun_out/s9
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_proven.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/s9/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/s9/pytest.log; exit 1; }
tail -1 gpurun_out/s9/pytest.log
BENCH_ARGS="--steps 96" bash tools/gpu_bench_ab.sh c12 wm || exit 1
BENCH_ARGS="--workload rl --steps 8" bash tools/gpu_bench_ab.sh c12 wm || exit 1
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for p in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 240 rocprofv3 --pmc $p --output-format csv -d gpurun_out/s9/$p -o $p -- python3 bench.py --cpu-seconds 0 > gpurun_out/s9/$p.log 2>&1 || exit 1
done
