set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 200 python -u tools/phase_breakdown.py --out gpurun_out/phase_jan_h24_direct.json > gpurun_out/phase1.log 2>&1
timeout -k 10 200 python -u tools/phase_breakdown.py --homes 10000 --horizon-hours 12 --month 7 --steps 6 --out gpurun_out/phase_jul_h48_direct.json > gpurun_out/phase2.log 2>&1
for nt in 64 128; do DRAGG_DIRECT_THREADS=$nt timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps 24 --homes 10000 > gpurun_out/bench_nt$nt.log 2>&1 || exit 1; done
timeout -k 10 300 python -u bench.py --cpu-seconds 0 > gpurun_out/bench.log 2>&1
