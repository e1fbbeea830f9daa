set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 300 python -u tools/dump_gpu_obj.py r01 round > gpurun_out/dump.log 2>&1 || { echo DUMP_FAIL; tail -30 gpurun_out/dump.log; exit 1; }
timeout -k 10 200 python -u bench.py --cpu-seconds 0 > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/smoke.log; tail -1 gpurun_out/bench.log
