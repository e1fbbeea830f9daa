set -o pipefail
mkdir -p gpurun_out/s15
timeout -k 10 200 python -u bench.py --cpu-seconds 0 --homes 1000 --horizon-hours 6 --month 1 > gpurun_out/s15/cfg1.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --cpu-seconds 0 --homes 10000 --horizon-hours 6 > gpurun_out/s15/h24.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --homes 100000 --horizon-hours 6 --steps 24 --cpu-seconds 0 > gpurun_out/s15/100k.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps 48 > gpurun_out/s15/bench.log 2>&1 || exit 1
for f in cfg1 h24 100k bench; do tail -1 gpurun_out/s15/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"], d["status_counts"], d["community"]["battery_home_swaps"])'; done
