#!/bin/bash
# Round measurement session: smoke, GPU tests, the default bench line (with the CPU baseline),
# the other BASELINE configs and per-GPU loads.  Logs under gpurun_out/final/.
set -o pipefail
O=gpurun_out/final
mkdir -p $O
line() { tail -1 $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"], 4), d["config"]["workload"])'; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 $O/smoke.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || exit 1; line $O/bench.log
timeout -k 10 200 python -u bench.py --cpu-seconds 0 --homes 1000 --horizon-hours 6 --month 1 > $O/bench_cfg1.log 2>&1 || exit 1; line $O/bench_cfg1.log
timeout -k 10 200 python -u bench.py --cpu-seconds 0 --homes 10000 --horizon-hours 6 > $O/bench_h24.log 2>&1 || exit 1; line $O/bench_h24.log
timeout -k 10 200 python -u bench.py --cpu-seconds 0 --month 1 > $O/bench_jan.log 2>&1 || exit 1; line $O/bench_jan.log
timeout -k 10 300 python -u bench.py --workload rl --cpu-seconds 0 --steps 48 > $O/bench_rl.log 2>&1 || exit 1; line $O/bench_rl.log
timeout -k 10 300 python -u bench.py --homes 100000 --horizon-hours 6 --steps 24 --cpu-seconds 0 > $O/bench_100k.log 2>&1 || exit 1; line $O/bench_100k.log
for homes in 1250 2500 5000; do
    timeout -k 10 120 python -u bench.py --cpu-seconds 0 --homes $homes --steps 48 --warmup 2 > $O/load_h${homes}.log 2>&1 || exit 1; line $O/load_h${homes}.log
done
echo final-done
