#!/bin/bash
# round-3 session A: measurement of the driver's command + diagnostics (each step time-limited)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_measure.sh r03a || exit 1
OUT=gpurun_out/r03a
timeout -k 10 400 python3 tools/dump_cases.py $OUT/cases.json > $OUT/dump_cases.log 2>&1 || { echo "dump failed"; tail -5 $OUT/dump_cases.log; exit 1; }
tail -3 $OUT/dump_cases.log
for w in 8 4 2; do
  timeout -k 10 300 python3 bench.py --steps 96 --warmup 0 --cpu-seconds 0 --shard-of $w > $OUT/shard$w.json 2> $OUT/shard$w.err || { echo "shard $w failed"; exit 1; }
done
timeout -k 10 300 python3 bench.py --steps 96 --warmup 0 --cpu-seconds 0 > $OUT/full96.json 2> $OUT/full96.err || { echo "full96 failed"; exit 1; }
timeout -k 10 300 python3 bench.py --workload rl --steps 6 --warmup 1 --cpu-seconds 0 > $OUT/rl_smooth.json 2> $OUT/rl_smooth.err || { echo "rl failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_rl -o trace -- python3 bench.py --workload rl --steps 6 --warmup 1 --cpu-seconds 0 > $OUT/prof_rl.log 2>&1 || { echo "rl trace failed"; exit 1; }
timeout -k 10 200 python3 tools/phase_breakdown.py --homes 10000 --world 8 --steps 48 --horizon-hours 12 --month 7 --out $OUT/phase_1250.json > /dev/null 2>&1 || { echo "phase 1250 failed"; exit 1; }
timeout -k 10 200 python3 tools/phase_breakdown.py --homes 10000 --world 1 --steps 48 --horizon-hours 12 --month 7 --out $OUT/phase_10k.json > /dev/null 2>&1 || { echo "phase 10k failed"; exit 1; }
echo session-done
