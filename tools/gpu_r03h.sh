#!/bin/bash
# kernel traces of the full day and of the varying-price RL line; launch counts per step
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03h
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof96 -o trace -- python3 bench.py --steps 96 --warmup 0 --cpu-seconds 0 > $OUT/prof96.log 2>&1 || { echo "trace failed"; tail -5 $OUT/prof96.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_rl -o trace -- python3 bench.py --workload rl --steps 6 --warmup 1 --cpu-seconds 0 > $OUT/prof_rl.log 2>&1 || { echo "rl trace failed"; exit 1; }
timeout -k 10 300 python3 tools/launch_counts.py --steps 96 > $OUT/counts_rbo.txt 2>&1 || { echo "counts failed"; exit 1; }
tail -1 $OUT/counts_rbo.txt
timeout -k 10 300 python3 tools/launch_counts.py --steps 6 --rl > $OUT/counts_rl.txt 2>&1 || { echo "counts rl failed"; exit 1; }
tail -1 $OUT/counts_rl.txt
python3 - <<'PY'
import csv
for f in ["prof96", "prof_rl"]:
    for r in list(csv.DictReader(open(f"gpurun_out/r03h/{f}/trace_kernel_stats.csv")))[:6]:
        print(f, r["Name"][:60], r["Calls"], round(float(r["TotalDurationNs"]) / 1e6, 2), "ms total", round(float(r["AverageNs"]) / 1e3, 1), "us avg", round(float(r["MaxNs"]) / 1e3, 1), "max")
PY
echo r03h-done
