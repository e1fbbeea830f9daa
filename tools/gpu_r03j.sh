#!/bin/bash
# RL path and 1,250-home shard: phase cycles per home, kernel traces
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03j
mkdir -p $OUT
timeout -k 10 200 python3 tools/phase_breakdown.py --homes 10000 --steps 4 --horizon-hours 12 --month 7 --rl --out $OUT/phase_rl.json > /dev/null 2> $OUT/phase_rl.err || { echo "phase rl failed"; tail -3 $OUT/phase_rl.err; exit 1; }
timeout -k 10 200 python3 tools/phase_breakdown.py --homes 10000 --world 8 --steps 48 --horizon-hours 12 --month 7 --out $OUT/phase_1250.json > /dev/null 2> $OUT/phase_1250.err || { echo "phase 1250 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_rl -o trace -- python3 bench.py --workload rl --steps 6 --warmup 1 --cpu-seconds 0 > $OUT/prof_rl.log 2>&1 || { echo "rl trace failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_s8 -o trace -- python3 bench.py --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 8 > $OUT/prof_s8.log 2>&1 || { echo "s8 trace failed"; exit 1; }
python3 - <<'PY'
import csv, json
for f in ["phase_rl", "phase_1250"]:
    d = json.load(open(f"gpurun_out/r03j/{f}.json"))
    print(f, "kernel ms mean", round(d["kernel_ms_mean"], 3), "phase mean cycles", {k: round(v) for k, v in d["phase_mean_cycles"].items() if v},
          "pct", d["home_total_cycles_pct"], "slowest", d["slowest_home_phase_cycles"])
for f in ["prof_rl", "prof_s8"]:
    for r in list(csv.DictReader(open(f"gpurun_out/r03j/{f}/trace_kernel_stats.csv")))[:6]:
        print(f, r["Name"][:60], r["Calls"], round(float(r["TotalDurationNs"]) / 1e6, 2), "ms total", round(float(r["AverageNs"]) / 1e3, 1), "us avg", round(float(r["MaxNs"]) / 1e3, 1), "max")
PY
echo r03j-done
