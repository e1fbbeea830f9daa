#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-trace96}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof96 -o trace -- python3 bench.py --steps 96 --warmup 4 --cpu-seconds 0 $EXTRA > $OUT/prof96.log 2>&1 || { echo "trace failed"; tail -5 $OUT/prof96.log; exit 1; }
python3 - <<PY
import csv
for r in list(csv.DictReader(open("$OUT/prof96/trace_kernel_stats.csv")))[:8]:
    print(r["Name"][:60], r["Calls"], round(float(r["TotalDurationNs"]) / 1e6, 2), "ms total", round(float(r["AverageNs"]) / 1e3, 1), "us avg", round(float(r["MaxNs"]) / 1e3, 1), "max")
PY
