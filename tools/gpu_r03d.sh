#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03d
mkdir -p $OUT
DRAGG_LIB=varlib/stprof.so timeout -k 10 300 python3 tools/step_prof.py --steps 96 > $OUT/step_prof.txt 2>&1 || { echo "step prof failed"; tail -5 $OUT/step_prof.txt; exit 1; }
tail -4 $OUT/step_prof.txt
for r in 1 2; do
for lib in kf nokf; do
  DRAGG_LIB=$PWD/varlib/$lib.so timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/driver_$lib.json 2> $OUT/driver_$lib.err || { echo "driver $lib failed"; exit 1; }
  DRAGG_LIB=$PWD/varlib/$lib.so timeout -k 10 300 python3 bench.py --steps 40 --warmup 50 --cpu-seconds 0 > $OUT/late_$lib.json 2> $OUT/late_$lib.err || { echo "late $lib failed"; exit 1; }
  DRAGG_LIB=$PWD/varlib/$lib.so timeout -k 10 300 python3 bench.py --steps 96 --warmup 0 --cpu-seconds 0 --shard-of 8 > $OUT/shard8_$lib.json 2> $OUT/shard8_$lib.err || { echo "shard8 $lib failed"; exit 1; }
  python3 - $lib <<'PY'
import json, sys
lib = sys.argv[1]
for f in ["driver", "late", "shard8"]:
    d = json.load(open(f"gpurun_out/r03d/{f}_{lib}.json"))
    print(lib, f, round(d["value"] / 1e6, 3), "M/s", round(d["ms_per_step"], 4), "ms/step")
PY
done
done
echo r03d-done
