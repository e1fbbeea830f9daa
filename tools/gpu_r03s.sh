#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03s
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "tests failed"; tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
for ab in 1 0; do
  DRAGG_ASYNC_BOUND=$ab timeout -k 10 300 python3 bench.py --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 8 > $OUT/shard8_ab$ab.json 2> $OUT/e.err || { echo "shard8 failed"; tail -3 $OUT/e.err; exit 1; }
  DRAGG_ASYNC_BOUND=$ab timeout -k 10 300 python3 bench.py --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 4 > $OUT/shard4_ab$ab.json 2> $OUT/e.err || { echo "shard4 failed"; exit 1; }
done
timeout -k 10 300 python3 bench.py --steps 96 --warmup 4 --cpu-seconds 0 > $OUT/full96.json 2> $OUT/e.err || { echo "full96 failed"; exit 1; }
python3 - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r03s/*.json")):
    d = json.load(open(f))
    print(os.path.basename(f), round(d["value"] / 1e6, 3), "M/s", round(d["ms_per_step"], 4), "ms/step", {k: v for k, v in d["status_counts"].items() if v and k != "optimal"})
PY
