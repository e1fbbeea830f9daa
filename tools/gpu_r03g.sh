#!/bin/bash
# round-3 re-entry: the GPU suite on the current build, the driver's bench command, the full day,
# the varying-price RL line and the 8-way shard load
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03g
mkdir -p $OUT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -2 $OUT/pytest_gpu.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/driver20.json 2> $OUT/driver20.err || { echo "bench failed"; tail -5 $OUT/driver20.err; exit 1; }
timeout -k 10 300 python3 bench.py --steps 96 --warmup 0 --cpu-seconds 0 > $OUT/full96.json 2> $OUT/full96.err || { echo "full96 failed"; exit 1; }
timeout -k 10 300 python3 bench.py --workload rl --steps 6 --warmup 1 --cpu-seconds 0 > $OUT/rl_smooth.json 2> $OUT/rl_smooth.err || { echo "rl failed"; exit 1; }
timeout -k 10 300 python3 bench.py --steps 96 --warmup 0 --cpu-seconds 0 --shard-of 8 > $OUT/shard8.json 2> $OUT/shard8.err || { echo "shard8 failed"; exit 1; }
python3 - <<'PY'
import json
for f in ["driver20", "full96", "rl_smooth", "shard8"]:
    d = json.load(open(f"gpurun_out/r03g/{f}.json"))
    print(f, round(d["value"] / 1e6, 3), "M/s", round(d["ms_per_step"], 4), "ms/step", d["status_counts"], d["occupancy"]["hot"])
PY
echo r03g-done
