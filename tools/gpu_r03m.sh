#!/bin/bash
# GPU suite + the bench lines of the current build (full day, driver window, 8-way shard, RL)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r03m}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
fi
for lib in cur $(cd varlib 2>/dev/null && ls *.so 2>/dev/null | sed 's/\.so$//'); do
  L=""; [ $lib != cur ] && L=$PWD/varlib/$lib.so
  DRAGG_LIB=$L timeout -k 10 300 python3 bench.py --steps 96 --warmup 4 --cpu-seconds 0 > $OUT/full96_$lib.json 2> $OUT/e1.err || { echo "full96 failed"; tail -3 $OUT/e1.err; exit 1; }
  DRAGG_LIB=$L timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/driver20_$lib.json 2> $OUT/e2.err || { echo "driver failed"; exit 1; }
  DRAGG_LIB=$L timeout -k 10 300 python3 bench.py --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 8 > $OUT/shard8_$lib.json 2> $OUT/e3.err || { echo "shard8 failed"; exit 1; }
  DRAGG_LIB=$L timeout -k 10 300 python3 bench.py --workload rl --steps 6 --warmup 1 --cpu-seconds 0 > $OUT/rl_$lib.json 2> $OUT/e4.err || { echo "rl failed"; exit 1; }
done
python3 - <<'PY'
import json, glob, os
out = os.environ.get("TAG", "r03m")
for f in sorted(glob.glob(f"gpurun_out/{out}/*.json")):
    d = json.load(open(f))
    print(os.path.basename(f), round(d["value"] / 1e6, 3), "M/s", round(d["ms_per_step"], 4), "ms/step", {k: v for k, v in d["status_counts"].items() if v and k != "optimal"})
PY
echo done
