#!/bin/bash
# multi-wave mid / big launches + feasibility pre-pass: GPU suite, then A/B of waves per home
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03i
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
grep -E "ROUND_FAIL cases|narrow-set cases" $OUT/pytest_gpu.txt
for lib in cur m1b1 m1b4 m1b2; do
  L=""; [ $lib != cur ] && L=$PWD/varlib/$lib.so
  DRAGG_LIB=$L timeout -k 10 300 python3 bench.py --workload rl --steps 6 --warmup 1 --cpu-seconds 0 > $OUT/rl_$lib.json 2> $OUT/rl_$lib.err || { echo "rl $lib failed"; tail -3 $OUT/rl_$lib.err; exit 1; }
done
for lib in cur m1b1; do
  L=""; [ $lib != cur ] && L=$PWD/varlib/$lib.so
  DRAGG_LIB=$L timeout -k 10 300 python3 bench.py --steps 96 --warmup 4 --cpu-seconds 0 > $OUT/full96_$lib.json 2> $OUT/full96_$lib.err || { echo "full96 $lib failed"; exit 1; }
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/driver20.json 2> $OUT/driver20.err || { echo "driver failed"; exit 1; }
python3 - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r03i/*.json")):
    d = json.load(open(f))
    print(os.path.basename(f), round(d["value"] / 1e6, 3), "M/s", round(d["ms_per_step"], 4), "ms/step", {k: v for k, v in d["status_counts"].items() if v})
PY
echo r03i-done
