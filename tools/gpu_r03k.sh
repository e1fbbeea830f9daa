#!/bin/bash
# front-DP stage sections at 1,250 homes (per waves-per-home) and 10k homes; shard-8 step time per NW
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03k
mkdir -p $OUT
for nw in 1 2 4; do
  DRAGG_LIB=$PWD/varlib/sprof.so DRAGG_WAVES_PER_HOME=$nw timeout -k 10 200 python3 tools/stage_prof.py --world 8 --steps 48 --out $OUT/stage_1250_nw$nw.json > /dev/null 2> $OUT/s$nw.err || { echo "stage prof $nw failed"; tail -3 $OUT/s$nw.err; exit 1; }
  DRAGG_WAVES_PER_HOME=$nw timeout -k 10 300 python3 bench.py --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 8 > $OUT/shard8_nw$nw.json 2> $OUT/shard8_nw$nw.err || { echo "shard8 $nw failed"; exit 1; }
done
DRAGG_LIB=$PWD/varlib/sprof.so timeout -k 10 200 python3 tools/stage_prof.py --world 1 --steps 48 --out $OUT/stage_10k.json > /dev/null 2> $OUT/s10k.err || { echo "stage prof 10k failed"; exit 1; }
python3 - <<'PY'
import json
for f in ["stage_1250_nw1", "stage_1250_nw2", "stage_1250_nw4", "stage_10k"]:
    d = json.load(open(f"gpurun_out/r03k/{f}.json"))
    print(f, d["cycles_per_stage_mean"], "slow1%", d["cycles_per_stage_slowest1pct"], d["dp_cycles_per_solve_pct"])
for nw in (1, 2, 4):
    d = json.load(open(f"gpurun_out/r03k/shard8_nw{nw}.json"))
    print("shard8 nw", nw, round(d["ms_per_step"], 4), "ms/step", round(d["roofline"]["kernel_ms"], 4))
PY
echo r03k-done
