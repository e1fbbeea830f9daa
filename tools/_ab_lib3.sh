#!/bin/bash
# A/B of the in-tree library against $PREV: bit-identity (1,250 homes x 60 steps; 10k homes x 30 steps),
# then the driver window, the 8-way shard maxima and the RL line, alternating builds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${T:-ab_lib3}; mkdir -p $OUT
for spec in "1250 60" "10000 30"; do set -- $spec
  DRAGG_LIB=$PREV timeout -k 10 240 python3 tools/ab_equal.py --homes $1 --steps $2 --dump $OUT/prev.npz > $OUT/dump1.log 2>&1 || { echo dump1 failed; tail -3 $OUT/dump1.log; exit 1; }
  timeout -k 10 240 python3 tools/ab_equal.py --homes $1 --steps $2 --dump $OUT/new.npz > $OUT/dump2.log 2>&1 || { echo dump2 failed; tail -3 $OUT/dump2.log; exit 1; }
  echo "homes $1:"; python3 tools/ab_equal.py --compare $OUT/prev.npz $OUT/new.npz | tail -2
  rm -f $OUT/prev.npz $OUT/new.npz
done
line() { name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $OUT/$name.out 2> $OUT/$name.err || { echo "$name failed"; tail -3 $OUT/$name.err; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('$OUT/$name.out') if l.startswith('{')][-1]; print('$name', round(d['ms_per_step'],4), 'ms/step kern', round(d['roofline']['kernel_ms'],4), (d.get('shard_emulation') or {}).get('max_over_shards'))"; }
for r in 1 2; do
  DRAGG_LIB=$PREV line drv_prev$r --steps 20 --warmup 5 --cpu-seconds 0
  line drv_new$r --steps 20 --warmup 5 --cpu-seconds 0
done
DRAGG_LIB=$PREV line sh8_prev --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 8 --shard-max
line sh8_new --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 8 --shard-max
DRAGG_LIB=$PREV line rl_prev --workload rl --steps 6 --warmup 1 --cpu-seconds 0
line rl_new --workload rl --steps 6 --warmup 1 --cpu-seconds 0
echo done
