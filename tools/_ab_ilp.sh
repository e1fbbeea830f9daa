#!/bin/bash
# A/B of the hot launch's chunks per front-DP pass (DRAGG_HOT_ILP): bit-identity at 1,250 homes over 60
# steps, then the 8-way shard maxima and the driver window with one and two chunks
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${T:-ab_ilp}; mkdir -p $OUT
DRAGG_HOT_ILP=1 timeout -k 10 240 python3 tools/ab_equal.py --homes 1250 --steps 60 --dump $OUT/ilp1.npz > $OUT/dump1.log 2>&1 || { echo dump1 failed; tail -3 $OUT/dump1.log; exit 1; }
DRAGG_HOT_ILP=2 timeout -k 10 240 python3 tools/ab_equal.py --homes 1250 --steps 60 --dump $OUT/ilp2.npz > $OUT/dump2.log 2>&1 || { echo dump2 failed; tail -3 $OUT/dump2.log; exit 1; }
python3 tools/ab_equal.py --compare $OUT/ilp1.npz $OUT/ilp2.npz | tail -3
rm -f $OUT/ilp1.npz $OUT/ilp2.npz
line() { name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $OUT/$name.out 2> $OUT/$name.err || { echo "$name failed"; tail -3 $OUT/$name.err; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('$OUT/$name.out') if l.startswith('{')][-1]; print('$name', round(d['ms_per_step'],4), 'ms/step kern', round(d['roofline']['kernel_ms'],4), (d.get('shard_emulation') or {}).get('max_over_shards'))"; }
DRAGG_HOT_ILP=1 line sh8_ilp1 --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 8 --shard-max
DRAGG_HOT_ILP=2 line sh8_ilp2 --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 8 --shard-max
DRAGG_HOT_ILP=1 line sh4_ilp1 --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 4 --shard-max
DRAGG_HOT_ILP=2 line sh4_ilp2 --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 4 --shard-max
DRAGG_HOT_ILP=2 line drv_ilp2 --steps 20 --warmup 5 --cpu-seconds 0
line drv_auto --steps 20 --warmup 5 --cpu-seconds 0
echo done
