#!/bin/bash
# A/B of the in-tree library against abl/prev.so (the previous build): bit-identity of a 1,250-home
# closed loop (60 steps), then the 8-way shard maxima over the driver's window and the driver window
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${T:-ab_lib}; mkdir -p $OUT
DRAGG_LIB=${PREV:-abl/prev.so} timeout -k 10 240 python3 tools/ab_equal.py --homes 1250 --steps 60 --dump $OUT/prev.npz > $OUT/dump1.log 2>&1 || { echo dump1 failed; tail -3 $OUT/dump1.log; exit 1; }
DRAGG_LIB=${NEW:-} timeout -k 10 240 python3 tools/ab_equal.py --homes 1250 --steps 60 --dump $OUT/new.npz > $OUT/dump2.log 2>&1 || { echo dump2 failed; tail -3 $OUT/dump2.log; exit 1; }
python3 tools/ab_equal.py --compare $OUT/prev.npz $OUT/new.npz | tail -3
rm -f $OUT/prev.npz $OUT/new.npz
line() { name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $OUT/$name.out 2> $OUT/$name.err || { echo "$name failed"; tail -3 $OUT/$name.err; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('$OUT/$name.out') if l.startswith('{')][-1]; print('$name', round(d['ms_per_step'],4), 'ms/step kern', round(d['roofline']['kernel_ms'],4), (d.get('shard_emulation') or {}).get('max_over_shards'))"; }
DRAGG_LIB=${PREV:-abl/prev.so} line sh8_prev --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 8 --shard-max
DRAGG_LIB=${NEW:-} line sh8_new --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 8 --shard-max
DRAGG_LIB=${PREV:-abl/prev.so} line sh8_prev2 --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 8 --shard-max
DRAGG_LIB=${NEW:-} line sh8_new2 --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 8 --shard-max
DRAGG_LIB=${PREV:-abl/prev.so} line cfg1_prev --homes 1000 --horizon-hours 6 --month 1 --steps 96 --warmup 4 --cpu-seconds 0
DRAGG_LIB=${NEW:-} line cfg1_new --homes 1000 --horizon-hours 6 --month 1 --steps 96 --warmup 4 --cpu-seconds 0
echo done
