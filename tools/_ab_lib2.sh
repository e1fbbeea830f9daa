#!/bin/bash
# A/B of $NEW against $PREV on the 4-way and 8-way shard maxima over the driver's window (two rounds each)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${T:-ab_lib2}; mkdir -p $OUT
line() { name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $OUT/$name.out 2> $OUT/$name.err || { echo "$name failed"; tail -3 $OUT/$name.err; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('$OUT/$name.out') if l.startswith('{')][-1]; print('$name', round(d['ms_per_step'],4), 'ms/step kern', round(d['roofline']['kernel_ms'],4), (d.get('shard_emulation') or {}).get('max_over_shards'))"; }
for r in 1 2; do
  DRAGG_LIB=$PREV line sh4_prev$r --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 4 --shard-max
  DRAGG_LIB=$NEW line sh4_new$r --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 4 --shard-max
  DRAGG_LIB=$PREV line sh8_prev$r --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 8 --shard-max
  DRAGG_LIB=$NEW line sh8_new$r --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 8 --shard-max
done
echo done
