#!/bin/bash
# A/B of the lag mode's side-pass grids on the driver window and the full day
set -o pipefail
OUT=gpurun_out/${T:-ab_side}; mkdir -p $OUT
line() { name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $OUT/$name.out 2> $OUT/$name.err || { echo "$name failed"; tail -3 $OUT/$name.err; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('$OUT/$name.out') if l.startswith('{')][-1]; print('$name', round(d['ms_per_step'],4), 'ms/step kern', round(d['roofline']['kernel_ms'],4), 'lag', d.get('lag_mode'))"; }
line drv_serial --steps 20 --warmup 5 --cpu-seconds 0 --no-overlap
line drv_lag --steps 20 --warmup 5 --cpu-seconds 0
DRAGG_SIDE_GRID=16,16,16,2 line drv_lag16 --steps 20 --warmup 5 --cpu-seconds 0
DRAGG_SIDE_GRID=4,4,4,1 line drv_lag4 --steps 20 --warmup 5 --cpu-seconds 0
DRAGG_SIDE_GRID=16,16,16,2 line full_lag16 --steps 96 --warmup 4 --cpu-seconds 0
DRAGG_SIDE_GRID=4,4,4,1 line full_lag4 --steps 96 --warmup 4 --cpu-seconds 0
line drv_serial2 --steps 20 --warmup 5 --cpu-seconds 0 --no-overlap
echo done
