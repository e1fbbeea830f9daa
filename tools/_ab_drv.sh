#!/bin/bash
# A/B of $NEW against the in-tree library on the driver window (three rounds, alternating)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${T:-ab_drv}; mkdir -p $OUT
line() { name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $OUT/$name.out 2> $OUT/$name.err || { echo "$name failed"; tail -3 $OUT/$name.err; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('$OUT/$name.out') if l.startswith('{')][-1]; print('$name', round(d['ms_per_step'],4), 'ms/step kern', round(d['roofline']['kernel_ms'],4))"; }
for r in 1 2 3; do
  line drv_main$r --steps 20 --warmup 5 --cpu-seconds 0
  DRAGG_LIB=$NEW line drv_new$r --steps 20 --warmup 5 --cpu-seconds 0
done
echo done
