#!/bin/bash
# A/B of library variants on the RL line: tools/_rlab.sh (uses $LIBS: name=path ...)
set -o pipefail
OUT=gpurun_out/${T:-rlab}; mkdir -p $OUT
for spec in $LIBS; do
  name=${spec%%=*}; lib=${spec#*=}
  if [ "$lib" = main ]; then unset DRAGG_LIB; else export DRAGG_LIB=$lib; fi
  timeout -k 10 300 python3 bench.py --workload rl --steps 6 --warmup 1 --cpu-seconds 0 > $OUT/$name.out 2> $OUT/$name.err || { echo "$name failed"; tail -3 $OUT/$name.err; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('$OUT/$name.out') if l.startswith('{')][-1]; print('$name', round(d['ms_per_step'],3), 'ms/action')"
done
