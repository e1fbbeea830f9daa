#!/bin/bash
# A/B of the in-tree library against $PREV on the 8-way straggler shard over the full day (lag mode),
# after the lag-mode bit-identity tests on the in-tree build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${T:-ab_side2}; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_overlap.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
line() { name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $OUT/$name.out 2> $OUT/$name.err || { echo "$name failed"; tail -3 $OUT/$name.err; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('$OUT/$name.out') if l.startswith('{')][-1]; print('$name', round(d['ms_per_step'],4), 'ms/step kern', round(d['roofline']['kernel_ms'],4))"; }
for r in 1 2 3; do
  DRAGG_LIB=$PREV line s7_prev$r --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 8 --shard-rank 7
  line s7_new$r --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 8 --shard-rank 7
done
echo done
