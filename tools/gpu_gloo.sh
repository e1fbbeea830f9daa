#!/bin/bash
# the multi-rank bench path rehearsed on one GPU: ranks share the device, gloo in place of RCCL
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/gloo
mkdir -p $OUT
for n in 2 4; do
  DRAGG_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 20 --warmup 5 > $OUT/gloo$n.json 2> $OUT/gloo$n.err || { echo "gloo $n failed"; tail -5 $OUT/gloo$n.err; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$OUT/gloo$n.json') if l.startswith('{')][-1]); print($n, 'ranks', round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],4), 'ms/step', d['n_gpus'], d['config']['parallelism'], {k: v for k, v in d['status_counts'].items() if v})"
done
