#!/bin/bash
# the bench lines of the final build, each time-limited
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-lines}
mkdir -p $OUT
run() { name=$1; shift; timeout -k 10 400 python3 bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -3 $OUT/$name.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print('$name', round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],4), 'ms/step', 'kernel', round(r['kernel_ms'],4), 'frac', r['frac'], 'traffic', r['traffic'], 'valu', d.get('roofline_valu',{}).get('frac'), {k: v for k, v in d['status_counts'].items() if v and k != 'optimal'})"; }
run driver --gpus 1 --steps 20 --warmup 5
run full96 --steps 96 --warmup 4 --cpu-seconds 0
run rl --workload rl --steps 6 --warmup 1 --cpu-seconds 0
run rl_flat --workload rl --rl-price flat --steps 6 --warmup 1 --cpu-seconds 0
run shard2 --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 2
run shard4 --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 4
run shard8 --steps 96 --warmup 4 --cpu-seconds 0 --shard-of 8
run h24 --steps 96 --warmup 4 --cpu-seconds 0 --horizon-hours 6
run cfg1 --homes 1000 --steps 96 --warmup 4 --cpu-seconds 0 --horizon-hours 6 --month 1
run jan --steps 96 --warmup 4 --cpu-seconds 0 --month 1
run cfg3size --homes 100000 --steps 24 --warmup 2 --cpu-seconds 0 --horizon-hours 6
echo lines-done
