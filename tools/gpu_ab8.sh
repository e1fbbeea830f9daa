#!/bin/bash
# Round-6 A/B: (1) the cell kernel's launch bounds on the RL action (cur = 4 blocks per CU at 128 VGPRs with
# spills; cell_lb3 / cell_lb2: 3 / 2 blocks per CU without); (2) the RL phase split; (3) the side stream's
# priority (DRAGG_SIDE_PRIORITY 0 / -1) on the full day: the 8-way shard holding home 7519, and 10k homes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab8
mkdir -p $OUT
( while sleep 60; do echo "tick $(date +%T)" >> $OUT/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
TAG=ab8r ROUNDS=${ROUNDS:-2} ABARGS="--workload rl --steps 6 --warmup 1" bash tools/gpu_ab6.sh "$@" || exit 1
timeout -k 10 300 python3 -u tools/phase_breakdown.py --rl --homes 10000 --horizon-hours 12 --month 7 --steps 4 --out $OUT/phase_rl.json > $OUT/phase_rl.log 2>&1 || { tail -5 $OUT/phase_rl.log; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/phase_rl.json')); print(d['kernel_ms_mean'], d['phase_share'], d['phase_mean_cycles'])"
for r in 1 2; do
  for p in 0 -1; do
    for w in "shard8r7:--shard-of 8 --shard-rank 7" "full96:"; do
      name=${w%%:*}; args=${w#*:}
      [ "$name" = full96 ] && [ $r = 2 ] && continue
      DRAGG_SIDE_PRIORITY=$p timeout -k 10 300 python3 bench.py --steps 96 --warmup 4 --cpu-seconds 0 $args > $OUT/prio${p}_$name.$r.out 2> $OUT/prio${p}_$name.$r.err || { echo "prio $p $name failed"; tail -5 $OUT/prio${p}_$name.$r.err; exit 1; }
      grep '^{' $OUT/prio${p}_$name.$r.out | tail -1 > $OUT/prio${p}_$name.$r.json
      python3 -c "import json; d=json.load(open('$OUT/prio${p}_$name.$r.json')); print('prio', '$p', '$name', $r, round(d['ms_per_step'],4))"
    done
  done
done
echo ab8-done
