"""Diagnostic: cycles per front-DP stage, by section, from the DRAGG_STAGE_PROF variant build
(tools/build_variant.sh sprof '1i #define DRAGG_STAGE_PROF').  Sections: 0 ranges / bound trigger,
1 pass 1 (bucket atomics), 2 scans, 3 pass 3 (dominance tests, appends), 4 reductions, clears,
W table + barrier.  Usage: DRAGG_LIB=varlib/sprof.so python tools/stage_prof.py --world 8 --steps 48"""
import argparse
import json
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dragg_amd import _lib as L                                      # noqa: E402
from dragg_amd.aggregator import DeviceAggregator                   # noqa: E402
from dragg_amd.community import synthetic_homes, synthetic_weather  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--homes", type=int, default=10000)
ap.add_argument("--world", type=int, default=1)
ap.add_argument("--steps", type=int, default=48)
ap.add_argument("--out", default=None)
ap.add_argument("--rank", type=int, default=0, help="the shard of --world to profile")
a = ap.parse_args()
dt, hh = 4, 12
days = math.ceil((math.ceil(a.steps / dt) + hh + 2) / 24) + 1
homes = synthetic_homes(a.homes, seed=12, days=days, dt=dt, horizon_hours=hh)
oat, ghi, tou = synthetic_weather(days, dt, math.ceil(a.steps / dt), seed=3, month=7)
agg = DeviceAggregator(homes, oat, ghi, tou, 0, a.steps, reward_price=[0.0], seed=12, keep_history=False,
                       rank=a.rank, world=a.world)
N, H = agg.batch.N, agg.batch.H
par = ((N * H * 336 * 2 + 255) // 256) * 256
acc = []
for t in range(a.steps):
    agg.run_iteration()
    torch.cuda.synchronize()
    x = agg.batch.workspace.view(torch.uint8)[par:par + N * 8 * H * 8].view(torch.float64).view(N, H, 8)[:, :9, 7]
    st = agg.batch.status.cpu().numpy()
    v = x.cpu().numpy().copy()
    acc.append(v[st == L.ST_OPTIMAL])
acc = np.concatenate(acc)                      # [solves][7]
acc[:, 0] += acc[:, 6]                         # (section 0 = ranges + the bound trigger; 6 = the trigger)
per_stage = acc[:, :5] / np.maximum(acc[:, 5:6], 1)
tot = acc[:, :5].sum(1)
slow = tot >= np.percentile(tot, 99)
names = ["ranges", "pass1", "scans", "pass3", "tail"]
res = {"homes": N, "world": a.world, "steps": a.steps,
       "cycles_per_stage_mean": dict(zip(names, per_stage.mean(0).round(1).tolist())),
       "cycles_per_stage_slowest1pct": dict(zip(names, per_stage[slow].mean(0).round(1).tolist())),
       "stages_per_solve_mean": float(acc[:, 5].mean()),
       "trigger_cycles_per_solve_mean": float(acc[:, 6].mean()),
       "trigger_cycles_per_solve_slowest1pct": float(acc[slow, 6].mean()),
       "trigger_share_of_dp": float(acc[:, 6].sum() / max(1.0, tot.sum())),
       "bound_backward_cycles_per_solve_mean": float(acc[:, 7].mean()),
       "bound_greedy_cycles_per_solve_mean": float(acc[:, 8].mean()),
       "bound_rows_per_solve_mean": None,
       "trigger_share_of_dp_slowest1pct": float(acc[slow, 6].sum() / max(1.0, tot[slow].sum())),
       "dp_cycles_per_solve_pct": {str(q): float(np.percentile(tot, q)) for q in (50, 90, 99, 100)},
       "slowest_solve": {"sections": dict(zip(names, acc[int(np.argmax(tot)), :5].round(0).tolist())),
                         "stages": float(acc[int(np.argmax(tot)), 5]),
                         "trigger": float(acc[int(np.argmax(tot)), 6]),
                         "bound_backward": float(acc[int(np.argmax(tot)), 7]),
                         "bound_greedy": float(acc[int(np.argmax(tot)), 8])}}
print(json.dumps(res, indent=1))
if a.out:
    json.dump(res, open(a.out, "w"), indent=1)
