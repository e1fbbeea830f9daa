"""Count, per step, the homes whose integer solve left the exact front DP (int_path != 0):
front overflow, a feasible set narrower than one duty step, or mixed-sign duty prices.
python tools/count_paths.py N HOURS STEPS MONTH [rl]"""
import math
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from dragg_amd.aggregator import DeviceAggregator          # noqa: E402
from dragg_amd.community import synthetic_homes, synthetic_weather   # noqa: E402

N, HH, STEPS, MONTH = (int(x) for x in sys.argv[1:5])
rl = len(sys.argv) > 5
dt = 4
sim_hours = math.ceil(STEPS / dt)
days = math.ceil((sim_hours + HH + 2) / 24) + 1
homes = synthetic_homes(N, seed=12, days=days, dt=dt, horizon_hours=HH)
oat, ghi, tou = synthetic_weather(days, dt, sim_hours, seed=3, month=MONTH)
H = HH * dt
rp = list(-0.03 * np.cos(np.arange(H) / 3.0)) if rl else [0.0]
agg = DeviceAggregator(homes, oat, ghi, tou, 0, STEPS, reward_price=rp, seed=12, keep_history=False)
tot = {}
per = []
for t in range(STEPS):
    agg.run_iteration()
    p = agg.batch.int_path.cpu().numpy()
    st = agg.batch.status.cpu().numpy()
    per.append(int((p != 0).sum()))
    for v in np.unique(p):
        tot[int(v)] = tot.get(int(v), 0) + int((p == v).sum())
print(f"N={N} H={H} steps={STEPS} month={MONTH} rl={rl}: int_path totals {tot}; homes off the exact path per step: "
      f"max {max(per)}, mean {np.mean(per):.2f}, steps with any {sum(1 for x in per if x)}")
