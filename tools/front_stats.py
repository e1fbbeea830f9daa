"""Diagnostic (variant build with DRAGG_FRONT_STATS): front sizes per stage and whether the LP
bound was on, read back from the workspace's S_PAD slots after one step.
DRAGG_LIB=varlib/stats.so python tools/front_stats.py N HOURS MONTH [rl] [--steps K] (statistics of step K-1)"""
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from dragg_amd.mpc import MPCBatch                                   # noqa: E402
from dragg_amd.community import synthetic_homes, synthetic_weather   # noqa: E402

N, HH, MONTH = (int(x) for x in sys.argv[1:4])
rl = "rl" in sys.argv[4:]
STEPS = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 1
dt = 4
days = 3 + (STEPS + 95) // 96
homes = synthetic_homes(N, seed=12, days=days, dt=dt, horizon_hours=HH)
oat, ghi, tou = synthetic_weather(days, dt, 2 + STEPS // dt, seed=3, month=MONTH)
H = HH * dt
rp = list(-0.03 * np.cos(np.arange(H) / 3.0)) if rl else [0.0]
b = MPCBatch(homes, oat, ghi, tou, 0, rp, int_mode="round", seed=12)
for t in range(STEPS):
    b.step(t)
torch.cuda.synchronize()
NBC = int(os.environ.get("NB_CAP", "336"))
par = ((N * H * NBC * 2 + 255) // 256) * 256
x = b.workspace.view(torch.uint8)[par:par + N * 8 * H * 8].view(torch.float64).view(N, H, 8)[:, :, 7].cpu().numpy()
st = b.status.cpu().numpy()
v = x.copy()
pr = np.floor(v[:, 0] / 1e8)
v[:, 0] -= pr * 1e8
nW = np.floor(v / 1e4)
nT = v - nW * 1e4
ok = st == 0
if "--json" in sys.argv:
    import json
    # children evaluated per stage = 7 x the previous stage's front (1 label before stage 0)
    prevT = np.concatenate([np.ones((N, 1)), nT[:, :-1]], axis=1)
    prevW = np.concatenate([np.ones((N, 1)), nW[:, :-1]], axis=1)
    kids = 7.0 * (prevT[ok].sum() + prevW[ok].sum())
    json.dump({"workload": f"{N} homes, H={H}, month {MONTH}, rl={rl}, one step (t = 0)",
               "front_mean_T": float(nT[ok].mean()), "front_mean_W": float(nW[ok].mean()),
               "front_max": float(max(nT[ok].max(), nW[ok].max())),
               "children_per_launch": float(kids) * N / max(1, int(ok.sum())),
               "note": "label relaxations (children) per launch, scaled from the optimal homes to all homes"},
              open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
print(f"N={N} H={H} rl={rl}: optimal {ok.sum()}; prune flag (1 T, 2 W, 3 both) counts {np.unique(pr[ok], return_counts=True)}")
for name, a in (("T", nT[ok]), ("W", nW[ok])):
    mx = a.max(axis=1)
    print(f"  {name}: front size mean {a.mean():.2f}, per-home max: median {np.median(mx):.0f}, p90 {np.percentile(mx, 90):.0f}, "
          f"p99 {np.percentile(mx, 99):.0f}, p99.9 {np.percentile(mx, 99.9):.0f}, max {mx.max():.0f}")
