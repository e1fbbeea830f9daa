"""Diagnostic: section cycles of the exact step-function DP (DRAGG_STEP_PROF variant) on every home
that took it in the bench workload: (1a) ranks, (1b) merge, (2-3) interval values, (4) compaction,
-, recovery; breakpoints summed and max over the stages.  Usage:
DRAGG_LIB=varlib/stprof.so python tools/step_prof.py [--exact] [--steps K]"""
import argparse
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
ap.add_argument("--steps", type=int, default=96)
ap.add_argument("--exact", action="store_true", help="DRAGG_FLAG_EXACT: every narrow chain takes the step DP")
a = ap.parse_args()
dt, hh = 4, 12
days = math.ceil((math.ceil(a.steps / dt) + hh + 2) / 24) + 1
homes = synthetic_homes(a.homes, seed=12, days=days, dt=dt, horizon_hours=hh)
oat, ghi, tou = synthetic_weather(days, dt, math.ceil(a.steps / dt), seed=3, month=7)
agg = DeviceAggregator(homes, oat, ghi, tou, 0, a.steps, reward_price=[0.0], seed=12, keep_history=False,
                       exact=a.exact)
N, H = agg.batch.N, agg.batch.H
par = ((N * H * 336 * 2 + 255) // 256) * 256
rows = []
for t in range(a.steps):
    ws = agg.batch.workspace.view(torch.uint8)[par:par + N * 8 * H * 8].view(torch.float64).view(N, H, 8)
    ws[:, 10:18, 7] = 0.0
    agg.run_iteration()
    torch.cuda.synchronize()
    path = agg.batch.int_path.cpu().numpy()
    idx = np.flatnonzero(path & L.PATH_STEPS)
    if len(idx):
        v = ws[idx][:, 10:18, 7].cpu().numpy()
        for j, i in enumerate(idx):
            rows.append([t, int(i)] + v[j].tolist())
            print(f"t={t} home {i}: cycles (1a) {v[j,0]:.3g} (1b) {v[j,1]:.3g} (2-3) {v[j,2]:.3g} (4) {v[j,3]:.3g} "
                  f"rec {v[j,5]:.3g}; sum np {v[j,6]:.0f}, max np {v[j,7]:.0f}", flush=True)
r = np.array(rows)
if len(r):
    print("mean cycles per home:", r[:, 2:8].mean(0).round(0).tolist(), "sum np mean", r[:, 8].mean(), "max np", r[:, 9].max())
