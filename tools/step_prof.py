"""Diagnostic: the exact step-function DP (DM_NARROW) on every home-step that took it in the bench
workload, from the DRAGG_STEP_PROF variant (tools/build_variant.sh stprof '1i #define DRAGG_STEP_PROF'):
shader cycles of the feasibility pass, lp_domains, the cut full pass (backward) and the recoveries;
breakpoints summed / max over the stages, stages past the LDS staging (np > BS_CAP: +1, Mc > CL_CAP:
+1000), cut stages (x100) / uncut retries (+1) / capacity fallbacks (+10), the bound.
Usage: DRAGG_LIB=varlib/stprof.so python tools/step_prof.py [--steps K]"""
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
a = ap.parse_args()
dt, hh = 4, 12
days = math.ceil((math.ceil(a.steps / dt) + hh + 2) / 24) + 1
homes = synthetic_homes(a.homes, seed=12, days=days, dt=dt, horizon_hours=hh)
oat, ghi, tou = synthetic_weather(days, dt, math.ceil(a.steps / dt), seed=3, month=7)
agg = DeviceAggregator(homes, oat, ghi, tou, 0, a.steps, reward_price=[0.0], seed=12, keep_history=False)
N, H = agg.batch.N, agg.batch.H
par = ((N * H * 336 * 2 + 255) // 256) * 256
rows = []
names = ["feas", "lpdom", "cutpass", "recov", "sum_np", "max_np", "global", "flags", "sum_Mc", "ub_ext", "ub", "ranges", "-", "compact", "vstage", "merge", "values"]
for t in range(a.steps):
    ws = agg.batch.workspace.view(torch.uint8)[par:par + N * 8 * H * 8].view(torch.float64).view(N, H, 8)
    ws[:, 10:27, 7] = 0.0
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    agg.run_iteration()
    t1.record()
    torch.cuda.synchronize()
    path = agg.batch.int_path.cpu().numpy()
    idx = np.flatnonzero(path & L.PATH_STEPS)
    if len(idx):
        v = ws[idx][:, 10:27, 7].cpu().numpy()
        for j, i in enumerate(idx):
            rows.append([t, int(i)] + v[j].tolist())
            print(f"t={t} home {i} step {t0.elapsed_time(t1):.3f} ms: " +
                  ", ".join(f"{n} {x:.4g}" for n, x in zip(names, v[j])), flush=True)
r = np.array(rows)
if len(r):
    print("mean per home-step:", dict(zip(names, r[:, 2:].mean(0).round(1).tolist())))
