"""Diagnostic: int_path reasons of the RL-priced workload (bench's smooth price), per chain.
Usage: [DRAGG_NO_STEP_DP=1] python tools/rl_paths.py [--steps K]"""
import argparse
import collections
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
ap.add_argument("--steps", type=int, default=4)
a = ap.parse_args()
dt, hh = 4, 12
days = math.ceil((math.ceil(a.steps / dt) + hh + 2) / 24) + 1
homes = synthetic_homes(a.homes, seed=12, days=days, dt=dt, horizon_hours=hh)
oat, ghi, tou = synthetic_weather(days, dt, math.ceil(a.steps / dt), seed=3, month=7)
agg = DeviceAggregator(homes, oat, ghi, tou, 0, a.steps, reward_price=[0.0], seed=12, keep_history=False)
H = agg.batch.H
agg.batch.enable_phase_timing()
ph_sum, ph_n = np.zeros(L.NPHASE), 0
rng = np.random.default_rng(5)
cnt = collections.Counter()
for t in range(a.steps):
    agg.set_reward_price(rng.uniform(-0.02, 0.02) - 0.03 * np.cos(np.arange(H) / 3.0))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    agg.run_iteration()
    e1.record()
    torch.cuda.synchronize()
    p = agg.batch.int_path.cpu().numpy()
    st = agg.batch.status.cpu().numpy()
    for c in (0, 1):
        r = (p >> (4 + 4 * c)) & 0xF
        on = (p >> c) & 1
        for v, n in zip(*np.unique(r[on == 1], return_counts=True)):
            cnt[(c, int(v))] += int(n)
    cnt["steps_dp"] += int(((p & L.PATH_STEPS) != 0).sum())
    cyc = agg.batch.cycles.cpu().numpy().astype(float)
    ph_sum += cyc.sum(1)
    ph_n += cyc.shape[1]
    cnt["second"] += int(((p & L.PATH_SECOND) != 0).sum())
    approx = (p & 1) != 0
    for b, name in ((16, "cells"), (17, "beam_ub"), (18, "big")):
        cnt[name] += int(((p >> b) & 1).sum())
        cnt[name + "_approx"] += int((((p >> b) & 1) & approx).sum())
    print(f"t={t}: {e0.elapsed_time(e1):.1f} ms, statuses {np.bincount(st).tolist()}", flush=True)
print({str(k): v for k, v in cnt.items()})
print("mean shader cycles per home-step by phase:", {n: round(v / max(1, ph_n)) for n, v in zip(L.PHASES, ph_sum)})
