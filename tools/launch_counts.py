"""Diagnostic: per step, how many homes each later launch took (the lists in the workspace):
hot -> mid (deferred), mid -> big (past 384 labels), any -> step-function DP.
Usage: python tools/launch_counts.py [--rl] [--steps K] [--homes N]"""
import argparse
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dragg_amd.aggregator import DeviceAggregator                   # noqa: E402
from dragg_amd.community import synthetic_homes, synthetic_weather  # noqa: E402


def offsets(N, H):
    """mpc_kernel.hip's workspace layout (par_region_bytes ... mid_list_offset)."""
    r = lambda x: (x + 255) // 256 * 256  # noqa: E731
    par = r(N * H * 336 * 2)
    defer = par + N * 8 * H * 8
    w_off = r(defer + (N + 2) * 4)
    big = r(w_off + N * (H + 1) * 64 * 16)
    nl = r(big + 512 * H * 2048 * 2)
    slot = (2 * (H + 1) * 16384 + 2 * 16 * 16385) * 8 + (16 + 16 * 15) * 16385 * 4
    nr = r(nl + (N + 2) * 4)
    ml = r(nr + 8 * slot)
    return defer, ml, nl


ap = argparse.ArgumentParser()
ap.add_argument("--homes", type=int, default=10000)
ap.add_argument("--steps", type=int, default=24)
ap.add_argument("--rl", action="store_true")
a = ap.parse_args()
dt, hh = 4, 12
days = math.ceil((math.ceil(a.steps / dt) + hh + 2) / 24) + 1
homes = synthetic_homes(a.homes, seed=12, days=days, dt=dt, horizon_hours=hh)
oat, ghi, tou = synthetic_weather(days, dt, math.ceil(a.steps / dt), seed=3, month=7)
agg = DeviceAggregator(homes, oat, ghi, tou, 0, a.steps, reward_price=[0.0], seed=12, keep_history=False)
N, H = agg.batch.N, agg.batch.H
offs = offsets(N, H)
rng = np.random.default_rng(5)
tot = np.zeros(3, int)
for t in range(a.steps):
    if a.rl:
        agg.set_reward_price(rng.uniform(-0.02, 0.02) - 0.03 * np.cos(np.arange(H) / 3.0))
    agg.run_iteration()
    torch.cuda.synchronize()
    ws = agg.batch.workspace.view(torch.uint8)
    c = [int(ws[o + 4 * N:o + 4 * N + 4].view(torch.int32).item()) for o in offs]
    tot += c
    print(f"t={t}: deferred {c[0]}, to big {c[1]}, to step DP {c[2]}", flush=True)
print(f"total over {a.steps} steps: deferred {tot[0]}, to big {tot[1]}, to step DP {tot[2]}")
