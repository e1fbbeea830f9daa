"""Diagnostic: run the configs[3] community (tests/test_gpu_configs.py) step by step and report every
home whose p_grid_opt turns NaN (status, int_path, type).  Usage: python tools/nan_hunt.py [--steps K]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.test_gpu_configs import _community              # noqa: E402
from dragg_amd.aggregator import DeviceAggregator          # noqa: E402
from dragg_amd import _lib as L                            # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=120)
ap.add_argument("--homes", type=int, default=100000)
a = ap.parse_args()
homes, oat, ghi, tou = _community(a.homes, 6, 4, 672, 7, 41)
agg = DeviceAggregator(homes, oat, ghi, tou, 0, 672, reward_price=[0.0], int_mode="round", seed=41, keep_history=False)
b = agg.batch
found = 0
for t in range(a.steps):
    agg.run_iteration()
    torch.cuda.synchronize()
    pg = b.vals[L.V_P_GRID if hasattr(L, "V_P_GRID") else 0].cpu().numpy()
    bad = np.flatnonzero(~np.isfinite(pg))
    if len(bad):
        st = b.status.cpu().numpy(); ip = b.int_path.cpu().numpy() if b.int_path is not None else None
        for i in bad[:10]:
            print(f"t={t} home {i} type {homes[i]['type']} status {L.STATUS_NAMES[st[i]]} int_path {hex(int(ip[i])) if ip is not None else None} "
                  f"obj {float(b.obj[i])}", flush=True)
        found += len(bad)
        if found > 20:
            break
print(f"done: {found} NaN p_grid values in {t + 1} steps")
