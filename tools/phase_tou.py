"""Diagnostic: per-phase shader cycles of the hot launch's homes over the bench's driver window
(bench.py --steps 20 --warmup 5: steps 5..24 of the 10k-home July community, H = 48), by home type.
Usage: python tools/phase_tou.py [--steps 25] [--first 5]"""
import argparse
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench                                                          # noqa: E402
from dragg_amd import _lib as L                                      # noqa: E402
from dragg_amd.aggregator import DeviceAggregator                   # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=25)
ap.add_argument("--first", type=int, default=5)
a = ap.parse_args()
bargs = bench.parse(["--steps", str(a.steps - a.first), "--warmup", str(a.first)])
homes, oat, ghi, tou = bench.bench_community(bargs)
homes, _ = bench.reference_completable(homes, oat, ghi, tou, seed=12)
agg = DeviceAggregator(homes, oat, ghi, tou, 0, a.steps, reward_price=[0.0], seed=12, keep_history=False)
agg.batch.enable_phase_timing()
types = agg.batch.types_host
acc = {ty: np.zeros(L.NPHASE) for ty in range(4)}
n = {ty: 0 for ty in range(4)}
for t in range(a.steps):
    agg.run_iteration()
    torch.cuda.synchronize()
    if t < a.first:
        continue
    cyc = agg.batch.cycles.cpu().numpy().astype(float)
    st = agg.batch.status.cpu().numpy()
    for ty in range(4):
        m = (types == ty) & (st == 0)
        acc[ty] += cyc[:, m].sum(1)
        n[ty] += int(m.sum())
for ty, name in enumerate(["base", "pv_only", "battery_only", "pv_battery"]):
    print(name, n[ty], {p: round(v / max(1, n[ty])) for p, v in zip(L.PHASES, acc[ty])})
