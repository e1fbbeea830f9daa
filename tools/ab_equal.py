#!/usr/bin/env python3
"""Bit-for-bit comparison of two builds of the library (kernel changes meant to be exact).

`python tools/ab_equal.py --dump out.npz` runs a closed loop of the bench workload with the
library DRAGG_LIB selects and saves every step's hash arrays, statuses and objectives;
`python tools/ab_equal.py --compare a.npz b.npz` checks that two dumps are identical."""
import argparse
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dump(a):
    import numpy as np
    import torch
    from dragg_amd.aggregator import DeviceAggregator
    from dragg_amd.community import synthetic_homes, synthetic_weather
    sim_hours = math.ceil(a.steps / a.dt)
    days = math.ceil((sim_hours + a.horizon_hours + 2) / 24) + 1
    homes = synthetic_homes(a.homes, seed=12, days=days, dt=a.dt, horizon_hours=a.horizon_hours)
    oat, ghi, tou = synthetic_weather(days, a.dt, sim_hours, seed=3, month=a.month)
    agg = DeviceAggregator(homes, oat, ghi, tou, 0, a.steps, reward_price=[0.0], int_mode="round", seed=12)
    out = {}
    for t in range(a.steps):
        agg.run_iteration()
        torch.cuda.synchronize()
        if t < a.first:
            continue
        out[f"vals{t}"] = agg.batch.vals.cpu().numpy()
        out[f"fc{t}"] = agg.batch.fc.cpu().numpy()
        out[f"st{t}"] = agg.batch.status.cpu().numpy()
        out[f"obj{t}"] = agg.batch.obj.cpu().numpy()
    np.savez_compressed(a.dump, **out)
    print("dumped", a.dump)


def compare(p, q):
    import numpy as np
    A, B = np.load(p), np.load(q)
    bad = 0
    for k in A.files:
        x, y = A[k], B[k]
        same = np.array_equal(x.view(np.uint64) if x.dtype == np.float64 else x,
                              y.view(np.uint64) if y.dtype == np.float64 else y)
        if not same:
            bad += 1
            d = np.argwhere((x != y) & ~(np.isnan(x) & np.isnan(y))) if x.dtype == np.float64 else np.argwhere(x != y)
            print(f"{k}: {len(d)} entries differ, first {d[:3].tolist()}")
            if k.startswith("obj"):               # approximation changes: objective shift of b vs a
                t = k[3:]
                ok = (A["st" + t] == 0) & (B["st" + t] == 0)
                g = (y[ok] - x[ok]) / np.maximum(1.0, np.abs(x[ok]))
                print(f"  {k}: (b - a)/max(1,|a|) over {ok.sum()} optimal: mean {g.mean():.2e} "
                      f"max {g.max():.2e} min {g.min():.2e}")
    print("IDENTICAL" if bad == 0 else f"DIFFERENT in {bad} arrays")
    return bad == 0


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--dump")
    ap.add_argument("--compare", nargs=2)
    ap.add_argument("--homes", type=int, default=10000)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--horizon-hours", type=int, default=12)
    ap.add_argument("--month", type=int, default=7)
    ap.add_argument("--dt", type=int, default=4)
    ap.add_argument("--first", type=int, default=0, help="dump the steps from this one on")
    a = ap.parse_args()
    if a.compare:
        sys.exit(0 if compare(*a.compare) else 1)
    dump(a)
