"""Diagnostic: what sets a small shard's step time (the per-GPU load of an 8-GPU strong-scaling run is
1,250 homes: below one home per wave slot the hot launch lasts as long as its slowest home).  For shard
r of N of the bench community over the driver's window, per step: the hot launch's duration (HIP events)
and the phase cycles of its slowest homes, and over the window the mean phase split of the slowest 1 %
against all homes, by home type.
Usage: python tools/shard_tail.py [--of 8] [--rank 0] [--steps 25] [--first 5]"""
import argparse
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
ap.add_argument("--of", type=int, default=8)
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--steps", type=int, default=25)
ap.add_argument("--first", type=int, default=5)
a = ap.parse_args()
bargs = bench.parse(["--steps", str(a.steps - a.first), "--warmup", str(a.first)])
homes, oat, ghi, tou = bench.bench_community(bargs)
homes, _ = bench.reference_completable(homes, oat, ghi, tou, seed=12)
agg = DeviceAggregator(homes, oat, ghi, tou, 0, a.steps, reward_price=[0.0], seed=12, keep_history=False,
                       rank=a.rank, world=a.of)
agg.batch.enable_phase_timing()
types = agg.batch.types_host
names = ["base", "pv_only", "battery_only", "pv_battery"]
tail_acc, all_acc, tail_types, n_tail, n_all = np.zeros(L.NPHASE), np.zeros(L.NPHASE), np.zeros(4), 0, 0
ms = []
for t in range(a.steps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    agg.run_iteration()
    e1.record()
    torch.cuda.synchronize()
    if t < a.first:
        continue
    ms.append(e0.elapsed_time(e1))
    cyc = agg.batch.cycles.cpu().numpy().astype(float)
    tot = cyc.sum(0)
    o = np.argsort(-tot)
    k = max(1, len(tot) // 100)
    tail_acc += cyc[:, o[:k]].sum(1)
    all_acc += cyc.sum(1)
    n_tail += k
    n_all += len(tot)
    for i in o[:k]:
        tail_types[types[i]] += 1
    top = o[0]
    print(f"t={t}: step {ms[-1]:.3f} ms, slowest home {top} ({names[types[top]]}) {tot[top]:.0f} cycles "
          f"{ {p: int(v) for p, v in zip(L.PHASES, cyc[:, top]) if v} }, median home {np.median(tot):.0f}", flush=True)
print("mean step ms", np.mean(ms))
print("slowest 1 %:", {p: round(v / n_tail) for p, v in zip(L.PHASES, tail_acc) if v},
      "types", dict(zip(names, tail_types.astype(int).tolist())))
print("all homes:  ", {p: round(v / n_all) for p, v in zip(L.PHASES, all_acc) if v},
      "types", dict(zip(names, np.bincount(types, minlength=4).tolist())))
