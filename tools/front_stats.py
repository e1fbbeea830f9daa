"""Diagnostic: DP work (label relaxations) per step over a bench command's timed window.

Runs the bench's workload (bench.py's community, completable swaps, history on) with a variant
build that records each front-DP stage's front size into the workspace's S_PAD slots
(-DDRAGG_FRONT_STATS: tools/build_variant.sh stats '1i #define DRAGG_FRONT_STATS'), and after
every TIMED step reads them back: children (parent label, duty) per stage = 7 x the previous
stage's front (1 label before stage 0), summed over the homes whose DP ran (optimal or
round_fail).  Usage (same arguments as bench.py):
    DRAGG_LIB=varlib/stats.so python tools/front_stats.py --json OUT.json -- --steps 20 --warmup 5"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench                                                          # noqa: E402
from dragg_amd import _lib as L                                      # noqa: E402
from dragg_amd.aggregator import DeviceAggregator                   # noqa: E402

argv = sys.argv[1:]
out_path = argv[argv.index("--json") + 1] if "--json" in argv else None
bargs = bench.parse(argv[argv.index("--") + 1:] if "--" in argv else [])
assert bargs.workload == "rbo", "rbo workload only"
homes, oat, ghi, tou = bench.bench_community(bargs)
torch.cuda.set_device(0)
homes, _ = bench.reference_completable(homes, oat, ghi, tou, seed=12)
total = bargs.warmup + bargs.steps
agg = DeviceAggregator(homes, oat, ghi, tou, 0, total, reward_price=[0.0], int_mode=bargs.int_mode, seed=12,
                       keep_history=not bargs.no_history)
N, H = agg.batch.N, agg.batch.H
NBC = 336                                      # NB_CAP: the back-pointer rows before the solutions
par = ((N * H * NBC * 2 + 255) // 256) * 256
kids_tot, fT, fW, n_ran = 0.0, [], [], 0
for t in range(total):
    agg.run_iteration()
    if t < bargs.warmup:
        continue
    torch.cuda.synchronize()
    x = agg.batch.workspace.view(torch.uint8)[par:par + N * 8 * H * 8].view(torch.float64).view(N, H, 8)[:, :, 7]
    v = x.cpu().numpy().copy()
    st = agg.batch.status.cpu().numpy()
    ran = (st == L.ST_OPTIMAL) | (st == L.ST_ROUND_FAIL)
    pr = np.floor(v[:, 0] / 1e8)
    v[:, 0] -= pr * 1e8
    nW = np.floor(v / 1e4)
    nT = v - nW * 1e4
    prevT = np.concatenate([np.ones((N, 1)), nT[:, :-1]], axis=1)
    prevW = np.concatenate([np.ones((N, 1)), nW[:, :-1]], axis=1)
    kids_tot += 7.0 * (prevT[ran].sum() + prevW[ran].sum())
    fT.append(nT[ran].mean())
    fW.append(nW[ran].mean())
    n_ran += int(ran.sum())
res = {"window": [bargs.warmup, total], "children_per_step": kids_tot / bargs.steps,
       "front_mean_T": float(np.mean(fT)), "front_mean_W": float(np.mean(fW)), "homes_dp_per_step": n_ran / bargs.steps,
       "workload": bench.traffic_key(bargs.homes, H, bargs.dt, bargs.month, bargs.int_mode, 1, "rbo", bargs.steps,
                                     bargs.warmup)}
print(json.dumps(res))
if out_path:
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
