"""GPU diagnostic: dump the inputs of the solves the exactness questions are about, for the CPU side.

Runs (a) the bench workload (BASELINE configs[2]: bench.py's 10,000-home community, July, H = 48)
for 100 closed-loop steps and (b) configs[3] (100,000 homes, H = 24, July, 672 steps, the at-size
test's community) and writes, for every solve whose status is ROUND_FAIL or whose integer path
used the bucketed approximation because of a narrow feasible set (int_path reason 2), the solve's
inputs as the oracle restates them from the previous step's hash (oracle/mpc.py), with our status,
objective and int_path.  tests/golden/make_round_fail_verdicts.py decides them on the full reference
model with HiGHS.   Usage: python tools/dump_cases.py OUT.json [--skip-100k]"""
import json
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dragg_amd import _lib as L                                       # noqa: E402
from dragg_amd.aggregator import DeviceAggregator                     # noqa: E402
from dragg_amd.community import synthetic_homes, synthetic_weather, reference_completable  # noqa: E402
from oracle import mpc as M                                           # noqa: E402
from tests.test_gpu_fullsize import _hash_dict                        # noqa: E402


def reason(path, chain):
    return (int(path) >> (4 + 4 * chain)) & 0xF if int(path) & (1 << chain) else 0


def run(tag, n, hours, dt, steps, month, seed_h, seed_w, seed, completable, out):
    sim_hours = math.ceil(steps / dt)
    days = math.ceil((sim_hours + hours + 2) / 24) + 1
    homes = synthetic_homes(n, seed=seed_h, days=days, dt=dt, horizon_hours=hours)
    oat, ghi, tou = synthetic_weather(days, dt, sim_hours, seed=seed_w, month=month)
    if completable:
        homes, _ = reference_completable(homes, oat, ghi, tou, seed=seed)
    agg = DeviceAggregator(homes, oat, ghi, tou, 0, steps, reward_price=[0.0], seed=seed, keep_history=False)
    b = agg.batch
    n_rf = n_nar = 0
    for t in range(steps):
        prev = (b.vals.clone(), b.fc.clone())
        agg.run_iteration()
        st = b.status.cpu().numpy()
        path = b.int_path.cpu().numpy()
        narrow = np.array([reason(p, 0) == 2 or reason(p, 1) == 2 or (int(p) & L.PATH_STEPS) != 0 for p in path])
        pick = np.flatnonzero((st == L.ST_ROUND_FAIL) | narrow)
        if len(pick) == 0:
            continue
        noise = b.season_noise(t).cpu().numpy()
        pv, pf = prev[0].cpu().numpy(), prev[1].cpu().numpy()
        obj = b.obj.cpu().numpy()
        for i in pick:
            hc = M.home_const(homes[i])
            draw, _, _ = M.water_draws(hc, t)
            hsh = _hash_dict(pv, pf, i) if t else {}
            T0, Tw0, E0, cnt = M.initial_conditions(hc, t, hsh, draw)
            o, g, tt = M.env_slice(oat, ghi, tou, 0, t, hc.H)
            out.append(dict(source=tag, t=t, i=int(i), home=homes[i], T0=T0, Tw0=Tw0, E0=E0, counter=cnt,
                            oat=list(map(float, o)), ghi=list(map(float, g)),
                            price=list(map(float, M.total_price(tt, [0.0], hc.H))), draw=list(map(float, draw)),
                            winter=bool(M.season_is_winter(o, noise[:, i])),
                            status=L.STATUS_NAMES[st[i]], obj=float(obj[i]), int_path=int(path[i])))
            n_rf += st[i] == L.ST_ROUND_FAIL
            n_nar += bool(narrow[i])
    torch.cuda.synchronize()
    print(f"{tag}: {n_rf} ROUND_FAIL, {n_nar} narrow-set solves dumped", flush=True)


if __name__ == "__main__":
    out = []
    torch.cuda.set_device(0)
    run("bench_h48_july_100", 10000, 12, 4, 100, 7, 12, 3, 12, False, out)
    if "--skip-100k" not in sys.argv:
        run("configs3_100k_h24_july_672", 100000, 6, 4, 672, 7, 41, 42, 41, True, out)
    with open(sys.argv[1], "w") as f:
        json.dump(out, f)
    print(f"{len(out)} cases -> {sys.argv[1]}")
