#!/usr/bin/env python3
"""Proven-optimum fixture at the headline configuration (BASELINE configs[2]: 12 h horizon at
15-min steps, H = 48, July) -- TEST INFRASTRUCTURE, run in this container only.

Takes homes of the bench's 10,000-home synthetic community (`dragg_amd.community`, the same
generator and seeds as bench.py), builds each solve's inputs with the oracle's restatement of
the reference (`oracle/mpc.py`: water draws, initial conditions, environment slices), and
solves the reference MILP (`mpc_calc.py:291-451`, assembled in the reference's own row order)
with HiGHS to PROVEN optimality (mip_rel_gap 0, no incumbent accepted).  Half the instances
are t = 0, half t = 1 (the hash of a t = 0 solve feeds the t = 1 inputs, as the reference's
redis round trip does, `mpc_calc.py:264-289`).  The records carry explicit inputs, so the GPU
tests need nothing but this file.

Usage:  python tests/golden/make_proven_h48.py [n_instances] [workers]
"""
import gzip
import json
import math
import multiprocessing as mp
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

N_COMMUNITY, SEED_HOMES, SEED_WEATHER, MONTH, DT, HH = 10000, 12, 3, 7, 4, 12


_CACHE = {}


def community():
    if "c" in _CACHE:
        return _CACHE["c"]
    from dragg_amd.community import synthetic_homes, synthetic_weather
    steps = 100
    sim_hours = math.ceil(steps / DT)
    days = math.ceil((sim_hours + HH + 2) / 24) + 1
    homes = synthetic_homes(N_COMMUNITY, seed=SEED_HOMES, days=days, dt=DT, horizon_hours=HH)
    oat, ghi, tou = synthetic_weather(days, DT, sim_hours, seed=SEED_WEATHER, month=MONTH)
    _CACHE["c"] = homes, np.asarray(oat, float), np.asarray(ghi, float), np.asarray(tou, float)
    return _CACHE["c"]


def milp(P, time_limit):
    """HiGHS on the reference model; returns (status, objective, x, gap, seconds)."""
    from scipy.optimize import milp as _milp, LinearConstraint, Bounds
    t0 = time.time()
    res = _milp(P["c"], constraints=[LinearConstraint(P["A_eq"], P["b_eq"], P["b_eq"]),
                                     LinearConstraint(P["A_ub"], -np.inf, P["b_ub"])],
                integrality=P["integrality"], bounds=Bounds(-np.inf, np.inf),
                options={"time_limit": time_limit, "mip_rel_gap": 0.0, "presolve": True})
    dt = time.time() - t0
    x = None if res.x is None else res.x.copy()
    if x is not None:
        ii = P["integrality"] == 1
        x[ii] = np.floor(x[ii] + 0.5)
    return int(res.status), (None if x is None else float(P["c"] @ x)), x, getattr(res, "mip_gap", None), dt


def solve_one(args):
    idx, t, time_limit = args
    from oracle import mpc as M
    homes, oat, ghi, tou = community()
    home = homes[idx]
    hc = M.home_const(home)
    env = dict(oat=oat, ghi=ghi, tou=tou, start_hour_index=0, reward_price=[0.0])
    rng = np.random.default_rng([SEED_HOMES, idx])
    hsh = {}
    for tt in range(t + 1):
        draw, _, _ = M.water_draws(hc, tt)
        T0, Tw0, E0, counter = M.initial_conditions(hc, tt, hsh, draw)
        o, g, tu = M.env_slice(oat, ghi, tou, 0, tt, hc.H)
        noise = rng.standard_normal(hc.H)
        si = M.StepInput(t=tt, T0=T0, Tw0=Tw0, E0=E0, oat=o, ghi=g, price=M.total_price(tu, [0.0], hc.H),
                         draw=draw, winter=M.season_is_winter(o, noise))
        P = M.build_problem(hc, si)
        prev = dict(hsh)
        status, obj, x, gap, secs = milp(P, time_limit)
        st = "optimal" if status == 0 else ("infeasible" if status == 2 else f"highs_{status}")
        ov, _ = M.cleanup(hc, si, st if st in ("optimal", "infeasible") else "fail", x, hsh, counter)
        for kk, v in ov.items():
            hsh[kk] = M.enc(v)
    Lay = P["layout"]
    milp_x = None
    if x is not None:
        milp_x = {k: Lay.get(x, k).tolist() for k in ("hvac_cool_on", "hvac_heat_on", "wh_heat_on",
                                                       "temp_in_ev", "temp_wh_ev")}
    return dict(name=home["name"], home=idx, type=home["type"], t=t, T0=T0, Tw0=Tw0, E0=E0, counter_in=counter,
                draw_size=list(map(float, draw)), oat=list(map(float, o)), ghi=list(map(float, g)),
                tou=list(map(float, tu)), reward_price=[0.0], total_price=list(map(float, si.price)),
                noise=list(map(float, noise)), season="winter" if si.winter else "summer",
                status=st, milp_status=status, milp_obj=obj, milp_gap=None if gap is None else float(gap),
                milp_seconds=secs, prev_hash=prev, milp_x=milp_x)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    workers = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    # homes spread over the community, the same number of each type (the generator lists them in
    # blocks: pv_battery, pv_only, battery_only 20 % each, then base 40 %)
    homes = community()[0]
    blocks = {}
    for i, h in enumerate(homes):
        blocks.setdefault(h["type"], []).append(i)
    per = n // len(blocks)
    idx = [b[(j * 397) % len(b)] for b in blocks.values() for j in range(per)]
    jobs = [(h, i % 2, 3600.0) for i, h in enumerate(idx)]
    jobs.sort(key=lambda j: -j[1])                 # the t = 1 jobs (two solves) first
    with mp.get_context("fork").Pool(workers) as pool:
        recs = pool.map(solve_one, jobs, chunksize=1)
    used = sorted({r["home"] for r in recs})
    out = dict(scenario="proven_h48_july", params=dict(community=N_COMMUNITY, seed_homes=SEED_HOMES,
               seed_weather=SEED_WEATHER, month=MONTH, dt=DT, horizon_hours=HH),
               homes=[homes[i] for i in used], records=recs)
    os.makedirs(os.path.join(HERE, "proven"), exist_ok=True)
    path = os.path.join(HERE, "proven", "h48_july.json.gz")
    with gzip.open(path, "wt") as f:
        json.dump(out, f, separators=(",", ":"), default=float)
    st = {}
    for r in recs:
        st[(r["status"], r["milp_status"])] = st.get((r["status"], r["milp_status"]), 0) + 1
    print(f"{len(recs)} records, statuses {st}, max HiGHS time {max(r['milp_seconds'] for r in recs):.1f}s, "
          f"file {os.path.getsize(path) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
