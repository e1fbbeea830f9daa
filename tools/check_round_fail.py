#!/usr/bin/env python3
"""Diagnostic (GPU + CPU oracle): run the bench workload's closed loop, collect every home-step
the integer DP reported as ST_ROUND_FAIL (relaxation feasible, no integer schedule found) and
re-solve those exact MILPs with the oracle (HiGHS).  A HiGHS 'infeasible' confirms the
reference would fall back too; an 'optimal' is a home the bucketing lost."""
import argparse
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--homes", type=int, default=10000)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--horizon-hours", type=int, default=12)
    ap.add_argument("--month", type=int, default=7)
    ap.add_argument("--max-cases", type=int, default=20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import numpy as np
    import torch
    from dragg_amd import _lib as L
    from dragg_amd.aggregator import DeviceAggregator
    from dragg_amd.community import synthetic_homes, synthetic_weather
    from oracle import mpc as M
    dt = 4
    sim_hours = math.ceil(a.steps / dt)
    days = math.ceil((sim_hours + a.horizon_hours + 2) / 24) + 1
    homes = synthetic_homes(a.homes, seed=12, days=days, dt=dt, horizon_hours=a.horizon_hours)
    oat, ghi, tou = synthetic_weather(days, dt, sim_hours, seed=3, month=a.month)
    agg = DeviceAggregator(homes, oat, ghi, tou, 0, a.steps, reward_price=[0.0], seed=12, keep_history=True)
    for _ in range(a.steps):
        agg.run_iteration()
        agg.collect_data()
    torch.cuda.synchronize()
    st = agg.status_hist.cpu().numpy()
    hist = agg.hist.cpu().numpy()
    cases = np.argwhere(st == L.ST_ROUND_FAIL)
    res = {"round_fail": int(len(cases)), "solves": int(st.size), "checked": []}
    for t, i in cases[:a.max_cases]:
        t, i = int(t), int(i)
        hc = M.home_const(homes[i])
        draw, _, _ = M.water_draws(hc, t)
        if t == 0:
            T0, Tw0, E0, cnt = M.initial_conditions(hc, 0, {}, draw)
        else:
            prev = {k: hist[t - 1, L.K[k], i] for k in ("temp_in_opt", "temp_wh_opt", "solve_counter", "e_batt_opt",
                                                        "p_batt_ch", "p_batt_disch")}
            hsh = {k: repr(float(v)) for k, v in prev.items() if not np.isnan(v)}
            hsh["solve_counter"] = str(int(prev["solve_counter"]))
            T0, Tw0, E0, cnt = M.initial_conditions(hc, t, hsh, draw)
        o, g, tt = M.env_slice(oat, ghi, tou, 0, t, hc.H)
        noise = agg.batch.season_noise(t)[:, i].cpu().numpy()
        si = M.StepInput(t=t, T0=T0, Tw0=Tw0, E0=E0, oat=o, ghi=g, price=M.total_price(tt, [0.0], hc.H),
                         draw=draw, winter=M.season_is_winter(o, noise))
        P = M.build_problem(hc, si)
        s_lp, _, _ = M.solve_problem(P, integer=False)
        s_ip, _, obj = M.solve_problem(P, integer=True, time_limit=60.0)
        res["checked"].append({"t": t, "home": i, "type": homes[i]["type"], "lp": s_lp, "milp": s_ip, "milp_obj": obj})
        print(res["checked"][-1], flush=True)
    s = json.dumps(res, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s)


if __name__ == "__main__":
    main()
