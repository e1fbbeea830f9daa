#!/usr/bin/env python3
"""Per-phase cycle breakdown of the solver kernel (diagnostic, GPU only).

Runs the bench workload with `dragg_mpc_out.cycles` enabled and prints, per phase, the
mean shader cycles per home, the share of the total, and the distribution of per-home
totals (the launch time is set by the slowest home of the step)."""
import argparse
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--homes", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--horizon-hours", type=int, default=6)
    ap.add_argument("--dt", type=int, default=4)
    ap.add_argument("--int-mode", default="round")
    ap.add_argument("--month", type=int, default=1)
    ap.add_argument("--out", default=None)
    ap.add_argument("--world", type=int, default=1, help="rank 0's strided shard of a community sharded this wide")
    ap.add_argument("--rl", action="store_true", help="bench.py's smooth RL reward price, a new one every step")
    a = ap.parse_args()
    import numpy as np
    import torch
    from dragg_amd import _lib as L
    from dragg_amd.aggregator import DeviceAggregator
    from dragg_amd.community import synthetic_homes, synthetic_weather
    sim_hours = math.ceil(a.steps / a.dt)
    days = math.ceil((sim_hours + a.horizon_hours + 2) / 24) + 1
    homes = synthetic_homes(a.homes, seed=12, days=days, dt=a.dt, horizon_hours=a.horizon_hours)
    oat, ghi, tou = synthetic_weather(days, a.dt, sim_hours, seed=3, month=a.month)
    agg = DeviceAggregator(homes, oat, ghi, tou, 0, a.steps, reward_price=[0.0], int_mode=a.int_mode,
                           seed=12, keep_history=False, rank=0, world=a.world)
    agg.batch.enable_phase_timing(True)
    cyc, st, it, kms = [], [], [], []
    H = agg.batch.H
    rng = np.random.default_rng(5)
    for _ in range(a.steps):
        if a.rl:
            agg.set_reward_price(rng.uniform(-0.02, 0.02) - 0.03 * np.cos(np.arange(H) / 3.0))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        agg.run_iteration()
        e1.record()
        agg.collect_data(defer=True)
        torch.cuda.synchronize()
        kms.append(e0.elapsed_time(e1))
        cyc.append(agg.batch.cycles.cpu().numpy().copy())
        st.append(agg.batch.status.cpu().numpy().copy())
        it.append(agg.batch.iters.cpu().numpy().copy())
    cyc = np.stack(cyc)            # [T][NPHASE][N]
    st, it = np.stack(st), np.stack(it)
    tot = cyc.sum(1)               # [T][N]
    res = {"homes": a.homes, "steps": a.steps, "H": agg.batch.H, "kernel_ms_mean": float(np.mean(kms)),
           "kernel_ms_max": float(np.max(kms)), "phase_mean_cycles": {}, "phase_share": {},
           "home_total_cycles_pct": {}, "slowest_home_phase_cycles": {}}
    for p, name in enumerate(L.PHASES):
        res["phase_mean_cycles"][name] = float(cyc[:, p].mean())
        res["phase_share"][name] = float(cyc[:, p].sum() / max(1, tot.sum()))
    for q in (50, 90, 99, 100):
        res["home_total_cycles_pct"][str(q)] = float(np.percentile(tot, q))
    t_i, h_i = np.unravel_index(np.argmax(tot), tot.shape)
    for p, name in enumerate(L.PHASES):
        res["slowest_home_phase_cycles"][name] = int(cyc[t_i, p, h_i])
    res["slowest_home"] = {"step": int(t_i), "home": int(h_i), "type": int(agg.batch.types_host[h_i]),
                           "status": int(st[t_i, h_i]), "iters": int(it[t_i, h_i])}
    res["per_step_max_over_mean"] = float(np.mean(tot.max(1) / tot.mean(1)))
    # the step's slowest home (sets the launch time when homes < resident slots): its phase split
    slow = np.argmax(tot, axis=1)
    res["step_slowest_phase_share"] = {name: float(np.mean([cyc[t, p, slow[t]] / tot[t, slow[t]]
                                                            for t in range(a.steps)])) for p, name in enumerate(L.PHASES)}
    res["step_slowest_type_counts"] = np.bincount(agg.batch.types_host[slow], minlength=4).tolist()
    res["step_max_cycles_pct"] = {str(q): float(np.percentile(tot.max(1), q)) for q in (10, 50, 90)}
    res["kernel_ms_per_step"] = [round(x, 4) for x in kms]
    res["iters_pct"] = {str(q): float(np.percentile(it, q)) for q in (50, 90, 99, 100)}
    res["status_counts"] = {n: int((st == i).sum()) for i, n in enumerate(L.STATUS_NAMES)}
    by_type = {}
    for ty in range(4):
        m = agg.batch.types_host == ty
        by_type[str(ty)] = float(tot[:, m].mean()) if m.any() else None
    res["mean_total_cycles_by_type"] = by_type
    s = json.dumps(res, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s)


if __name__ == "__main__":
    main()
