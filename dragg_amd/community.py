"""Synthetic communities and NSRDB-shaped weather for runs without the reference's data.

There is no network here: the benchmark configs use seeded synthetic
inputs of the reference's shapes.
* `synthetic_weather`: half-hourly integer OAT/GHI like `dragg/data/nsrdb.csv` (Houston,
  January: OAT 5-15 C, GHI peak ~323 W/m2), upsampled to `dt` steps per hour exactly as
  `Aggregator._import_ts_data` does (aggregator.py:140-154: ceil(dt/2) copies of the :00
  row, floor(dt/2) of the :30 row), and the TOU list of `_build_tou_price` with the
  reference's peak-overwrite quirk (aggregator.py:206-216: 0.09 for hours 9-20, else 0.07)
  forward-filled past the end (aggregator.py:219-230).
* `synthetic_homes`: home dicts with the schema of `create_homes` (aggregator.py:273-587),
  parameters drawn uniformly from the config.toml ranges (config.toml:32-58) and hourly
  water draws shaped like waterdraw_profiles.csv (per-minute flows in multiples of
  3.78 L/min, ~3 % of minutes non-zero), clipped to the tank size (aggregator.py:376).
"""
import math

import numpy as np

CONFIG_RANGES = dict(  # config.toml:32-58
    hvac=dict(r=(6.8, 9.199999999999999), c=(4.25, 5.75), p_c=(3.5, 3.5), p_h=(3.5, 3.5),
              sp=(18, 22), db=(2, 3)),
    wh=dict(r=(18.7, 25.3), p=(2.5, 2.5), sp=(45.5, 48.5), db=(9, 12), size=(200, 300)),
    battery=dict(max_rate=(3, 5), capacity=(9.0, 13.5), lower=(0.01, 0.15), upper=(0.85, 0.99),
                 ch_eff=(0.85, 0.95), disch_eff=(0.97, 0.99)),
    pv=dict(area=(20, 32), eff=(0.15, 0.2)),
)


# Houston-like monthly climate (NSRDB-shaped): mean OAT, diurnal amplitude, clear-sky GHI peak,
# daylight window.  January matches dragg/data/nsrdb.csv's first days (OAT 5-15 C, peak ~323).
CLIMATE = {1: (10.0, 5.0, 323.0, 7.0, 17.5), 4: (21.0, 5.0, 760.0, 6.5, 19.0),
           7: (29.0, 5.0, 900.0, 6.0, 20.0), 10: (22.0, 5.0, 650.0, 7.0, 18.5)}


def half_hourly_weather(days, seed=0, t_mean=10.0, t_amp=5.0, ghi_peak=323.0, sun=(7.0, 17.5)):
    """Integer OAT (C) and GHI (W/m2) at :00 and :30 of each hour (NSRDB rows)."""
    rng = np.random.default_rng(seed)
    n = days * 48
    hours = np.arange(n) / 2.0
    hod = hours % 24
    day = np.floor(hours / 24)
    drift = np.repeat(rng.normal(0, 1.5, days + 1), 48)[:n]
    oat = t_mean + drift + t_amp * np.sin(2 * math.pi * (hod - 9) / 24) + rng.normal(0, 0.4, n)
    oat = np.trunc(oat).astype(int)
    cloud = np.repeat(rng.uniform(0.55, 1.0, days + 1), 48)[:n]
    rise, set_ = sun
    ghi = np.where((hod >= rise) & (hod <= set_),
                   ghi_peak * cloud * np.sin(math.pi * (hod - rise) / (set_ - rise)), 0.0)
    ghi = np.trunc(np.clip(ghi, 0, None)).astype(int)
    del day
    return oat, ghi


def upsample(rows, dt):
    """`_import_ts_data` row repetition (aggregator.py:140-154)."""
    rows = np.asarray(rows)
    reps = np.tile([math.ceil(dt / 2), math.floor(dt / 2)], len(rows) // 2)
    return np.repeat(rows, reps)


def tou_hourly(hours, start_hour=0, base=0.07, shoulder=(9, 21), shoulder_price=0.09):
    """`_build_tou_price` (aggregator.py:206-216); the peak assignment is overwritten there."""
    hod = (start_hour + np.arange(hours)) % 24
    return np.where((hod >= shoulder[0]) & (hod < shoulder[1]), shoulder_price, base)


def synthetic_weather(days, dt, sim_hours, seed=0, month=1):
    """(oat, ghi, tou) lists at dt steps per hour covering `days` days; tou forward-filled past
    `sim_hours` like `join_data` (aggregator.py:219-230).  `month` picks the climate row."""
    tm, ta, gp, rise, set_ = CLIMATE[month]
    oat_hh, ghi_hh = half_hourly_weather(days, seed, tm, ta, gp, (rise, set_))
    oat = upsample(oat_hh, dt).astype(float)
    ghi = upsample(ghi_hh, dt).astype(float)
    tou_h = tou_hourly(sim_hours)
    n = len(oat)
    tou = np.empty(n)
    idx = np.arange(n) // dt
    tou[:] = tou_h[np.minimum(idx, sim_hours - 1)]
    return oat, ghi, tou


def hourly_water_draws(n_homes, hours, rng, sizes):
    """Hourly draw volumes (L) shaped like waterdraw_profiles.csv, clipped to the tank size."""
    hod = np.arange(hours) % 24
    shape = 0.4 + np.exp(-0.5 * ((hod - 7.5) / 1.5) ** 2) * 2.2 + np.exp(-0.5 * ((hod - 19.5) / 2.0) ** 2) * 1.8
    p_min = 0.03 * shape / shape.mean()                      # share of non-zero minutes
    active = rng.binomial(60, np.clip(p_min, 0, 1)[None, :], size=(n_homes, hours))
    flow = 3.78 * rng.integers(1, 4, size=(n_homes, hours))   # L/min in multiples of 3.78
    vol = active * flow * (1 + 0.2 * rng.standard_normal((n_homes, hours)))
    return np.clip(vol, 0, sizes[:, None])


def synthetic_homes(n, mix=(0.4, 0.2, 0.2, 0.2), seed=12, days=2, dt=4, horizon_hours=6,
                    sub_steps=6, discount=0.92):
    """n home dicts; mix = fractions of (base, pv_only, battery_only, pv_battery).

    Listed in the reference's order: pv_battery, pv_only, battery_only, base
    (aggregator.py:392-560)."""
    rng = np.random.default_rng(seed)
    n_pv = int(round(n * mix[1]))
    n_b = int(round(n * mix[2]))
    n_pvb = int(round(n * mix[3]))
    n_base = n - n_pv - n_b - n_pvb
    u = lambda lo_hi, size=n: rng.uniform(lo_hi[0], lo_hi[1], size)  # noqa: E731
    H, W = CONFIG_RANGES["hvac"], CONFIG_RANGES["wh"]
    r, c, pc, ph = u(H["r"]), u(H["c"]), u(H["p_c"]), u(H["p_h"])
    sp, db, pos = u(H["sp"]), u(H["db"]), rng.uniform(0.25, 0.75, n)
    tmin, tmax = sp - 0.5 * db, sp + 0.5 * db
    tinit = tmin + pos * db
    wr, wp, wsp, wdb, wpos = u(W["r"]), u(W["p"]), u(W["sp"]), u(W["db"]), rng.uniform(0.25, 0.75, n)
    wmin, wmax = wsp - 0.5 * wdb, wsp + 0.5 * wdb
    winit = wmin + wpos * wdb
    size = u(W["size"])
    draws = hourly_water_draws(n, 24 * days, rng, size)
    hems = {"horizon": horizon_hours, "hourly_agg_steps": dt, "sub_subhourly_steps": sub_steps,
            "solver": "MI355X", "discount_factor": discount}
    types = ["pv_battery"] * n_pvb + ["pv_only"] * n_pv + ["battery_only"] * n_b + ["base"] * n_base
    B, PV = CONFIG_RANGES["battery"], CONFIG_RANGES["pv"]
    homes = []
    for i, ty in enumerate(types):
        h = {"name": f"home-{i:06d}", "type": ty,
             "hvac": {"r": r[i], "c": c[i], "p_c": pc[i], "p_h": ph[i], "temp_in_min": tmin[i],
                      "temp_in_max": tmax[i], "temp_in_sp": sp[i], "temp_in_init": tinit[i]},
             "wh": {"r": wr[i], "p": wp[i], "temp_wh_min": wmin[i], "temp_wh_max": wmax[i],
                    "temp_wh_sp": wsp[i], "temp_wh_init": winit[i], "tank_size": size[i],
                    "draw_sizes": draws[i].tolist()},
             "hems": dict(hems)}
        if "battery" in ty:
            h["battery"] = {"max_rate": rng.uniform(*B["max_rate"]), "capacity": rng.uniform(*B["capacity"]),
                            "capacity_lower": rng.uniform(*B["lower"]), "capacity_upper": rng.uniform(*B["upper"]),
                            "ch_eff": rng.uniform(*B["ch_eff"]), "disch_eff": rng.uniform(*B["disch_eff"]),
                            "e_batt_init": rng.uniform(B["lower"][1], B["upper"][0])}
        if "pv" in ty:
            h["pv"] = {"area": rng.uniform(*PV["area"]), "eff": rng.uniform(*PV["eff"])}
        homes.append(h)
    return homes


def reference_completable(homes, oat, ghi, tou, seed, reward_price=(0.0,), start_index=0, rounds=8):
    """A community the reference completes.  A battery home whose t = 0 solve fails leaves no
    e_batt_opt in its hash, and the reference raises KeyError('e_batt_opt') at t = 1
    (mpc_calc.py:280-289).  The failures come from the season draw (keyed by the home's index and
    the run's `seed`: a "winter" draw on a hot day leaves the cooling duty at zero), not from the
    home's parameters, so each such battery home swaps places with a home without a battery (whose
    failed t = 0 solve the reference survives) until the t = 0 step solves every battery home.
    Runs t = 0 on the GPU; deterministic (every rank builds the same community).
    -> (homes, swaps)"""
    import torch
    from . import _lib as L
    from .mpc import MPCBatch
    homes, swaps = list(homes), 0
    donors = [j for j in range(len(homes) - 1, -1, -1) if "battery" not in homes[j]["type"]]
    for _ in range(rounds):
        b = MPCBatch(homes, oat, ghi, tou, start_index, list(reward_price), int_mode="round", seed=seed)
        b.step(0)
        st = b.status.cpu().numpy()
        del b
        torch.cuda.empty_cache()
        bad = [i for i, h in enumerate(homes) if "battery" in h["type"] and st[i] != L.ST_OPTIMAL]
        if not bad or not donors:
            break
        for i in bad:
            if not donors:
                break
            j = donors.pop(0)
            homes[i], homes[j] = homes[j], homes[i]
            swaps += 1
    return homes, swaps
