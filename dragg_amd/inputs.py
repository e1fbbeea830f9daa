"""Host-side input pipeline of a dragg run: config, weather / price series, community.

SURVEY.md §8 rows F2 (environment pipeline) and F3 (community generator).  These produce
the solver's inputs once per run; they are restated here so that a run configured like the
reference (its config.toml, NSRDB csv and water-draw profiles) feeds the MI355X solver the
same numbers the reference's MPCCalc would see:

* `load_weather`     aggregator.py:129-165  `_import_ts_data` (row repetition per dt)
* `tou_prices`       aggregator.py:206-216  `_build_tou_price` (peak overwritten by shoulder)
* `join_series`      aggregator.py:219-230  `join_data` (outer join + forward fill, run mask)
* `start_hour_index` aggregator.py:630-638  (an HOUR count later used as a STEP index)
* `check_series`     aggregator.py:617-628  `check_all_data_indices`
* `create_homes`     aggregator.py:273-587  (legacy global-RNG draw order, bit-exact)

The pandas operations whose rounding or ordering defines the reference's numbers (the
hourly resampling sum, the outer-join forward fill, the column sample) are done with pandas
itself; everything else is vectorised numpy.  Parity: tests/test_inputs.py against the
communities, series and start indices the reference produced (tests/golden/*.json.gz).
"""
import math
import os
import random
import string
from datetime import datetime, timedelta

import numpy as np
import pandas as pd

TYPES = ("pv_battery", "pv_only", "battery_only", "base")   # creation order, aggregator.py:391-578


class ConfigError(ValueError):
    """A configuration or data problem the reference reports with sys.exit(1)."""


def read_config(path):
    """config.toml -> dict (the reference's `toml.load` + top-level key check,
    aggregator.py:88-109; tomli here)."""
    import tomli
    if not os.path.exists(path):
        raise ConfigError(f"Configuration file does not exist: {path}")
    with open(path, "rb") as f:
        cfg = tomli.load(f)
    missing = {"community", "home", "simulation", "agg"} - set(cfg)
    if missing:
        raise ConfigError(f"{missing} must be configured in the config file.")
    return cfg


def run_window(cfg):
    """(start_dt, end_dt, hours) from [simulation] (aggregator.py:111-127)."""
    try:
        start = datetime.strptime(cfg["simulation"]["start_datetime"], "%Y-%m-%d %H")
        end = datetime.strptime(cfg["simulation"]["end_datetime"], "%Y-%m-%d %H")
    except ValueError as e:
        raise ConfigError(f"Error parsing datetimes: {e}") from e
    return start, end, int((end - start).total_seconds() / 3600)


def load_weather(path, dt):
    """NSRDB csv (2 preamble lines; columns Year, Month, Day, Hour, Minute, GHI, ...,
    Temperature) -> DataFrame indexed by timestamp at 60/dt-minute steps, int columns GHI, OAT.

    Each :00 row is repeated ceil(dt/2) times and each :30 row floor(dt/2) times, then the
    minutes are relabelled 0, 60/dt, ... within every hour (aggregator.py:140-146)."""
    if not os.path.exists(path):
        raise ConfigError(f"Timeseries data file does not exist: {path}")
    raw = pd.read_csv(path, skiprows=2)
    reps = np.where(raw["Minute"].to_numpy() == 0, math.ceil(dt / 2), math.floor(dt / 2)).astype(np.int64)
    rows = np.repeat(np.arange(len(raw)), reps)
    n = len(rows)
    if n % dt:
        raise ConfigError("weather rows do not form whole hours at this dt")
    sel = raw.iloc[rows]
    minute = (60 // dt) * np.tile(np.arange(dt), n // dt)
    ts = pd.to_datetime(pd.DataFrame({"year": sel["Year"].to_numpy(), "month": sel["Month"].to_numpy(),
                                      "day": sel["Day"].to_numpy(), "hour": sel["Hour"].to_numpy(),
                                      "minute": minute}))
    return pd.DataFrame({"GHI": sel["GHI"].astype(str).astype(int).to_numpy(),
                         "OAT": sel["Temperature"].astype(str).astype(int).to_numpy()},
                        index=pd.DatetimeIndex(ts, name="ts"))


def tou_prices(start, hours, agg):
    """Hourly TOU price from `start` for `hours` hours (aggregator.py:206-216).  With TOU on,
    the reference assigns the peak price and then overwrites the whole column with the
    shoulder assignment, so only the shoulder window survives (reproduced; the peak keys
    must still be present)."""
    idx = pd.date_range(start=start, periods=hours, freq="h")
    base = float(agg["base_price"])
    tou = np.full(hours, base)
    if agg["tou_enabled"] == True:  # noqa: E712  (the reference's comparison)
        t = agg["tou"]
        sd = [int(i) for i in t["shoulder_times"]]
        [int(i) for i in t["peak_times"]]
        float(t["peak_price"])
        hod = idx.hour.to_numpy()
        tou = np.where((hod >= sd[0]) & (hod < sd[1]), float(t["shoulder_price"]), base)
    return pd.DataFrame({"tou": tou}, index=idx)


def join_series(weather, tou, start, end):
    """Outer join on the timestamp, forward fill, and the run mask (aggregator.py:219-230).
    Steps before `start` keep a NaN price; the last hourly price is carried to the end of
    the weather data."""
    df = pd.merge(weather, tou, how="outer", left_index=True, right_index=True).ffill()
    mask = (df.index >= start) & (df.index < end)
    return df, mask


def check_series(all_data, start, end, horizon_hours):
    """aggregator.py:617-628."""
    if not start >= all_data.index[0]:
        raise ConfigError("The start datetime must exist in the data provided.")
    if not end + timedelta(hours=horizon_hours) <= all_data.index[-1]:
        raise ConfigError("The end datetime + the largest prediction horizon must exist in the data provided.")


def start_hour_index(all_data, start):
    """Hours from the first row to `start` (aggregator.py:630-638).  The MPC uses it as an
    index into the dt-step lists, so at dt > 1 it points at an earlier step than `start`
    (a reference quirk, kept)."""
    return int((start - all_data.index[0]).total_seconds() / 3600)


class FirstNames:
    """Stand-in for `names.get_first_name()` (the `names` package is not available here).
    The golden fixtures were generated with the same stand-in, so home names match them;
    names drawn by the real package (which also consumes Python's `random` stream and so
    changes the later name suffixes) are not reproduced -- parity of names is unpinned."""

    def __init__(self):
        self.n = 0

    def __call__(self):
        self.n += 1
        return f"Home{self.n:05d}"


def _draw_profiles(path, n_homes, ndays, tank_size):
    """Hourly water-draw lists per home (aggregator.py:361-377): per-minute flows times
    (1 + 0.2 z) with one legacy-RNG normal per cell, drawn column by column as `applymap`
    visits them; hourly sums; then per home a random profile column and `ndays` random days
    of it, clipped to the tank size."""
    wd = pd.read_csv(path, index_col=0)
    wd.index = pd.to_datetime(wd.index, format="%Y-%m-%d %H:%M:%S")
    nr, nc = wd.shape
    z = np.random.randn(nc * nr).reshape(nc, nr).T
    wd = pd.DataFrame(wd.to_numpy() * (1 + 0.2 * z), index=wd.index, columns=wd.columns)
    hourly = wd.resample("h").sum().to_numpy()
    out = []
    nc_ = hourly.shape[1]
    for j in range(n_homes):
        # `wd.sample(axis="columns")` is np.random.choice(columns, size=1, replace=False) on the global
        # legacy stream (pandas' sample with random_state=None), then that column: the same draw here,
        # without the 10^4 DataFrame copies
        col = np.random.choice(nc_, size=1, replace=False)
        prof = hourly[:, col].reshape(-1, 24)
        days = prof[np.random.choice(prof.shape[0], ndays)].flatten()
        out.append(np.clip(days, 0, tank_size[j]).tolist())
    return out


def create_homes(cfg, num_timesteps, dt, waterdraw_path, first_name=None):
    """The community of `create_homes` (aggregator.py:273-587), bit-exact: the legacy numpy
    and Python RNG streams seeded with [simulation] random_seed and consumed in the same
    order (11 parameter vectors, the draw noise and samples, then per home -- pv_battery,
    pv_only, battery_only, base -- its name suffix and its battery / PV draws)."""
    first_name = first_name or FirstNames()
    seed = cfg["simulation"]["random_seed"]
    np.random.seed(seed)
    random.seed(seed)
    com, home = cfg["community"], cfg["home"]
    n = com["total_number_homes"]
    hv, wh = home["hvac"], home["wh"]

    def u(lohi, size=n):
        return np.random.uniform(lohi[0], lohi[1], size)

    r, c, p_c, p_h = u(hv["r_dist"]), u(hv["c_dist"]), u(hv["p_cool_dist"]), u(hv["p_heat_dist"])
    sp, db, pos = u(hv["temp_sp_dist"]), u(hv["temp_deadband_dist"]), u((0.25, 0.75))
    t_lo, t_hi = sp - 0.5 * db, sp + 0.5 * db
    t_init = np.add(t_lo, np.multiply(pos, db))
    w_r, w_p, w_sp, w_db = u(wh["r_dist"]), u(wh["p_dist"]), u(wh["sp_dist"]), u(wh["deadband_dist"])
    w_pos = u((0.25, 0.75))
    w_lo, w_hi = w_sp - 0.5 * w_db, w_sp + 0.5 * w_db
    w_init = np.add(w_lo, np.multiply(w_pos, w_db))
    size = u(wh["size_dist"])
    draws = _draw_profiles(waterdraw_path, n, num_timesteps // (24 * dt) + 1, size)

    hems = {"horizon": home["hems"]["prediction_horizon"], "hourly_agg_steps": dt,
            "sub_subhourly_steps": home["hems"]["sub_subhourly_steps"],
            "solver": home["hems"]["solver"], "discount_factor": home["hems"]["discount_factor"]}
    count = {"pv_battery": com["homes_pv_battery"], "pv_only": com["homes_pv"],
             "battery_only": com["homes_battery"]}
    count["base"] = n - count["battery_only"] - count["pv_only"] - count["pv_battery"]
    bat, pv = home.get("battery"), home.get("pv")
    homes = []
    for typ in TYPES:
        for _ in range(int(count[typ])):
            i = len(homes)
            suffix = "".join(random.choices(string.ascii_uppercase + string.digits, k=5))
            rec = {"name": first_name() + "-" + suffix, "type": typ,
                   "hvac": {"r": r[i], "c": c[i], "p_c": p_c[i], "p_h": p_h[i], "temp_in_min": t_lo[i],
                            "temp_in_max": t_hi[i], "temp_in_sp": sp[i], "temp_in_init": t_init[i]},
                   "wh": {"r": w_r[i], "p": w_p[i], "temp_wh_min": w_lo[i], "temp_wh_max": w_hi[i],
                          "temp_wh_sp": w_sp[i], "temp_wh_init": w_init[i], "tank_size": size[i],
                          "draw_sizes": draws[i]},
                   "hems": hems}
            if "battery" in typ:
                rec["battery"] = {k: np.random.uniform(lo, hi) for k, (lo, hi) in (
                    ("max_rate", bat["max_rate"]), ("capacity", bat["capacity"]),
                    ("capacity_lower", bat["lower_bound"]), ("capacity_upper", bat["upper_bound"]),
                    ("ch_eff", bat["charge_eff"]), ("disch_eff", bat["discharge_eff"]),
                    ("e_batt_init", (bat["lower_bound"][1], bat["upper_bound"][0])))}
            if "pv" in typ:
                rec["pv"] = {"area": np.random.uniform(*pv["area"]), "eff": np.random.uniform(*pv["efficiency"])}
            homes.append(rec)
    return homes


def check_home_counts(homes, cfg):
    """aggregator.py:235-253 (`_check_home_configs`)."""
    com = cfg["community"]
    n = {t: sum(1 for h in homes if h["type"] == t) for t in TYPES}
    want = {"base": com["total_number_homes"] - com["homes_battery"] - com["homes_pv"] - com["homes_pv_battery"],
            "pv_battery": com["homes_pv_battery"], "pv_only": com["homes_pv"],
            "battery_only": com["homes_battery"]}
    for t in ("base", "pv_battery", "pv_only", "battery_only"):
        if n[t] != want[t]:
            raise ConfigError(f"Incorrect number of {t} homes.")


def max_load(home):
    """`MPCCalc.max_load` (mpc_calc.py:148, 159-162, 191): the home's largest step load."""
    S = max(1, int(home["hems"]["sub_subhourly_steps"]))
    return (max(float(home["hvac"]["p_c"]) / S, float(home["hvac"]["p_h"]) / S) + float(home["wh"]["p"]) / S) * S
