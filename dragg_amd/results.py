"""Outputs of a dragg run: collected data, Summary, results.json, the community file.

SURVEY.md §8 row F1.  During a run the per-step hash fields stay on the GPU
(`DeviceAggregator.hist`, [T][19][N]); these functions turn them into the reference's files:

* `new_collected`       aggregator.py:589-615  `reset_collected_data` (key order kept)
* `append_history`      aggregator.py:737-750  `collect_data` (a field absent from the hash is
                        skipped; a field a fallback step did not rewrite is appended again,
                        as the reference re-reads the stale redis value)
* `aggregate_loads`     aggregator.py:748-751  np.sum over the homes' p_grid_opt, in home order
* `summary`             aggregator.py:783-816  `summarize_baseline` (incl. the trailing comma
                        that makes TOU / SPP a one-element tuple, written as [[...]])
* `run_dir`             aggregator.py:818-829  `set_run_dir`
* `write_results`       aggregator.py:831-844  `write_outputs`
* `write_home_configs`  aggregator.py:846-854
* `checkpoint_interval` aggregator.py:949-955
"""
import json
import os

import numpy as np

from . import _lib as L

BASE_KEYS = ["p_grid_opt", "forecast_p_grid_opt", "p_load_opt", "temp_in_opt", "temp_wh_opt",
             "hvac_cool_on_opt", "hvac_heat_on_opt", "wh_heat_on_opt", "cost_opt", "waterdraws",
             "correct_solve"]


def collect_keys(home_type):
    """The hash fields collect_data appends for a home type (aggregator.py:741-745)."""
    keys = list(BASE_KEYS)
    if "pv" in home_type:
        keys += ["p_pv_opt", "u_pv_curt_opt"]
    if "battery" in home_type:
        keys += ["p_batt_ch", "p_batt_disch", "e_batt_opt"]
    return keys


def new_collected(homes):
    """Per-home series, initial entries included (aggregator.py:589-615)."""
    out = {}
    for h in homes:
        d = {"type": h["type"], "temp_in_sp": h["hvac"]["temp_in_sp"], "temp_wh_sp": h["wh"]["temp_wh_sp"],
             "temp_in_opt": [h["hvac"]["temp_in_init"]], "temp_wh_opt": [h["wh"]["temp_wh_init"]]}
        for k in ("p_grid_opt", "forecast_p_grid_opt", "p_load_opt", "hvac_cool_on_opt", "hvac_heat_on_opt",
                  "wh_heat_on_opt", "cost_opt", "waterdraws", "correct_solve"):
            d[k] = []
        if "pv" in h["type"]:
            d["p_pv_opt"] = []
            d["u_pv_curt_opt"] = []
        if "battery" in h["type"]:
            d["e_batt_opt"] = [h["battery"]["e_batt_init"]]
            d["p_batt_ch"] = []
            d["p_batt_disch"] = []
        out[h["name"]] = d
    return out


def append_history(collected, homes, hist):
    """Append steps of the hash history `hist` [T][NVAL][len(homes)] (NaN = field absent)
    to the homes' series, as collect_data does after each step."""
    hist = np.asarray(hist)
    for i, h in enumerate(homes):
        d = collected[h["name"]]
        for k in collect_keys(h["type"]):
            col = hist[:, L.K[k], i]
            d[k].extend(float(v) for v in col[~np.isnan(col)])
    return collected


def aggregate_loads(hist):
    """Per-step community load: np.sum of the homes' p_grid_opt in home order
    (aggregator.py:748-751), from the hash history [T][NVAL][N]."""
    p = np.asarray(hist)[:, L.K["p_grid_opt"], :]
    return [np.sum([float(v) for v in row]) for row in p]


def summary(case, start, end, solve_time, horizon, num_homes, agg_loads, oat, ghi, rps, sps,
            tou=None, spp=None):
    """The results' "Summary" entry (aggregator.py:795-816)."""
    s = {"case": case, "start_datetime": start.strftime("%Y-%m-%d %H"),
         "end_datetime": end.strftime("%Y-%m-%d %H"), "solve_time": solve_time, "horizon": horizon,
         "num_homes": num_homes, "p_max_aggregate": max(agg_loads), "p_grid_aggregate": list(agg_loads),
         "OAT": list(oat), "GHI": list(ghi), "RP": list(rps), "p_grid_setpoint": list(sps)}
    if spp is not None:
        s["SPP"] = (list(spp),)
    else:
        s["TOU"] = (list(tou),)
    return s


def run_dir(outputs_dir, start, end, check_type, n_homes, horizon, dt_interval, sub_steps, solver, version):
    """outputs/<start>_<end>/<check>-homes_<N>-horizon_<h>-interval_<m>-<m//S>-solver_<s>/version-<v>
    (aggregator.py:818-829)."""
    date = f"{start.strftime('%Y-%m-%dT%H')}_{end.strftime('%Y-%m-%dT%H')}"
    mpc = (f"{check_type}-homes_{n_homes}-horizon_{horizon}-interval_{dt_interval}-"
           f"{dt_interval // sub_steps}-solver_{solver}")
    return os.path.join(outputs_dir, date, mpc, f"version-{version}")


def write_results(rdir, case, collected):
    """<run_dir>/<case>/results.json, indent 4 (aggregator.py:839-844)."""
    case_dir = os.path.join(rdir, case)
    os.makedirs(case_dir, exist_ok=True)
    path = os.path.join(case_dir, "results.json")
    with open(path, "w+") as f:
        json.dump(collected, f, indent=4)
    return path


def write_home_configs(outputs_dir, homes, n_homes):
    """outputs/all_homes-<N>-config.json (aggregator.py:846-854)."""
    path = os.path.join(outputs_dir, f"all_homes-{n_homes}-config.json")
    with open(path, "w+") as f:
        json.dump(homes, f, indent=4)
    return path


def checkpoint_interval(setting, dt):
    """Steps between checkpoint writes (aggregator.py:949-955)."""
    return {"hourly": dt, "daily": dt * 24, "weekly": dt * 24 * 7}.get(setting, 500)
