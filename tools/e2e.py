#!/usr/bin/env python3
"""End-to-end simulation wall time of the drop-in runner (missing 1).

Times `dragg_amd.runner.Aggregator().run()` -- what `python -m dragg.main` does in the reference
(aggregator.py:941-970): config.toml + NSRDB weather pipeline, `create_homes` (legacy-RNG draw order),
upload to the GPU, the run_rbo_mpc step loop, the history gather and the results.json / Summary writer
(aggregator.py:273-587, 757-854) -- on synthetic NSRDB-format data of the reference's file formats
(no reference file is read).  Prints one JSON line: the total wall time, the runner's phase breakdown
(`Aggregator.timings`) and the host share against the device step loop.

    python tools/e2e.py --homes 10000 --horizon-hours 6      # BASELINE north star: 10k x 24 h, H = 24
    python tools/e2e.py --homes 10000 --horizon-hours 12     # configs[2]: H = 48
"""
import argparse
import json
import math
import os
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIG = """[community]
total_number_homes = {n}
homes_battery = {batt}
homes_pv = {pv}
homes_pv_battery = {pvb}
overwrite_existing = true
house_p_avg = 1.2

[simulation]
start_datetime = "{start}"
end_datetime = "{end}"
random_seed = 12
n_nodes = 4
load_zone = "LZ_HOUSTON"
check_type = "all"
run_rbo_mpc = true
checkpoint_interval = "{checkpoint}"
named_version = "e2e"

[agg]
base_price = 0.07
subhourly_steps = {dt}
tou_enabled = true
spp_enabled = false

[agg.rl]
action_horizon = {horizon}
forecast_horizon = 1
prev_timesteps = 12
max_rp = 0.02

[home.hvac]
r_dist = [ 6.8, 9.199999999999999,]
c_dist = [ 4.25, 5.75,]
p_cool_dist = [ 3.5, 3.5,]
p_heat_dist = [ 3.5, 3.5,]
temp_sp_dist = [ 18, 22,]
temp_deadband_dist = [ 2, 3,]

[home.wh]
r_dist = [ 18.7, 25.3,]
p_dist = [ 2.5, 2.5,]
sp_dist = [ 45.5, 48.5,]
deadband_dist = [ 9, 12,]
size_dist = [ 200, 300,]
waterdraw_file = 'waterdraw_profiles.csv'

[home.battery]
max_rate = [3,5]
capacity = [9.0,13.5]
lower_bound = [ 0.01, 0.15]
upper_bound = [ 0.85, 0.99]
charge_eff = [0.85, 0.95]
discharge_eff = [0.97, 0.99]

[home.pv]
area = [20, 32]
efficiency = [0.15, 0.2]

[home.hems]
prediction_horizon = {horizon}
sub_subhourly_steps = 6
discount_factor = 0.92
solver = "GLPK_MI"

[agg.tou]
shoulder_times = [ 9, 21,]
shoulder_price = 0.09
peak_times = [ 14, 18,]
peak_price = 0.13
"""


def write_data(root, days, month, n_profiles=100, seed=3):
    """NSRDB-format half-hourly weather (the month's climate, community.CLIMATE) and a water-draw
    profile file of the reference's format (minute rows, one column per profile, 2 days)."""
    from dragg_amd.community import CLIMATE, half_hourly_weather
    t_mean, t_amp, ghi_peak, rise, set_ = CLIMATE[month]
    oat, ghi = half_hourly_weather(days, seed=seed, t_mean=t_mean, t_amp=t_amp, ghi_peak=ghi_peak, sun=(rise, set_))
    rows = []
    for k in range(days * 48):
        day, hh = divmod(k, 48)
        rows.append(f"2015,{month},{day + 1},{hh // 2},{30 * (hh % 2)},{ghi[k]},60.0,{oat[k]},1015.0")
    with open(os.path.join(root, "nsrdb.csv"), "w") as f:
        f.write("Source,Location ID\nNSRDB,0\nYear,Month,Day,Hour,Minute,GHI,Relative Humidity,Temperature,Pressure\n")
        f.write("\n".join(rows) + "\n")
    rng = np.random.default_rng(seed)
    mins = 2 * 24 * 60
    flow = np.where(rng.random((mins, n_profiles)) < 0.03, 3.78 * rng.integers(1, 4, (mins, n_profiles)), 0.0)
    ts = np.datetime64("2020-01-01T00:00") + np.arange(mins).astype("timedelta64[m]")
    with open(os.path.join(root, "waterdraw_profiles.csv"), "w") as f:
        f.write("," + ",".join(f"Flow_{j}" for j in range(n_profiles)) + "\n")
        for i in range(mins):
            f.write(str(ts[i]).replace("T", " ") + ":00," + ",".join(f"{v:.2f}" for v in flow[i]) + "\n")


# (action_horizon = the prediction horizon: the redis reward_price list is action_horizon * dt long, and
# the reference's MPCCalc needs it of length 1 or >= H = horizon * dt, mpc_calc.py:353)


def write_config(data, a, seed):
    n = a.homes
    mix = dict(batt=n // 5, pv=n // 5, pvb=n // 5)
    start = f"2015-{a.month:02d}-01 00"
    end = f"2015-{a.month:02d}-{1 + a.hours // 24:02d} {a.hours % 24:02d}"
    with open(os.path.join(data, "config.toml"), "w") as f:
        f.write(CONFIG.format(n=n, start=start, end=end, checkpoint=a.checkpoint, dt=a.dt, horizon=a.horizon_hours,
                              **mix).replace("random_seed = 12", f"random_seed = {seed}"))
    return mix


def completable_community(data, outs, a):
    """The reference raises KeyError at t = 1 when a battery home's t = 0 solve fails (mpc_calc.py:280-289);
    at 10k homes some battery home always does (the season draw keyed by the seed: 16 seeds tried in January
    at H = 24, round 6).  So, untimed, as bench.py does: the runner's own pipeline and generator
    (create_homes), then t = 0 on the GPU with the runner's environment and each failing battery home
    swapped with a home without a battery (community.reference_completable), written as the run's
    all_homes-N-config.json; the timed run loads it (overwrite_existing = false, aggregator.py:263-271).
    -> (seconds of create_homes, battery-home swaps)"""
    from dragg_amd import inputs as I
    from dragg_amd import results as R
    from dragg_amd.community import reference_completable
    from dragg_amd.runner import Aggregator
    agg = Aggregator(data_dir=data, outputs_dir=outs)
    agg.flush()
    t0 = time.perf_counter()
    agg.get_homes()
    t_create = agg.timings.get("create_homes", time.perf_counter() - t0)
    col = lambda c: agg.all_data[c].to_numpy(dtype=float)  # noqa: E731
    homes, swaps = reference_completable(agg.all_homes, col("OAT"), col("GHI"), col("tou"),
                                         int(agg.config["simulation"]["random_seed"]),
                                         reward_price=list(agg.reward_price), start_index=agg.start_hour_index)
    I.check_home_counts(homes, agg.config)
    R.write_home_configs(outs, homes, len(homes))
    return t_create, swaps


def use_reference_writer():
    """The reference's writer in place of dragg_amd.results' (the same bytes, json.dump's own speed)."""
    from dragg_amd import results as R

    def results_json(rdir, case, all_homes, checked, hist, summary_, cache=None):
        c = R.new_collected(all_homes)
        R.append_history(c, checked, hist)
        c["Summary"] = summary_
        os.makedirs(os.path.join(rdir, case), exist_ok=True)
        path = os.path.join(rdir, case, "results.json")
        with open(path, "w+") as f:
            json.dump(c, f, indent=4)
        return path

    def home_configs(outputs_dir, homes, n_homes):
        path = os.path.join(outputs_dir, f"all_homes-{n_homes}-config.json")
        with open(path, "w+") as f:
            json.dump(homes, f, indent=4)
        return path
    R.write_results_history = results_json
    R.write_home_configs = home_configs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--homes", type=int, default=10000)
    ap.add_argument("--horizon-hours", type=int, default=6)
    ap.add_argument("--hours", type=int, default=24, help="simulated hours")
    ap.add_argument("--dt", type=int, default=4)
    ap.add_argument("--month", type=int, default=7, choices=[1, 4, 7, 10])
    ap.add_argument("--checkpoint", default="daily", choices=["hourly", "daily", "weekly"])
    ap.add_argument("--workdir", default=None, help="data and outputs here (default: a temporary directory)")
    ap.add_argument("--keep", action="store_true")
    ap.add_argument("--out", default=None, help="also write the JSON line to this file")
    ap.add_argument("--seed", type=int, default=12, help="simulation.random_seed")
    ap.add_argument("--reference-writer", action="store_true",
                    help="write results.json and all_homes-N-config.json with json.dump(..., indent=4) as the "
                         "reference does (aggregator.py:839-854), for the before / after of the output phase")
    a = ap.parse_args()
    n = a.homes
    days = math.ceil((a.hours + a.horizon_hours + 2) / 24) + 1
    work = a.workdir or tempfile.mkdtemp(prefix="dragg_e2e_")
    data, outs = os.path.join(work, "data"), os.path.join(work, "outputs")
    os.makedirs(data, exist_ok=True)
    write_data(data, days, a.month)
    import torch
    from dragg_amd.runner import Aggregator
    torch.cuda.init()
    torch.zeros(1, device="cuda")                 # (the CUDA context, outside the timed run)
    seed = a.seed if a.seed is not None else 12
    mix = write_config(data, a, seed)
    t_create, swaps = completable_community(data, outs, a)
    with open(os.path.join(data, "config.toml")) as f:
        txt = f.read().replace("overwrite_existing = true", "overwrite_existing = false")
    with open(os.path.join(data, "config.toml"), "w") as f:
        f.write(txt)
    if a.reference_writer:
        use_reference_writer()
    t0 = time.perf_counter()
    agg = Aggregator(data_dir=data, outputs_dir=outs)
    path = agg.run()
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    ph = {k: round(v, 4) for k, v in agg.timings.items()}
    loop = agg.timings.get("step_loop", 0.0)
    size = os.path.getsize(path)
    out = {
        "metric": "end-to-end simulation wall time (Aggregator().run(), run_rbo_mpc)",
        "value": total, "unit": "s", "higher_is_better": False,
        "config": {"homes": n, "steps": agg.num_timesteps, "H": a.horizon_hours * a.dt, "dt": a.dt,
                   "month": a.month, "checkpoint_interval": a.checkpoint, "homes_mix": mix, "random_seed": seed},
        "phases_s": ph,
        "create_homes_generator_s": t_create,
        "community": {"battery_home_swaps": swaps,
                      "note": "the community create_homes draws (legacy-RNG order), with each battery home whose t = 0 "
                              "solve fails swapped with a home without a battery (the reference raises KeyError at "
                              "t = 1 otherwise), written as all_homes-N-config.json before the timed run, which "
                              "loads it (phase create_homes); the generator itself took create_homes_generator_s"},
        "phase_note": "checkpoints = the in-loop check_errors + write_outputs + save_state (its results.json "
                      "write is also counted in history_gather / results_build / results_write); step_loop = the "
                      "steps' launches and device time without the checkpoint writes",
        "device_loop_s": loop, "host_s": total - loop, "host_share": (total - loop) / total,
        "ms_per_step_in_loop": loop / agg.num_timesteps * 1e3,
        "solves_per_s_end_to_end": n * agg.num_timesteps / total,
        "solve_paths": getattr(agg, "solve_paths", None),
        "results_json_bytes": size, "results_json_homes": len(agg.all_homes),
        "data": "synthetic NSRDB-format weather and water-draw profile files (the reference's formats)",
        "writer": "json.dump(indent=4), the reference's" if a.reference_writer else
                  "dragg_amd.results (libdragg_results.so; the same bytes)",
    }
    line = json.dumps(out)
    print(line)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(line + "\n")
    if not a.keep and not a.workdir:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
