"""The drop-in Aggregator (dragg_amd.runner) end to end.

CPU: the host side of a run configured like a golden scenario (config -> weather / TOU ->
start index -> community -> all_homes file, run directory) against what the reference's own
Aggregator produced; needs the reference's data files in place (skips otherwise).
GPU: a whole run on synthetic NSRDB-format weather and water-draw files (nothing from the
reference is read): results.json layout, series lengths (the reference's
check_baseline_vals rule), Summary sums, checkpoints, and identity with a DeviceAggregator
driven directly."""
import json
import os

import numpy as np
import pytest

from tests import fixtures as F
from tests.test_inputs import DATA, needs_data, _cfg


def _write_config(path, params):
    with open(path, "w") as f:
        f.write(F.config_text(params))


@needs_data
@pytest.mark.parametrize("name", ["c1_h24", "spring_dt1", "negprice_dt2"])
def test_runner_host_side_matches_reference(tmp_path, name):
    from dragg_amd.runner import Aggregator
    d = F.load(name)
    data = tmp_path / "data"
    data.mkdir()
    _write_config(data / "config.toml", d["params"])
    for f in ("nsrdb.csv", "waterdraw_profiles.csv"):
        os.symlink(os.path.join(DATA, f), data / f)
    a = Aggregator(data_dir=str(data), outputs_dir=str(tmp_path / "outputs"))
    assert a.num_timesteps == d["env"]["num_timesteps"]
    a.flush()
    assert a.start_hour_index == d["env"]["start_hour_index"]
    assert len(a.reward_price) == d["params"]["action_horizon"] * d["params"]["dt"]
    a.get_homes()
    assert json.loads(json.dumps(a.all_homes)) == d["homes"]
    with open(tmp_path / "outputs" / f"all_homes-{d['params']['n']}-config.json") as f:
        assert json.load(f) == d["homes"]
    cfg = _cfg(d["params"])
    assert a.max_poss_load == pytest.approx(sum(
        (max(h["hvac"]["p_c"], h["hvac"]["p_h"]) / 6 + h["wh"]["p"] / 6) * 6 for h in d["homes"]))
    assert cfg["simulation"]["check_type"] == a.check_type


# ------------------------------------------------------------------------------- GPU
def _synthetic_data(root, days=3, n_profiles=4, seed=0):
    """NSRDB-format weather and minute-resolution water-draw profiles (synthetic)."""
    from dragg_amd.community import half_hourly_weather
    oat, ghi = half_hourly_weather(days, seed=seed)
    rows = []
    for k in range(days * 48):
        day, hh = divmod(k, 48)
        rows.append(f"2015,1,{day + 1},{hh // 2},{30 * (hh % 2)},{ghi[k]},90.0,{oat[k]},1020.0")
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


@pytest.mark.gpu
def test_runner_end_to_end(gpu, tmp_path):
    import torch
    from dragg_amd.aggregator import DeviceAggregator
    from dragg_amd.runner import Aggregator
    data = tmp_path / "data"
    data.mkdir()
    _synthetic_data(str(data))
    params = dict(n=12, batt=3, pv=3, pvb=2, start="2015-01-01 00", end="2015-01-01 12", dt=4, horizon=6,
                  action_horizon=6, seed=21)
    _write_config(data / "config.toml", params)
    with open(data / "config.toml") as f:
        txt = f.read().replace('checkpoint_interval = "daily"', 'checkpoint_interval = "hourly"')
    with open(data / "config.toml", "w") as f:
        f.write(txt)
    a = Aggregator(data_dir=str(data), outputs_dir=str(tmp_path / "outputs"))
    path = a.run()
    with open(path) as f:
        res = json.load(f)
    T = a.num_timesteps
    assert T == 48
    names = [h["name"] for h in a.all_homes]
    assert list(res) == names + ["Summary"]
    for h in a.all_homes:
        d = res[h["name"]]
        for k, v in d.items():
            if k in ("temp_in_opt", "temp_wh_opt", "e_batt_opt"):
                assert len(v) == T + 1, (h["name"], k)
            elif isinstance(v, list):
                assert len(v) == T, (h["name"], k)
    s = res["Summary"]
    assert len(s["p_grid_aggregate"]) == T and len(s["OAT"]) == T and len(s["TOU"]) == 1 and len(s["TOU"][0]) == T
    for t in range(T):
        assert s["p_grid_aggregate"][t] == np.sum([res[n]["p_grid_opt"][t] for n in names])
    # the same community driven directly gives the same per-home series
    col = lambda c: a.all_data[c].to_numpy(dtype=float)  # noqa: E731
    dev = DeviceAggregator(a.all_homes, col("OAT"), col("GHI"), col("tou"), a.start_hour_index, T,
                           reward_price=a.reward_price, seed=params["seed"])
    for _ in range(T):
        dev.run_iteration()
        dev.collect_data()
    torch.cuda.synchronize()
    direct = dev.collected_data()
    for n in names:
        assert direct[n] == res[n], n


@pytest.mark.gpu
def test_runner_resume_from_checkpoint(gpu, tmp_path):
    """A run stopped after a checkpoint and resumed from the saved device state writes the
    results.json of an uninterrupted run, value for value (the noise stream is keyed by step)."""
    from dragg_amd.runner import Aggregator
    data = tmp_path / "data"
    data.mkdir()
    _synthetic_data(str(data))
    params = dict(n=12, batt=3, pv=3, pvb=2, start="2015-01-01 00", end="2015-01-01 06", dt=4, horizon=6,
                  action_horizon=6, seed=23)
    _write_config(data / "config.toml", params)
    with open(data / "config.toml") as f:
        txt = f.read().replace('checkpoint_interval = "daily"', 'checkpoint_interval = "hourly"')
    with open(data / "config.toml", "w") as f:
        f.write(txt)
    full = Aggregator(data_dir=str(data), outputs_dir=str(tmp_path / "full")).run()
    a = Aggregator(data_dir=str(data), outputs_dir=str(tmp_path / "split"))
    assert a.run(stop_after=8) is None                # "crash" after the second hourly checkpoint
    assert os.path.isfile(a.state_path())
    b = Aggregator(data_dir=str(data), outputs_dir=str(tmp_path / "split"))
    path = b.run(resume=True)
    with open(full) as f:
        want = json.load(f)
    with open(path) as f:
        got = json.load(f)
    for k in want:
        if k == "Summary":
            for s in want[k]:
                if s != "solve_time":
                    assert got[k][s] == want[k][s], s
        else:
            assert got[k] == want[k], k
