"""Host input pipeline (dragg_amd.inputs) against what the
reference produced for every golden scenario (tests/golden/make_golden.py ran the
reference's own Aggregator): the community of `create_homes`, the upsampled weather, the
TOU window after `join_data`'s forward fill, the start index and the run mask's series.

The inputs are the reference's own data files (NSRDB weather, water-draw profiles), read in
place (DRAGG_REFERENCE_DATA, default /root/reference/dragg/data); they are not copied into
this repository, so these CPU tests skip where that directory is absent."""
import json
import math
import os

import numpy as np
import pytest

from tests import fixtures as F

DATA = os.environ.get("DRAGG_REFERENCE_DATA", "/root/reference/dragg/data")
NSRDB = os.path.join(DATA, "nsrdb.csv")
DRAWS = os.path.join(DATA, "waterdraw_profiles.csv")
needs_data = pytest.mark.skipif(not (os.path.exists(NSRDB) and os.path.exists(DRAWS)),
                                reason="reference data files not present")


def _cfg(params):
    import tomli
    return tomli.loads(F.config_text(params))


def _window(cfg):
    from dragg_amd import inputs as I
    start, end, hours = I.run_window(cfg)
    dt = int(cfg["agg"]["subhourly_steps"])
    return start, end, hours, dt, int(math.ceil(hours * dt))


@needs_data
@pytest.mark.parametrize("name", F.scenarios())
def test_create_homes_matches_reference(name):
    """Every parameter, water-draw list and name of the community, bit-exact."""
    from dragg_amd import inputs as I
    d = F.load(name)
    cfg = _cfg(d["params"])
    _, _, _, dt, nts = _window(cfg)
    homes = I.create_homes(cfg, nts, dt, DRAWS)
    I.check_home_counts(homes, cfg)
    assert json.loads(json.dumps(homes)) == d["homes"]


@needs_data
@pytest.mark.parametrize("name", F.scenarios())
def test_environment_matches_reference(name):
    """Weather rows per dt, the TOU list with its quirks, the start index and the run mask."""
    from dragg_amd import inputs as I
    d = F.load(name)
    cfg = _cfg(d["params"])
    start, end, hours, dt, nts = _window(cfg)
    env = d["env"]
    assert nts == env["num_timesteps"]
    all_data, mask = I.join_series(I.load_weather(NSRDB, dt), I.tou_prices(start, hours, cfg["agg"]), start, end)
    I.check_series(all_data, start, end, cfg["home"]["hems"]["prediction_horizon"])
    n = len(env["oat"])
    assert all_data["OAT"].values[:n].tolist() == env["oat"]
    assert all_data["GHI"].values[:n].tolist() == env["ghi"]
    shi = I.start_hour_index(all_data, start)
    assert shi == env["start_hour_index"]
    tw = all_data["tou"].values[shi:shi + nts + 60 * dt]
    np.testing.assert_array_equal(tw, np.array(env["tou_window"], dtype=float))
    summ = d["results"]["Summary"]
    assert all_data.loc[mask, "OAT"].values.tolist() == summ["OAT"]
    assert all_data.loc[mask, "GHI"].values.tolist() == summ["GHI"]
    assert [all_data.loc[mask, "tou"].values.tolist()] == summ["TOU"]


def test_tou_quirk_and_errors():
    """The peak window is overwritten by the shoulder one (aggregator.py:214-215); bad
    datetimes and a window past the data are configuration errors (sys.exit in the reference)."""
    from datetime import datetime
    import pandas as pd
    from dragg_amd import inputs as I
    agg = {"base_price": 0.07, "tou_enabled": True,
           "tou": {"shoulder_times": [9, 21], "shoulder_price": 0.09, "peak_times": [14, 18], "peak_price": 0.13}}
    t = I.tou_prices(datetime(2015, 1, 1), 24, agg)["tou"].to_numpy()
    assert t[8] == 0.07 and t[9] == 0.09 and t[15] == 0.09 and t[20] == 0.09 and t[21] == 0.07
    assert I.tou_prices(datetime(2015, 1, 1), 5, dict(agg, tou_enabled=False))["tou"].tolist() == [0.07] * 5
    with pytest.raises(I.ConfigError):
        I.run_window({"simulation": {"start_datetime": "2015-01-01", "end_datetime": "2015-01-02 00"}})
    idx = pd.date_range("2015-01-01", periods=48, freq="h")
    df = pd.DataFrame({"OAT": np.zeros(48)}, index=idx)
    with pytest.raises(I.ConfigError):
        I.check_series(df, datetime(2015, 1, 1), datetime(2015, 1, 2, 20), 6)
    I.check_series(df, datetime(2015, 1, 1), datetime(2015, 1, 2, 12), 6)
