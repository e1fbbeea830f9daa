"""results.json assembly (dragg_amd.results) against the results.json the
reference wrote for every golden scenario.  The per-step redis hashes are rebuilt from the
fields the reference wrote at each step (the fixture records), laid out as the device hash
history [T][19][N] that DeviceAggregator keeps, and turned into the collected-data series and
the Summary: every series must equal the reference's, value for value."""
import json
from datetime import datetime

import numpy as np
import pytest

from tests import fixtures as F


def _history(d):
    """Hash history [T][NVAL][N] from the fields written at each step (HSET semantics: a field
    keeps its last written value; never written = NaN)."""
    from dragg_amd import _lib as L
    homes = d["homes"]
    col = {h["name"]: i for i, h in enumerate(homes)}
    T = d["env"]["num_timesteps"]
    hist = np.full((T, L.NVAL, len(homes)), np.nan)
    recs = sorted(d["records"], key=lambda r: (r["t"], col[r["name"]]))
    state = [dict() for _ in homes]
    by_t = {}
    for r in recs:
        by_t.setdefault(r["t"], []).append(r)
    for t in range(T):
        for r in by_t.get(t, []):
            state[col[r["name"]]].update({k: float(v) for k, v in r["optimal_vals"].items() if k in L.K})
        for i, s in enumerate(state):
            for k, v in s.items():
                hist[t, L.K[k], i] = v
    return hist


@pytest.mark.parametrize("name", F.scenarios())
def test_collected_series_match_reference(name):
    from dragg_amd import results as R
    d = F.load(name)
    if len({r["t"] for r in d["records"]}) != d["env"]["num_timesteps"]:
        pytest.skip("fixture does not record every step")
    hist = _history(d)
    got = R.append_history(R.new_collected(d["homes"]), d["homes"], hist)
    ref = d["results"]
    for h in d["homes"]:
        assert list(got[h["name"]]) == list(ref[h["name"]]), h["name"]          # key order too
        assert got[h["name"]] == ref[h["name"]], h["name"]
    loads = R.aggregate_loads(hist)
    assert loads == ref["Summary"]["p_grid_aggregate"]
    assert max(loads) == ref["Summary"]["p_max_aggregate"]


@pytest.mark.parametrize("name", F.scenarios())
def test_summary_layout(name):
    """Summary keys, order and values (solve_time aside), incl. TOU written as [[...]]."""
    from dragg_amd import results as R
    d = F.load(name)
    ref = d["results"]["Summary"]
    p = d["params"]
    s = R.summary("baseline", datetime.strptime(p["start"], "%Y-%m-%d %H"),
                  datetime.strptime(p["end"], "%Y-%m-%d %H"), ref["solve_time"], p["horizon"], p["n"],
                  ref["p_grid_aggregate"], ref["OAT"], ref["GHI"], [0.0] * len(ref["RP"]),
                  [0.0] * len(ref["p_grid_setpoint"]), tou=ref["TOU"][0])
    assert json.loads(json.dumps(s)) == ref
    assert list(s) == list(ref)


def test_run_dir_and_checkpoints(tmp_path):
    from dragg_amd import results as R
    rd = R.run_dir("outputs", datetime(2015, 1, 1), datetime(2015, 1, 2), "all", 20, 6, 15, 6, "GLPK_MI", "golden")
    assert rd == ("outputs/2015-01-01T00_2015-01-02T00/all-homes_20-horizon_6-interval_15-2-solver_GLPK_MI/"
                  "version-golden")
    assert [R.checkpoint_interval(s, 4) for s in ("hourly", "daily", "weekly", "never")] == [4, 96, 672, 500]
    path = R.write_results(str(tmp_path), "baseline", {"a": [1.0], "Summary": {"TOU": ([0.07],)}})
    with open(path) as f:
        assert json.load(f) == {"a": [1.0], "Summary": {"TOU": [[0.07]]}}
