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


# ------------------------------------------------------------------ the fast writer (libdragg_results.so)
def _fuzz(rng, d=0):
    r = rng.random()
    if d > 3 or r < 0.3:
        return rng.choice([1.5, -0.0, float("nan"), float("inf"), -float("inf"), 3, True, False, None, "aé\"x\n",
                           1e-7, 1e16, 12345678901234567.0, np.float64(0.1), [], {}, (1,), (2.5, 3.5), 5e-324])
    if r < 0.5:
        return [rng.uniform(-1e3, 1e3) * 10.0 ** rng.randint(-8, 20) for _ in range(rng.randint(0, 6))]
    if r < 0.7:
        return [_fuzz(rng, d + 1) for _ in range(rng.randint(0, 4))]
    if r < 0.8:
        return tuple(_fuzz(rng, d + 1) for _ in range(rng.randint(0, 3)))
    return {(rng.choice(["k", "é", "x y", 1, 2.5, True, None]) if rng.random() < 0.3 else f"k{i}"): _fuzz(rng, d + 1)
            for i in range(rng.randint(0, 4))}


def test_dump_json_is_json_dump_byte_for_byte(tmp_path):
    """dump_json / dumps_json write exactly what json.dump(obj, f, indent=4) writes (the reference's
    writer, aggregator.py:839-854): random nested documents with every JSON type, float subclasses,
    non-finite values, non-str keys, empty containers and tuples."""
    import random
    from dragg_amd import results as R
    rng = random.Random(7)
    for i in range(1500):
        o = _fuzz(rng)
        want = json.dumps(o, indent=4)
        assert R.dumps_json(o) == want
        if i % 50 == 0:
            R.dump_json(o, str(tmp_path / "x.json"))
            assert (tmp_path / "x.json").read_text() == want


def test_number_formatter_is_float_repr():
    """libdragg_results.so renders doubles as repr(float): random bit patterns, every magnitude,
    the repr rule's notation switches (decimal exponents -4 / 16), subnormals, signed zero."""
    from dragg_amd import results as R
    rng = np.random.default_rng(3)
    x = np.concatenate([rng.integers(0, 2 ** 64, 200_000, dtype=np.uint64).view(np.float64),
                        rng.standard_normal(100_000) * 10.0 ** rng.integers(-30, 30, 100_000),
                        np.array([0.0, -0.0, 1e16, 1e15, 9999999999999998.0, 1e-4, 1e-5, 0.0001, 0.00011,
                                  5e-324, 1.7976931348623157e308, np.nan, np.inf, -np.inf, 0.1, 100.0, 1e22])])
    got = bytes(R.format_series(x, [0], [x.size], ",")[0]).decode().split(",")
    want = [("NaN" if v != v else "Infinity" if v == float("inf") else "-Infinity" if v == -float("inf")
             else float.__repr__(v)) for v in x.tolist()]
    assert got == want


@pytest.mark.parametrize("T", [0, 1, 7])
def test_history_writer_is_json_dump_of_collected_data(tmp_path, T):
    """write_results_history writes the bytes json.dump(collected, indent=4) writes for the collected
    data of the same history (new_collected + append_history + Summary): absent fields (NaN) skipped,
    homes outside the checked set, all four home types."""
    from dragg_amd import _lib as L
    from dragg_amd import results as R
    from dragg_amd.community import synthetic_homes
    homes = synthetic_homes(23, seed=4)
    for h in homes:
        h["name"] = str(h["name"])
    checked = [h for i, h in enumerate(homes) if i % 5 != 3]
    rng = np.random.default_rng(T)
    hist = rng.standard_normal((T, L.NVAL, len(checked))) * 10.0 ** rng.integers(-6, 6, (T, L.NVAL, len(checked)))
    hist[rng.random(hist.shape) < 0.1] = np.nan
    summary = R.summary("baseline", datetime(2015, 1, 1), datetime(2015, 1, 2), 1.25, 6, len(homes),
                        [1.0 + t for t in range(max(T, 1))], [10.0] * T, [0.0] * T, [0.0] * T, [0.0] * T,
                        tou=[0.07] * T)
    path = R.write_results_history(str(tmp_path), "baseline", homes, checked, hist, summary)
    c = R.new_collected(homes)
    R.append_history(c, checked, hist)
    c["Summary"] = summary
    with open(path) as f:
        assert f.read() == json.dumps(c, indent=4)
    # a rewrite for the same history (the final write after the last checkpoint): Summary only, same bytes
    cache = {}
    R.write_results_history(str(tmp_path), "c", homes, checked, hist, summary, cache=cache)
    summary2 = dict(summary, solve_time=2.5)
    path = R.write_results_history(str(tmp_path), "c", homes, checked, hist, summary2, cache=cache)
    c["Summary"] = summary2
    with open(path) as f:
        assert f.read() == json.dumps(c, indent=4)
    # an int initial entry: json.dump writes it as an int -- the writer falls back to the generic path
    homes[0]["hvac"]["temp_in_init"] = 20
    path = R.write_results_history(str(tmp_path), "b2", homes, checked, hist, summary)
    c = R.new_collected(homes)
    R.append_history(c, checked, hist)
    c["Summary"] = summary
    with open(path) as f:
        assert f.read() == json.dumps(c, indent=4)
