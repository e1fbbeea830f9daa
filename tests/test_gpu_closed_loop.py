"""Whole closed-loop runs on the GPU against the reference's results.json.

Each golden scenario is replayed end to end on the device: the same community, the same
weather / price windows (rebuilt from the per-solve records), the same reward price and the
noise the reference drew at every (home, step), all `num_timesteps` steps chained through
the device-resident hash.  The collected series must match the reference's results.json.

Where the reference's solver returned a HiGHS incumbent (c1_h24: 5 s MILP limit, §2 of
DESIGN.md) our exact optimum can differ and the closed loop then departs from the
reference's path for that home; those homes are counted and bounded, the rest must match."""
import numpy as np
import pytest

from tests import fixtures as F

pytestmark = pytest.mark.gpu

# scenario -> homes whose closed loop may depart from the reference (HiGHS incumbents)
ALLOWED_DEPARTURES = {"c1_h24": 20}


def _windows(d):
    H = max(len(r["noise"]) for r in d["records"])
    T = d["env"]["num_timesteps"]
    oat, ghi = np.full(T + H + 1, np.nan), np.full(T + H + 1, np.nan)
    for r in d["records"]:
        t = r["t"]
        for w, k in ((oat, "oat"), (ghi, "ghi")):
            v = np.asarray(r[k], dtype=float)
            seg = w[t:t + len(v)]
            known = ~np.isnan(seg)
            assert np.array_equal(seg[known], v[known])
            w[t:t + len(v)] = v
    return H, T, oat, ghi, np.asarray(d["env"]["tou_window"], dtype=float)


@pytest.mark.parametrize("name", F.scenarios())
def test_closed_loop_matches_reference_results(gpu, name):
    import torch
    from dragg_amd.aggregator import DeviceAggregator
    from dragg_amd import results as R
    d = F.load(name)
    homes = d["homes"]
    H, T, oat, ghi, tou = _windows(d)
    p = d["params"]
    rp = p.get("rp") or [0.0] * (p["action_horizon"] * p["dt"])
    noise = {(r["t"], r["name"]): r["noise"] for r in d["records"]}
    dev = DeviceAggregator(homes, oat, ghi, tou, 0, T, reward_price=rp, seed=p["seed"])
    for t in range(T):
        z = np.stack([noise[(t, h["name"])] for h in homes], axis=1)
        dev.run_iteration(torch.tensor(z))
        dev.collect_data()
    torch.cuda.synchronize()
    got = dev.collected_data()
    ref = d["results"]
    departed = []
    for h in homes:
        a, b = got[h["name"]], ref[h["name"]]
        assert list(a) == list(b)
        ok = True
        for k in b:
            if isinstance(b[k], list):
                assert len(a[k]) == len(b[k]), (h["name"], k)
                if not np.allclose(a[k], b[k], rtol=1e-6, atol=1e-6):
                    ok = False
        if not ok:
            departed.append(h["name"])
    loads = R.aggregate_loads(dev.hist[:T].cpu().numpy())
    close = np.isclose(loads, ref["Summary"]["p_grid_aggregate"], rtol=1e-6, atol=1e-6)
    print(f"{name}: {len(homes) - len(departed)}/{len(homes)} homes follow the reference's closed loop "
          f"over {T} steps; community load equal (1e-6) at {int(close.sum())}/{T} steps")
    assert len(departed) <= ALLOWED_DEPARTURES.get(name, 0), departed
