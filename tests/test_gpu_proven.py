"""The headline configuration against PROVEN MILP optima (BASELINE.json configs[2]: 15-min
steps, 12 h horizon, H = 48, July).

tests/golden/proven/h48_july.json.gz (tests/golden/make_proven_h48.py) holds solves of homes of
the bench's 10,000-home synthetic community -- every home type, t = 0 and t = 1 -- with the
reference's MILP (`mpc_calc.py:291-451`, assembled by the oracle in the reference's row order)
solved by HiGHS to proven optimality (mip_rel_gap 0).  The kernel (int_mode round, through the
C ABI) must reach the same status and the same objective.  The bound 1e-6 relative is HiGHS's
own slack: its objective is c.x of a solution whose continuous columns meet the constraints to
its ~1e-7 feasibility tolerance.
"""
import gzip
import json
import os

import numpy as np
import pytest

from tests import fixtures as F

pytestmark = pytest.mark.gpu

PROVEN = os.path.join(F.GOLDEN, "proven", "h48_july.json.gz")


def _load():
    with gzip.open(PROVEN, "rt") as f:
        return json.load(f)


_RES = {}


def _solved():
    if "r" not in _RES:
        import torch
        from dragg_amd import _lib as L
        from dragg_amd.mpc import MPCBatch
        d = _load()
        recs = d["records"]
        homes, ex = F.explicit_inputs(d, recs)
        b = MPCBatch(homes, int_mode="round")
        fc, vals = F.prev_hash_arrays(recs, b.H, L.FC_KEYS, L.VAL_KEYS)
        b.fc.copy_(torch.tensor(fc))
        b.vals.copy_(torch.tensor(vals))
        b.solve_explicit(**ex)
        torch.cuda.synchronize()
        _RES["r"] = (d, dict(status=b.status.cpu().numpy(), obj=b.obj.cpu().numpy(), fc=b.fc.cpu().numpy(),
                             path=b.int_path.cpu().numpy() & L.PATH_APPROX_MASK, S=b.S, H=b.H))
    return _RES["r"]


def test_h48_status_and_objective_equal_proven_optimum(gpu):
    from dragg_amd import _lib as L
    d, res = _solved()
    assert res["H"] == 48
    gaps, types = [], {}
    for i, r in enumerate(d["records"]):
        assert r["milp_status"] in (0, 2), (i, r["milp_status"])          # proven or proven infeasible
        ours_ok = res["status"][i] == L.ST_OPTIMAL
        assert ours_ok == (r["status"] == "optimal"), (i, r["name"], r["t"], L.STATUS_NAMES[res["status"][i]])
        if not ours_ok:
            continue
        assert res["path"][i] == 0, (i, "exact DP fell back")
        gap = (res["obj"][i] - r["milp_obj"]) / max(1.0, abs(r["milp_obj"]))
        assert abs(gap) <= 1e-6, (i, r["name"], r["t"], r["type"], res["obj"][i], r["milp_obj"])
        gaps.append(gap)
        types[r["type"]] = types.get(r["type"], 0) + 1
    gaps = np.abs(np.array(gaps))
    print(f"H = 48 July: {len(gaps)} proven optima {types}: |gap| max {gaps.max():.2e}, mean {gaps.mean():.2e}")


def test_h48_duty_schedules_vs_proven(gpu):
    """Where the kernel's duty schedule differs from HiGHS's, the two must cost the same (an
    alternative optimum); report how many are identical."""
    from dragg_amd import _lib as L
    d, res = _solved()
    S = res["S"]
    same = diff = 0
    for i, r in enumerate(d["records"]):
        if res["status"][i] != L.ST_OPTIMAL or r["milp_x"] is None:
            continue
        key = "hvac_heat_on" if r["season"] == "winter" else "hvac_cool_on"
        u_ref = np.rint(np.array(r["milp_x"][key])).astype(int)
        w_ref = np.rint(np.array(r["milp_x"]["wh_heat_on"])).astype(int)
        u = np.rint(res["fc"][L.FC_KEYS.index(key + "_opt"), :, i] * S).astype(int)
        w = np.rint(res["fc"][L.FC_KEYS.index("wh_heat_on_opt"), :, i] * S).astype(int)
        if np.array_equal(u, u_ref) and np.array_equal(w, w_ref):
            same += 1
            t_ref = np.array(r["milp_x"]["temp_in_ev"][1:])
            t = res["fc"][L.FC_KEYS.index("temp_in_ev_opt"), :, i]
            assert np.abs(t - t_ref).max() <= 1e-6, (i, np.abs(t - t_ref).max())
        else:
            diff += 1
    print(f"H = 48 July: duty schedules identical to HiGHS's on {same}, different (equal cost) on {diff}")
    assert same >= 0.9 * (same + diff)
