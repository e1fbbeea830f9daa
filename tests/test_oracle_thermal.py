"""The exact thermal-chain checker (oracle/thermal.py) against enumeration and HiGHS.

CPU only.  The checker is what the GPU's integer DP is held to (tests/test_gpu_exact.py), so it
is pinned here first: (1) on random tiny chains it equals a brute-force enumeration of every
duty schedule, for either sign of the prices; (2) on the reference's own solves it reproduces
the MILP optimum of every base home (no battery, no PV: the MILP is the thermal part alone)
that HiGHS proved optimal, and is never worse than a HiGHS incumbent.  (The fixtures' MILP
objectives are c.x of HiGHS's own solution, whose continuous columns carry its ~1e-7 feasibility
slack: the comparison bound is 2e-6 relative.)
"""
import numpy as np
import pytest

from oracle import mpc as M
from oracle import thermal as TH
from tests import fixtures as F


def _random_chain(rng, H, S, sign):
    A = rng.uniform(0.6, 1.0, H)
    g = rng.choice([-1.0, 1.0]) * rng.uniform(0.2, 0.6)
    C = rng.normal(0, 0.3, H)
    q = rng.uniform(0.05, 1.0, H) * (1 if sign == "pos" else -1 if sign == "neg" else rng.choice([-1, 1], H))
    return dict(A=A, C=C, q=q, g=g, x0=rng.uniform(-0.5, 0.5), lo0=-1.0 - rng.uniform(0, 0.3), hi0=1.0,
                lo=-1.0, hi=1.0 + rng.uniform(0, 0.3), S=S)


@pytest.mark.parametrize("sign", ["pos", "neg", "mixed"])
def test_exact_chain_equals_enumeration(sign):
    rng = np.random.default_rng({"pos": 1, "neg": 2, "mixed": 3}[sign])
    n_feas = 0
    for _ in range(60):
        ch = _random_chain(rng, H=5, S=3, sign=sign)
        bf = TH.brute_force(ch)
        ex = TH.solve_chain(ch)
        if bf is None:
            assert ex is None
            continue
        n_feas += 1
        assert ex is not None
        assert abs(ex[0] - bf) <= 1e-12 * max(1.0, abs(bf)), (ex[0], bf)
        assert abs(float(np.dot(ch["q"], ex[1])) - ex[0]) <= 1e-12 * max(1.0, abs(bf))
    assert n_feas >= 20


def _si(r):
    return M.StepInput(t=r["t"], T0=r["T0"], Tw0=r["Tw0"], E0=r["E0"], oat=np.array(r["oat"]),
                       ghi=np.array(r["ghi"]), price=np.array(r["total_price"]), draw=np.array(r["draw_size"]),
                       winter=r["season"] == "winter")


@pytest.mark.parametrize("name", ["c1_h24", "spring_dt1", "summer_dt1"])
def test_exact_thermal_matches_reference_milp_on_base_homes(name):
    d = F.load(name)
    homes = {h["name"]: h for h in d["homes"]}
    n_proven = n_incumbent = 0
    for r in d["records"][::2]:
        if r["status"] != "optimal" or r["type"] != "base" or r["milp_obj"] is None:
            continue
        hc = M.home_const(homes[r["name"]])
        th = TH.thermal_optimum(hc, _si(r))
        assert th is not None, (name, r["name"], r["t"])
        ref = r["milp_obj"]
        if r["milp_status"] == 0:        # proven (HiGHS, mip_rel_gap <= 1e-6)
            n_proven += 1
            assert abs(th["cost"] - ref) <= 2e-6 * max(1.0, abs(ref)), (name, r["name"], r["t"], th["cost"], ref)
        else:                            # a time-limited incumbent: the exact optimum is no worse
            n_incumbent += 1
            assert th["cost"] <= ref + 2e-6 * max(1.0, abs(ref)), (name, r["name"], r["t"], th["cost"], ref)
    assert n_proven >= 5
    print(f"{name}: {n_proven} proven base-home optima reproduced, {n_incumbent} incumbents not beaten")


def _exact_fixture():
    import gzip
    import json
    import os
    with gzip.open(os.path.join(F.GOLDEN, "proven", "thermal_exact.json.gz"), "rt") as f:
        return json.load(f)


def _records(name):
    import gzip
    import json
    import os
    if name.startswith("proven/"):
        with gzip.open(os.path.join(F.GOLDEN, name + ".json.gz"), "rt") as f:
            return json.load(f)
    return F.load(name)


def test_exact_milp_optimum_pinned_by_highs():
    """The exact MILP optimum of every fixture solve (thermal DP + the LP of the rest with the
    duties fixed, make_thermal_exact.py) against the reference's HiGHS solves, all home types:
    equal to every PROVEN optimum (2e-6), None on every proven-infeasible record, and never
    above a time-limited incumbent.  This pins the separability argument (DESIGN.md section
    3.1) and the sequential tank-after-air solve on the full reference model."""
    ex = _exact_fixture()
    n = dict(proven=0, infeasible=0, incumbent=0, better=0)
    for name, rows in ex.items():
        d = _records(name)
        assert len(rows) == len(d["records"])
        for r, e in zip(d["records"], rows):
            ms, mo = r["milp_status"], r["milp_obj"]
            if ms == 2:
                n["infeasible"] += 1
                assert e["opt_obj"] is None, (name, r["name"], r["t"])
            elif mo is not None:
                assert e["opt_obj"] is not None, (name, r["name"], r["t"])
                rel = (e["opt_obj"] - mo) / max(1.0, abs(mo))
                if ms == 0:
                    n["proven"] += 1
                    assert abs(rel) <= 2e-6, (name, r["name"], r["t"], e["opt_obj"], mo)
                else:
                    n["incumbent"] += 1
                    n["better"] += rel < -2e-6
                    assert rel <= 2e-6, (name, r["name"], r["t"], e["opt_obj"], mo)
    assert n["proven"] >= 900 and n["infeasible"] >= 400
    print(f"exact MILP optimum: {n['proven']} proven optima reproduced, {n['infeasible']} proven-infeasible "
          f"agreed, {n['incumbent']} incumbents never beaten by them ({n['better']} improved on)")


def test_exact_fixture_recomputes():
    """A sample of thermal_exact.json.gz recomputed from the oracle (the file is what it says)."""
    ex = _exact_fixture()
    rng = np.random.default_rng(5)
    for name, rows in ex.items():
        d = _records(name)
        homes = {h["name"]: h for h in d["homes"]}
        for i in rng.choice(len(rows), size=min(6, len(rows)), replace=False):
            r, e = d["records"][i], rows[i]
            hc = M.home_const(homes[r["name"]])
            th = TH.thermal_optimum(hc, _si(r))
            opt = TH.exact_milp(hc, _si(r), th)
            assert (opt is None) == (e["opt_obj"] is None), (name, i)
            if opt is not None:
                assert opt == pytest.approx(e["opt_obj"], rel=1e-12, abs=1e-12), (name, i)


def test_exact_milp_on_the_proven_configs0_loop():
    """The configs[0] reference loop re-run to proven optimality (tests/golden/proven/c1_h24_proven.json.gz,
    HiGHS gap 0): on a sample of its solves the exact MILP optimum equals every proven optimum (2e-6),
    is None on every proven-infeasible record and never above a time-limited incumbent -- the CPU
    side of test_gpu_closed_loop.py's proven-loop test."""
    import gzip
    import json
    import os
    path = os.path.join(F.GOLDEN, "proven", "c1_h24_proven.json.gz")
    if not os.path.exists(path):
        pytest.skip("no proven configs[0] fixture")
    with gzip.open(path, "rt") as f:
        d = json.load(f)
    homes = {h["name"]: h for h in d["homes"]}
    n = dict(proven=0, infeasible=0, incumbent=0)
    for r in d["records"][::16]:
        hc = M.home_const(homes[r["name"]])
        opt = TH.exact_milp(hc, _si(r))
        ms, mo = r["milp_status"], r["milp_obj"]
        if ms == 2:
            n["infeasible"] += 1
            assert opt is None, (r["name"], r["t"])
        elif mo is not None:
            assert opt is not None, (r["name"], r["t"])
            rel = (opt - mo) / max(1.0, abs(mo))
            if ms == 0:
                n["proven"] += 1
                assert abs(rel) <= 2e-6, (r["name"], r["t"], opt, mo)
            else:
                n["incumbent"] += 1
                assert rel <= 2e-6, (r["name"], r["t"], opt, mo)
    assert n["proven"] >= 50
    print(n)
