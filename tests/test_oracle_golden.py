"""The CPU oracle (oracle/mpc.py) pinned against the reference's own outputs (CPU only).

tests/golden/*.json.gz were written by tests/golden/make_golden.py, which runs dragg's
unmodified Aggregator/MPCCalc (HiGHS standing in for GLPK_MI).  Each check below restates
one piece of mpc_calc.py and compares it with what the reference produced.
"""
import numpy as np
import pytest

from oracle import mpc as M
from tests import fixtures as F

SCEN = F.scenarios()


def _si(r):
    return M.StepInput(t=r["t"], T0=r["T0"], Tw0=r["Tw0"], E0=r["E0"], oat=np.array(r["oat"]),
                       ghi=np.array(r["ghi"]), price=np.array(r["total_price"]),
                       draw=np.array(r["draw_size"]), winter=r["season"] == "winter")


@pytest.fixture(scope="module", params=SCEN)
def scen(request):
    d = F.load(request.param)
    return request.param, d, {h["name"]: h for h in d["homes"]}


def test_water_draws_bitexact(scen):
    """mpc_calc.py:193-204 (lagged, repeated, 3-point averaged draws)."""
    name, d, homes = scen
    for r in d["records"]:
        hc = M.home_const(homes[r["name"]])
        draw, _, _ = M.water_draws(hc, r["t"])
        assert draw.tolist() == r["draw_size"], (name, r["name"], r["t"])


def test_season_and_price(scen):
    """mpc_calc.py:220-223, 303-309 (season from the noisy OAT forecast), :353 (total price)."""
    name, d, homes = scen
    for r in d["records"]:
        hc = M.home_const(homes[r["name"]])
        assert M.season_is_winter(r["oat"], r["noise"]) == (r["season"] == "winter")
        assert M.total_price(r["tou"], r["reward_price"], hc.H).tolist() == r["total_price"]


def test_env_slices(scen):
    """mpc_calc.py:211-226: the per-step OAT/GHI/TOU windows of the redis lists."""
    name, d, homes = scen
    env = d["env"]
    if env["start_hour_index"] != 0:
        pytest.skip("fixture stores the lists from index 0 only")
    for r in d["records"][:200]:
        hc = M.home_const(homes[r["name"]])
        oat, ghi, tou = M.env_slice(env["oat"], env["ghi"], env["tou_window"], 0, r["t"], hc.H)
        assert oat.tolist() == r["oat"] and ghi.tolist() == r["ghi"] and tou.tolist() == r["tou"]


def test_initial_conditions_chain(scen):
    """mpc_calc.py:264-289: each solve's T0/Tw0/E0/counter follow from the previous hash."""
    name, d, homes = scen
    by = {(r["name"], r["t"]): r for r in d["records"]}
    n = 0
    for (hname, t), r in by.items():
        hc = M.home_const(homes[hname])
        draw, _, _ = M.water_draws(hc, t)
        if t == 0:
            T0, Tw0, E0, cnt = M.initial_conditions(hc, 0, {}, draw)
        else:
            prev = by.get((hname, t - 1))
            if prev is None:
                continue
            hsh = {k: M.enc(int(v) if k in ("solve_counter", "correct_solve") else v)
                   for k, v in prev["optimal_vals"].items()}
            # fields the previous step did not write persist from earlier steps
            if "e_batt_opt" not in hsh and hc.has_batt:
                continue
            T0, Tw0, E0, cnt = M.initial_conditions(hc, t, hsh, draw)
        assert T0 == r["T0"] and Tw0 == r["Tw0"] and cnt == r["counter_in"], (hname, t)
        if hc.has_batt:
            assert E0 == r["E0"], (hname, t)
        n += 1
    assert n > 0


def test_lp_relaxation_objective(scen):
    """Problem assembly (mpc_calc.py:291-446): the LP relaxation of the oracle's model has the
    reference's status and objective."""
    name, d, homes = scen
    recs = d["records"][::3] if len(d["records"]) > 300 else d["records"]
    for r in recs:
        hc = M.home_const(homes[r["name"]])
        st, x, obj = M.solve_problem(M.build_problem(hc, _si(r)), integer=False)
        assert (st == "optimal") == (r["lp_status"] == 0), (name, r["name"], r["t"])
        if st == "optimal":
            assert abs(obj - r["lp_obj"]) <= 1e-8 * max(1.0, abs(r["lp_obj"])), (name, r["name"], r["t"])


def test_milp_status(scen):
    """Integer feasibility agrees with the reference's MILP status on a sample."""
    name, d, homes = scen
    recs = d["records"][::97][:8]
    for r in recs:
        hc = M.home_const(homes[r["name"]])
        st, x, obj = M.solve_problem(M.build_problem(hc, _si(r)), integer=True, time_limit=5.0)
        assert (st == "optimal") == (r["status"] == "optimal"), (name, r["name"], r["t"])
        if st == "optimal" and r["milp_obj"] is not None:
            lb = r["lp_obj"]
            assert obj >= lb - 1e-7 * max(1.0, abs(lb))


def test_fallback_bitexact(scen):
    """cleanup_and_finish failure branch (mpc_calc.py:527-595), including the first-character
    parse of the previous hash strings, bit for bit."""
    name, d, homes = scen
    n = 0
    for r in d["records"]:
        if r["status"] == "optimal":
            continue
        hc = M.home_const(homes[r["name"]])
        ov, cnt = M.cleanup(hc, _si(r), r["status"], None, r["prev_hash"], r["counter_in"])
        assert cnt == r["counter_out"]
        assert set(ov) == set(r["optimal_vals"]), (name, r["name"], r["t"])
        for k, v in r["optimal_vals"].items():
            if isinstance(v, str):          # copied verbatim from the previous hash
                assert ov[k] == v, (name, r["name"], r["t"], k, ov[k], v)
            else:
                assert float(ov[k]) == float(v), (name, r["name"], r["t"], k, ov[k], v)
        n += 1
    print(f"{name}: {n} fallback records bit-exact")


def test_success_extraction(scen):
    """Success branch (mpc_calc.py:486-526): feed the reference MILP's duty cycles back, solve
    the remaining LP and compare the extracted hash fields."""
    name, d, homes = scen
    recs = [r for r in d["records"] if r["status"] == "optimal" and r.get("milp_x")][::7][:40]
    for r in recs:
        hc = M.home_const(homes[r["name"]])
        si = _si(r)
        P = M.build_problem(hc, si)
        L = P["layout"]
        # fix the integer duty cycles to the reference's values
        A_fix, b_fix = [], []
        for k in ("hvac_cool_on", "hvac_heat_on", "wh_heat_on"):
            for j, v in enumerate(r["milp_x"][k]):
                row = np.zeros(L.n)
                row[L.idx(k, j)] = 1.0
                A_fix.append(row)
                b_fix.append(v)
        P2 = dict(P)
        P2["A_eq"] = np.vstack([P["A_eq"], np.array(A_fix)])
        P2["b_eq"] = np.concatenate([P["b_eq"], b_fix])
        st, x, obj = M.solve_problem(P2, integer=False)
        assert st == "optimal"
        ov, cnt = M.cleanup(hc, si, "optimal", x, {}, r["counter_in"])
        ref = r["optimal_vals"]
        assert set(ov) == set(ref)
        for k in ref:
            if any(k.startswith(p) for p in ("temp_in_ev_opt", "temp_wh_ev_opt", "hvac_", "wh_heat_on_opt",
                                              "p_load_opt", "waterdraws", "temp_in_opt", "temp_wh_opt",
                                              "correct_solve", "solve_counter")):
                assert abs(float(ov[k]) - float(ref[k])) <= 1e-6 * max(1.0, abs(float(ref[k]))), (k, ov[k], ref[k])


def test_collected_aggregates(scen):
    """collect_data (aggregator.py:737-755): p_grid_aggregate is the per-step sum of the
    homes' p_grid_opt fields."""
    name, d, homes = scen
    agg = d["results"]["Summary"]["p_grid_aggregate"]
    by_t = {}
    for r in d["records"]:
        by_t.setdefault(r["t"], []).append(float(r["optimal_vals"]["p_grid_opt"]))
    for t, vals in by_t.items():
        if len(vals) == len(homes):
            assert abs(sum(vals) - agg[t]) <= 1e-9 * max(1.0, abs(agg[t])), (name, t)


def _battery_lp(hc, si):
    """The battery block alone (mpc_calc.py:355-373 with its cost term S*(ch+dis), :405-432):
    min sum_k gamma^k price_k S (ch_k + dis_k), E_k = E0 + sum_{j<k} (eta_c ch_j + dis_j/eta_d)/dt."""
    from scipy.optimize import linprog
    H, S, dt, b = hc.H, hc.S, hc.dt, hc.batt
    w = np.power(hc.discount * np.ones(H), np.arange(H)) * np.asarray(si.price[:H], float) * S
    low = np.tril(np.ones((H, H)))
    A = np.hstack([low * (b["eta_c"] / dt), low * ((1.0 / b["eta_d"]) / dt)])
    res = linprog(np.r_[w, w], A_ub=np.vstack([A, -A]),
                  b_ub=np.r_[np.full(H, b["Emax"] - si.E0), np.full(H, si.E0 - b["Emin"])],
                  bounds=[(0, b["rate"])] * H + [(-b["rate"], 0)] * H, method="highs")
    assert res.status == 0
    return res.fun


def _pv_part(hc, si):
    """The PV block alone (mpc_calc.py:375-385): curtail (u = 1) only where the weight is < 0."""
    H, S = hc.H, hc.S
    w = np.power(hc.discount * np.ones(H), np.arange(H)) * np.asarray(si.price[:H], float) * S
    p = hc.pv["area"] * hc.pv["eff"] * np.asarray(si.ghi[:H], float) / 1000
    return float(np.sum(np.where(w < 0, 0.0, -w * p)))


def test_model_is_separable(scen):
    """The default GPU path rests on the model being separable: the
    reference's LP (and MILP) optimum = thermal part (the model of a 'base' home) + battery
    LP + PV LP.  Checked against the reference's recorded objectives."""
    import dataclasses
    name, d, homes = scen
    recs = [r for r in d["records"] if r["lp_status"] == 0 and r["type"] != "base"]
    recs = recs[::max(1, len(recs) // 60)]
    n_lp = n_milp = 0
    for r in recs:
        hc = M.home_const(homes[r["name"]])
        si = _si(r)
        base = dataclasses.replace(hc, type="base")
        st, _, thermal = M.solve_problem(M.build_problem(base, si), integer=False)
        assert st == "optimal"
        rest = (_battery_lp(hc, si) if hc.has_batt else 0.0) + (_pv_part(hc, si) if hc.has_pv else 0.0)
        assert abs(thermal + rest - r["lp_obj"]) <= 1e-7 * max(1.0, abs(r["lp_obj"])), (name, r["name"], r["t"])
        n_lp += 1
        if hc.H <= 12 and r["status"] == "optimal" and r["milp_obj"] is not None and (r["milp_gap"] or 0) < 1e-6:
            st, _, thermal_i = M.solve_problem(M.build_problem(base, si), integer=True, time_limit=20.0)
            assert abs(thermal_i + rest - r["milp_obj"]) <= 1e-6 * max(1.0, abs(r["milp_obj"])), (name, r["name"])
            n_milp += 1
    print(f"{name}: separable on {n_lp} LP and {n_milp} MILP records")
