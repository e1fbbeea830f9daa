"""Parity at the bench's full size (BASELINE configs[2] on one GPU: 10,000 homes, H = 48,
July, int_mode round) through size-independent properties -- the CPU oracle cannot solve
10k MILPs in a test, but it can check every answer the HIP path gives:

* no home hits a crashing path (the reference would raise);
* every optimal home's answer satisfies the reference model assembled by the oracle from
  inputs restated on the host (water draws, initial conditions from the previous step's hash,
  environment slices, season draw): equality and inequality violation <= 1e-5, duties
  integral, objective = c @ x (a 400-home sample per step, every home type);
* the integer optimum never undercuts the LP relaxation of the same state (relax mode on
  device), and a home whose relaxation is infeasible has no integer schedule either (all
  homes);
* strided shards reproduce the single batch bit for bit (all homes).
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, HOURS, DT, STEPS, SAMPLE = 10000, 12, 4, 2, 400


@pytest.fixture(scope="module")
def run(gpu):
    import torch
    from dragg_amd.aggregator import DeviceAggregator
    from dragg_amd.community import synthetic_homes, synthetic_weather
    sim_hours = math.ceil(STEPS / DT)
    days = math.ceil((sim_hours + HOURS + 2) / 24) + 1
    homes = synthetic_homes(N, seed=12, days=days, dt=DT, horizon_hours=HOURS)
    oat, ghi, tou = synthetic_weather(days, DT, sim_hours, seed=3, month=7)
    agg = DeviceAggregator(homes, oat, ghi, tou, 0, STEPS, reward_price=[0.0], seed=12)
    steps = []
    for t in range(STEPS):
        b = agg.batch
        prev_vals, prev_fc = b.vals.clone(), b.fc.clone()
        noise = b.season_noise(t)
        agg.run_iteration()
        torch.cuda.synchronize()
        steps.append(dict(t=t, prev_vals=prev_vals, prev_fc=prev_fc, noise=noise.cpu().numpy(),
                          status=b.status.cpu().numpy().copy(), obj=b.obj.cpu().numpy().copy(),
                          vals=b.vals.cpu().numpy().copy(), fc=b.fc.cpu().numpy().copy()))
    return dict(homes=homes, oat=oat, ghi=ghi, tou=tou, agg=agg, steps=steps)


def test_no_crashing_paths(run):
    from dragg_amd import _lib as L
    for s in run["steps"]:
        st = s["status"]
        assert not np.isin(st, [L.ST_ERR_MISSING, L.ST_ERR_PARSE]).any()
        assert (st == L.ST_OPTIMAL).mean() > 0.9, np.bincount(st)


def _hash_dict(vals, fc, i):
    """The home's redis hash (str values) as MPCBatch.hash_dict renders it."""
    from dragg_amd import _lib as L
    out = {}
    for k, name in enumerate(L.FC_KEYS):
        for j in range(fc.shape[1]):
            if not np.isnan(fc[k, j, i]):
                out[f"{name}_{j}"] = repr(float(fc[k, j, i]))
    for k, name in enumerate(L.VAL_KEYS):
        if not np.isnan(vals[k, i]):
            v = vals[k, i]
            out[name] = str(int(v)) if name in ("solve_counter", "correct_solve") else repr(float(v))
    return out


def test_answers_satisfy_reference_model(run):
    from oracle import mpc as M
    from dragg_amd import _lib as L
    from tests.test_gpu_parity import _expand
    rng = np.random.default_rng(0)
    types = np.array([h["type"] for h in run["homes"]])
    worst = 0.0
    for s in run["steps"]:
        t = s["t"]
        opt = np.flatnonzero(s["status"] == L.ST_OPTIMAL)
        # every type in the sample
        pick = np.concatenate([rng.choice(opt[types[opt] == ty], SAMPLE // 4, replace=False)
                               for ty in ("base", "pv_only", "battery_only", "pv_battery")])
        pv, pf = s["prev_vals"].cpu().numpy(), s["prev_fc"].cpu().numpy()
        for i in pick:
            hc = M.home_const(run["homes"][i])
            draw, _, _ = M.water_draws(hc, t)
            T0, Tw0, E0, _ = M.initial_conditions(hc, t, _hash_dict(pv, pf, i) if t else {}, draw)
            o, g, tt = M.env_slice(run["oat"], run["ghi"], run["tou"], 0, t, hc.H)
            si = M.StepInput(t=t, T0=T0, Tw0=Tw0, E0=E0, oat=o, ghi=g, price=M.total_price(tt, [0.0], hc.H),
                             draw=draw, winter=M.season_is_winter(o, s["noise"][:, i]))
            P, x = _expand(hc, si, s["vals"][:, i], s["fc"][:, :, i], hc.S)
            ve = np.abs(P["A_eq"] @ x - P["b_eq"]).max()
            vu = (P["A_ub"] @ x - P["b_ub"]).max()
            worst = max(worst, ve, vu)
            assert ve <= 1e-5 and vu <= 1e-5, (t, i, types[i], ve, vu)
            duties = x[P["integrality"] == 1]
            assert np.array_equal(duties, np.round(duties)), (t, i)
            assert abs(P["c"] @ x - s["obj"][i]) <= 1e-8 * max(1, abs(s["obj"][i])), (t, i)
    print(f"{len(run['steps'])} steps x {SAMPLE} homes: worst violation {worst:.2e}")


def test_integer_optimum_above_relaxation(run):
    """Same state, relax mode: obj(MILP) >= obj(LP) for every home optimal in both."""
    import torch
    from dragg_amd import _lib as L
    from dragg_amd.mpc import MPCBatch
    s = run["steps"][-1]
    b = run["agg"].batch
    r = MPCBatch(run["homes"], run["oat"], run["ghi"], run["tou"], 0, [0.0], int_mode="relax", seed=12)
    r.vals.copy_(s["prev_vals"])
    r.fc.copy_(s["prev_fc"])
    r.step(s["t"])
    torch.cuda.synchronize()
    rs, ro = r.status.cpu().numpy(), r.relax_obj.cpu().numpy()
    both = (rs == L.ST_OPTIMAL) & (s["status"] == L.ST_OPTIMAL)
    assert both.mean() > 0.9
    tol = 1e-7 * np.maximum(1.0, np.abs(ro[both]))
    assert (s["obj"][both] >= ro[both] - tol).all()
    lp_infeasible = np.isin(rs, [L.ST_INFEASIBLE, L.ST_INFEASIBLE_CERT])
    assert not (lp_infeasible & (s["status"] == L.ST_OPTIMAL)).any()
    gap = (s["obj"][both] - ro[both]) / np.maximum(1.0, np.abs(ro[both]))
    print(f"MILP - LP gap over {both.sum()} homes: mean {gap.mean():.2e}, max {gap.max():.2e}")
    assert b.N == N


def test_strided_shards_bitexact(run):
    import torch
    from dragg_amd.aggregator import DeviceAggregator
    full = run["agg"]
    parts = [DeviceAggregator(run["homes"], run["oat"], run["ghi"], run["tou"], 0, STEPS, reward_price=[0.0],
                              seed=12, rank=r, world=2) for r in range(2)]
    for _ in range(STEPS):
        for p in parts:
            p.run_iteration()
    torch.cuda.synchronize()
    joined = torch.empty_like(full.hist[:STEPS])
    for r, p in enumerate(parts):
        joined[:, :, r::2] = p.hist[:STEPS]
    assert torch.equal(torch.nan_to_num(full.hist[:STEPS], 7.0), torch.nan_to_num(joined, 7.0))
