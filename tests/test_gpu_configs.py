"""BASELINE configs[1], [3] and [4] at their own sizes on one GPU (configs[2] is
tests/test_gpu_fullsize.py and the bench).

The CPU oracle cannot solve these runs, but it can check any answer the HIP path gives, so each
test runs the whole workload on the device and then checks a sample of its solves on the host:

* the state a sampled solve started from is restated by the oracle from the previous step's
  hash (water draws, initial conditions, environment slices, the device's season draw);
* the exact MILP optimum of that state (oracle/thermal.py exact_milp: the thermal DP + the LP of the
  rest with the duties fixed; pinned on every HiGHS-proven fixture record by
  tests/test_oracle_thermal.py) decides the status -- ours optimal iff it exists -- and the
  objective must equal it (1e-6 relative);
* the written answer satisfies the reference model (violation <= 1e-5, duties integral,
  c.x = objective).

Synthetic communities can contain battery homes whose t = 0 solve fails; the reference then
raises KeyError('e_batt_opt') at t = 1 (mpc_calc.py:280-289), and a run that stops at t = 1 is
not a run of the reference.  The at-size tests therefore run communities the reference completes
(dragg_amd.community.reference_completable, the bench's rule: such battery homes swap places
with homes without a battery) and require no error; test_crashing_community_raises_the_references
_keyerror keeps one small community as drawn and asserts the reference's KeyError path.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _community(n, hours, dt, steps, month, seed, completable=True, rp=(0.0,)):
    from dragg_amd.community import synthetic_homes, synthetic_weather, reference_completable
    sim_hours = math.ceil(steps / dt)
    days = math.ceil((sim_hours + hours + 2) / 24) + 1
    homes = synthetic_homes(n, seed=seed, days=days, dt=dt, horizon_hours=hours)
    oat, ghi, tou = synthetic_weather(days, dt, sim_hours, seed=seed + 1, month=month)
    if completable:
        homes, _ = reference_completable(homes, oat, ghi, tou, seed=seed, reward_price=rp)
    return homes, oat, ghi, tou


def _check_sample(homes, oat, ghi, tou, rp, t, prev_vals, prev_fc, noise, status, obj, vals, fc, pick, path=None,
                  fallback_gaps=None, approx_bound=0.05):
    """Exact optimum + reference-model check of the solves `pick` of step t.  With `path` (the
    kernel's int_path), solves that left the exact front DP (front overflow under RL prices) are
    held to the bucketed fallback's bound instead: never below the optimum, at most 5 % above;
    their gaps go to `fallback_gaps`."""
    from oracle import mpc as M
    from oracle import thermal as TH
    from dragg_amd import _lib as L
    from tests.test_gpu_fullsize import _hash_dict
    from tests.test_gpu_parity import _expand
    worst_gap = worst_v = 0.0
    n_opt = n_none = 0
    for i in pick:
        hc = M.home_const(homes[i])
        draw, _, _ = M.water_draws(hc, t)
        hsh = _hash_dict(prev_vals, prev_fc, i) if t else {}
        if status[i] == L.ST_ERR_MISSING:            # the reference raises here too
            with pytest.raises(KeyError):
                M.initial_conditions(hc, t, hsh, draw)
            continue
        T0, Tw0, E0, _ = M.initial_conditions(hc, t, hsh, draw)
        o, g, tt = M.env_slice(oat, ghi, tou, 0, t, hc.H)
        si = M.StepInput(t=t, T0=T0, Tw0=Tw0, E0=E0, oat=o, ghi=g, price=M.total_price(tt, rp, hc.H), draw=draw,
                         winter=M.season_is_winter(o, noise[:, i]))
        opt = TH.exact_milp(hc, si)
        ours = status[i] == L.ST_OPTIMAL
        assert ours == (opt is not None), (t, i, homes[i]["type"], L.STATUS_NAMES[status[i]], opt)
        if not ours:
            n_none += 1
            continue
        n_opt += 1
        if path is not None and path[i] & L.PATH_APPROX_MASK:
            g = (obj[i] - opt) / max(1.0, abs(opt))
            assert -1e-9 <= g <= approx_bound, (t, i, homes[i]["type"], obj[i], opt, path[i])
            fallback_gaps.append(g)
            continue
        gap = abs(obj[i] - opt) / max(1.0, abs(opt))
        worst_gap = max(worst_gap, gap)
        if gap > 1e-6:
            _dump_failure(homes[i], si, t, i, obj[i], opt, vals[:, i], fc[:, :, i])
        assert gap <= 1e-6, (t, i, homes[i]["type"], obj[i], opt)
        P, x = _expand(hc, si, vals[:, i], fc[:, :, i], hc.S)
        ve = np.abs(P["A_eq"] @ x - P["b_eq"]).max()
        vu = (P["A_ub"] @ x - P["b_ub"]).max()
        worst_v = max(worst_v, ve, vu)
        assert ve <= 1e-5 and vu <= 1e-5, (t, i, ve, vu)
        duties = x[P["integrality"] == 1]
        assert np.array_equal(duties, np.round(duties)), (t, i)
        assert abs(P["c"] @ x - obj[i]) <= 1e-8 * max(1, abs(obj[i])), (t, i)
    return n_opt, n_none, worst_gap, worst_v


def _dump_failure(home, si, t, i, ours, opt, vals, fc):
    """Keep a failing solve's inputs and our answer (gpurun_out/, for the CPU side)."""
    import json
    import os
    os.makedirs("gpurun_out", exist_ok=True)
    rec = dict(home=home, t=t, i=int(i), ours=float(ours), opt=float(opt), T0=si.T0, Tw0=si.Tw0, E0=si.E0,
               oat=list(map(float, si.oat)), ghi=list(map(float, si.ghi)), price=list(map(float, si.price)),
               draw=list(map(float, si.draw)), winter=bool(si.winter), vals=vals.tolist(), fc=fc.tolist())
    with open(f"gpurun_out/fail_t{t}_h{int(i)}.json", "w") as f:
        json.dump(rec, f, default=float)


def _errors_are_the_references(agg, homes):
    """check_errors() raises iff a home hit a crashing path, and each such home is a battery home
    whose t = 0 solve failed (the reference's KeyError('e_batt_opt') at t = 1)."""
    from dragg_amd import _lib as L
    st = agg.status_hist[:agg.timestep].cpu().numpy()
    miss = np.argwhere(st == L.ST_ERR_MISSING)
    assert not (st == L.ST_ERR_PARSE).any()
    if len(miss) == 0:
        agg.check_errors()
        return 0
    with pytest.raises(KeyError):
        agg.check_errors()
    for _, i in miss:
        assert "battery" in homes[agg.index[i]]["type"]
        assert st[0, i] != L.ST_OPTIMAL
    return len(np.unique(miss[:, 1]))


def _sample(rng, status, homes, per_type):
    """per_type solves of each home type, drawn from the optimal ones and the others alike."""
    types = np.array([h["type"] for h in homes])
    out = []
    for ty in ("base", "pv_only", "battery_only", "pv_battery"):
        idx = np.flatnonzero(types == ty)
        out.extend(rng.choice(idx, min(per_type, len(idx)), replace=False))
    return np.array(out)


def _run(n, hours, dt, steps, month, seed, sample_steps, per_type, rp=(0.0,), keep_history=True, completable=True):
    import torch
    from dragg_amd.aggregator import DeviceAggregator
    homes, oat, ghi, tou = _community(n, hours, dt, steps, month, seed, completable, rp)
    agg = DeviceAggregator(homes, oat, ghi, tou, 0, steps, reward_price=list(rp), seed=seed,
                           keep_history=keep_history)
    rng = np.random.default_rng(seed)
    checked = []
    for t in range(steps):
        b = agg.batch
        snap = (t in sample_steps) and (b.vals.clone(), b.fc.clone(), b.season_noise(t).cpu().numpy())
        agg.run_iteration()
        agg.collect_data(defer=True)
        if snap:
            torch.cuda.synchronize()
            st, ob = b.status.cpu().numpy(), b.obj.cpu().numpy()
            pick = _sample(rng, st, homes, per_type)
            res = _check_sample(homes, oat, ghi, tou, list(rp), t, snap[0].cpu().numpy(), snap[1].cpu().numpy(),
                                snap[2], st, ob, b.vals.cpu().numpy(), b.fc.cpu().numpy(), pick)
            checked.append((t,) + res)
    agg.reduce_history()
    torch.cuda.synchronize()
    return homes, agg, checked


def _report(tag, agg, homes, checked, min_opt=50, completable=True):
    from dragg_amd import _lib as L
    st = agg.status_hist[:agg.timestep].cpu().numpy()
    counts = {L.STATUS_NAMES[c]: int((st == c).sum()) for c in np.unique(st)}
    n_err = _errors_are_the_references(agg, homes)
    if completable:                                  # a run the reference completes: no crash path
        assert n_err == 0 and not (st == L.ST_ERR_MISSING).any()
    n_opt = sum(c[1] for c in checked)
    n_none = sum(c[2] for c in checked)
    print(f"{tag}: {st.size} solves {counts}; homes on the reference's KeyError path: {n_err}; "
          f"checked {n_opt} exact-path optimal solves (|gap| to the exact MILP optimum max "
          f"{max(c[3] for c in checked):.1e}, violation max {max(c[4] for c in checked):.1e}) and "
          f"{n_none} without an integer schedule")
    assert n_opt >= min_opt
    return st


def test_config1_1k_homes_h24_96_steps(gpu):
    """configs[1]: 1,000 homes, run_rbo_mpc, 24 h at 15-min steps, 6 h horizon."""
    homes, agg, checked = _run(1000, 6, 4, 96, 1, 31, sample_steps={0, 1, 23, 47, 95}, per_type=25)
    st = _report("configs[1] 1k homes x 96 steps, H = 24, January", agg, homes, checked)
    assert st.shape == (96, 1000)
    # the collected sums are the homes' fields summed (aggregator.py:728-755)
    from dragg_amd import _lib as L
    hist = agg.hist[:96].cpu().numpy()
    want = np.stack([hist[:, L.K[k], :].sum(axis=1) for k in ("p_grid_opt", "forecast_p_grid_opt", "cost_opt")], 1)
    got = agg.agg_hist[:96].cpu().numpy()
    ok = ~np.isnan(want)
    assert np.allclose(got[ok], want[ok], rtol=1e-12, atol=1e-9)


def test_crashing_community_raises_the_references_keyerror(gpu):
    """configs[1]'s community as drawn (no swaps) holds battery homes whose t = 0 solve fails:
    the reference raises KeyError('e_batt_opt') at t = 1 (mpc_calc.py:280-289); check_errors()
    raises exactly that, for battery homes whose t = 0 solve failed, and nothing else differs."""
    homes, agg, checked = _run(1000, 6, 4, 4, 1, 31, sample_steps={0, 1}, per_type=25, completable=False)
    st = _report("configs[1] community as drawn, 4 steps", agg, homes, checked, min_opt=20, completable=False)
    from dragg_amd import _lib as L
    assert (st == L.ST_ERR_MISSING).any()


def test_config3_100k_homes_7_days(gpu):
    """configs[3]: 100,000 homes, 7 days at 15-min steps (672 steps), device-resident state,
    no per-step history (keep_history=False)."""
    homes, agg, checked = _run(100000, 6, 4, 672, 7, 41, sample_steps={0, 335, 671}, per_type=20,
                               keep_history=False)
    assert agg.hist is None
    st = _report("configs[3] 100k homes x 672 steps, H = 24, July", agg, homes, checked)
    assert st.shape == (672, 100000)
    assert np.isfinite(agg.agg_hist[:672].cpu().numpy()[:, 0]).all()


def test_config4_rl_10k_homes_price_broadcast_and_rollouts(gpu):
    """configs[4]: run_rl_agg at 10,000 homes (H = 48): per action the reward price is set,
    forecast_horizon rollout steps are solved and the state restored, then the committed steps
    must equal the rollout bit for bit; a sample of the committed RL-price solves is checked
    against the exact optimum (prices of either sign: the kernel's mixed-sign path included)."""
    import torch
    from dragg_amd import _lib as L
    from dragg_amd.aggregator import DeviceAggregator
    homes, oat, ghi, tou = _community(10000, 12, 4, 8, 7, 51, rp=[0.0] * 48)
    agg = DeviceAggregator(homes, oat, ghi, tou, 0, 8, reward_price=[0.0] * 48, seed=51)
    for _ in range(2):
        agg.run_iteration()
        agg.collect_data()
    rp = list(-0.03 * np.cos(np.arange(48) / 3.0))
    agg.set_reward_price(rp)
    snap = agg.snapshot()
    fc = agg.forecast(2)
    after = agg.snapshot()
    assert after[0] == snap[0]
    assert torch.equal(after[1].nan_to_num(7.7), snap[1].nan_to_num(7.7))
    assert torch.equal(after[2].nan_to_num(7.7), snap[2].nan_to_num(7.7))
    b = agg.batch
    t = agg.timestep
    prev_vals, prev_fc, noise = b.vals.cpu().numpy(), b.fc.cpu().numpy(), b.season_noise(t).cpu().numpy()
    committed = []
    for s in range(2):
        agg.run_iteration()
        committed.append(agg.collect_data().clone())
        if s == 0:
            torch.cuda.synchronize()
            st, ob = b.status.cpu().numpy(), b.obj.cpu().numpy()
            path = b.int_path.cpu().numpy()
            pick = _sample(np.random.default_rng(51), st, homes, 25)
            fb = []
            res = _check_sample(homes, oat, ghi, tou, rp, t, prev_vals, prev_fc, noise, st, ob,
                                b.vals.cpu().numpy(), b.fc.cpu().numpy(), pick, path=path, fallback_gaps=fb,
                                approx_bound=1e-9)
            n_off = int((path[st == 0] & L.PATH_APPROX_MASK != 0).sum())
    assert torch.equal(fc, torch.stack(committed))
    agg.restore(snap)
    agg.set_reward_price([x + 0.2 for x in rp])
    assert not torch.equal(agg.forecast(1), fc[:1])
    fb = np.array(fb)
    n_second = int((path[st == 0] & L.PATH_SECOND != 0).sum())
    print(f"configs[4]: {n_second} of {int((st == 0).sum())} optimal homes solved by the second launch (big "
          f"exact fronts under the smooth RL price), {n_off} of them left the exact DP (front overflow past "
          f"NF_BIG); sampled fallback gaps to the exact optimum: {len(fb)}, mean "
          f"{fb.mean() if len(fb) else 0:.1e}, max {fb.max() if len(fb) else 0:.1e}")
    # RL prices are exact by default since round 5 (the indoor-air chain's cell bound, the beam's upper
    # bound and the bisection on the bound): no chain keeps an approximate schedule
    assert n_off == 0, n_off
    _report("configs[4] RL 10k homes, H = 48, July, rollout = commit", agg, homes, [(t,) + res], min_opt=0)


def _narrow(path):
    """int_path: the home left the front DP for the exact step-function DP (bit 15: a feasible set
    narrower than one duty step, mixed-sign prices, ...), or a chain kept the bucketed
    approximation because its feasible set is narrower than one duty step (reason 2)."""
    from dragg_amd import _lib as L
    path = np.asarray(path, np.int64)
    return (((path & L.PATH_STEPS) != 0) | (((path & 1) != 0) & (((path >> 4) & 0xF) == 2)) |
            (((path & 2) != 0) & (((path >> 8) & 0xF) == 2)))


@pytest.fixture(scope="module")
def bench_day(gpu):
    """The bench workload (BASELINE configs[2]: the bench's own 10,000-home community, July, H = 48)
    for 100 closed-loop steps (a full simulated day and then some), keeping every step that has a
    ROUND_FAIL or a narrow-set solve."""
    import torch
    from dragg_amd import _lib as L
    from dragg_amd.aggregator import DeviceAggregator
    from dragg_amd.community import synthetic_homes, synthetic_weather
    dt, Hh, steps = 4, 12, 100
    sim_hours = math.ceil(steps / dt)
    days = math.ceil((sim_hours + Hh + 2) / 24) + 1
    homes = synthetic_homes(10000, seed=12, days=days, dt=dt, horizon_hours=Hh)
    oat, ghi, tou = synthetic_weather(days, dt, sim_hours, seed=3, month=7)
    agg = DeviceAggregator(homes, oat, ghi, tou, 0, steps, reward_price=[0.0], seed=12, keep_history=False)
    b = agg.batch
    kept = []
    n_approx = n_steps_dp = 0
    for t in range(steps):
        prev = (b.vals.clone(), b.fc.clone())
        agg.run_iteration()
        st = b.status.cpu().numpy()
        path = b.int_path.cpu().numpy()
        n_approx += int(((path & L.PATH_APPROX_MASK) != 0).sum())
        n_steps_dp += int(((path & L.PATH_STEPS) != 0).sum())
        if not ((st == L.ST_ROUND_FAIL).any() or _narrow(path).any()):
            continue
        kept.append(dict(t=t, prev_vals=prev[0].cpu().numpy(), prev_fc=prev[1].cpu().numpy(),
                         noise=b.season_noise(t).cpu().numpy(), status=st, obj=b.obj.cpu().numpy(),
                         vals=b.vals.cpu().numpy(), fc=b.fc.cpu().numpy(), path=path))
    torch.cuda.synchronize()
    return dict(homes=homes, oat=oat, ghi=ghi, tou=tou, steps=kept, n_steps=steps, n_approx=n_approx,
                n_steps_dp=n_steps_dp)


def test_bench_default_build_exact_on_every_solve(bench_day):
    """The default build over 100 bench steps (10,000 homes, H = 48, July: 1,000,000 solves): no solve
    keeps an approximate integer schedule (int_path bits 0-11 clear on every home and step) -- every
    chain the Pareto-front DPs cannot take is solved by the exact step-function DP (bit 15)."""
    d = bench_day
    print(f"bench workload, {d['n_steps']} steps: {d['n_steps_dp']} home-steps through the step-function DP, "
          f"{d['n_approx']} on an approximate schedule")
    assert d["n_approx"] == 0


def test_bench_round_fail_solves_have_no_integer_schedule(bench_day):
    """ST_ROUND_FAIL (box-feasible, no integer duty schedule) of the bench workload over 100 steps:
    oracle/thermal.py's exact checker must find no integer schedule either (the reference's GLPK_MI
    then reports infeasible and falls back, mpc_calc.py:447-455), and the kernel records which
    chain decided it (int_path bits 13 / 14).  The checker solves T first and Tw given T, as the
    kernel does; the joint verdict on the full model, independent of that decomposition, is
    test_gpu_joint.py's (HiGHS feasibility fixtures)."""
    from dragg_amd import _lib as L
    d = bench_day
    n_fail = n_checked = 0
    chains = [0, 0]
    for s in d["steps"]:
        st = s["status"]
        pick = np.flatnonzero(st == L.ST_ROUND_FAIL)
        if len(pick) == 0:
            continue
        n_fail += len(pick)
        for i in pick:
            p = int(s["path"][i])
            assert bool(p & L.PATH_FAIL_T) != bool(p & L.PATH_FAIL_TW), (s["t"], i, p)   # exactly one chain
            chains[bool(p & L.PATH_FAIL_TW)] += 1
        res = _check_sample(d["homes"], d["oat"], d["ghi"], d["tou"], [0.0], s["t"], s["prev_vals"], s["prev_fc"],
                            s["noise"], st, s["obj"], s["vals"], s["fc"], pick)
        n_checked += res[1]                        # solves the checker also found no schedule for
    print(f"bench workload, {d['n_steps']} steps: {n_fail} ROUND_FAIL solves ({chains[0]} decided by the indoor-air "
          f"chain, {chains[1]} by the tank chain), {n_checked} confirmed without an integer schedule by the "
          f"exact checker")
    assert n_fail > 0 and n_checked == n_fail


def test_bench_narrow_set_solves_gap_bound_and_exact_mode(bench_day):
    """A chain whose feasible set is narrower than one duty step somewhere in the horizon breaks the
    front DP's dominance; the exact step-function DP (DM_NARROW, int_path bit 15) solves it, on the
    domains cut by the LP bounds and the bucketed schedule's cost.  Every such solve of the bench
    workload over 100 steps: status and objective equal to the exact optimum (oracle/thermal.py
    exact_milp, the assumption-free backward DP; 1e-9).  MPCBatch(exact=True) (DRAGG_FLAG_EXACT: it only
    changes RL-priced chains whose fronts pass 2,048 labels, none here) gives the same: every one equals
    the exact optimum and none keeps an approximation."""
    import torch
    from dragg_amd import _lib as L
    from dragg_amd.aggregator import DeviceAggregator
    d = bench_day
    gaps, n = [], 0
    for s in d["steps"]:
        pick = np.flatnonzero(_narrow(s["path"]))
        if len(pick) == 0:
            continue
        n += len(pick)
        _check_sample(d["homes"], d["oat"], d["ghi"], d["tou"], [0.0], s["t"], s["prev_vals"], s["prev_fc"],
                      s["noise"], s["status"], s["obj"], s["vals"], s["fc"], pick, path=s["path"],
                      fallback_gaps=gaps, approx_bound=NARROW_GAP_BOUND)
    g = np.array(gaps)
    print(f"bench workload, {d['n_steps']} steps: {n} narrow-set solves, {len(g)} optimal on the bucketed schedule: "
          f"gap to the exact optimum max {g.max() if len(g) else 0:.2e}, {int((g > 1e-9).sum())} above 1e-9")
    assert n > 0 and (len(g) == 0 or g.max() <= NARROW_GAP_BOUND)
    # exact mode: re-solve those same steps from the same states with the step-function DP
    from dragg_amd.mpc import MPCBatch
    n_exact = 0
    for s in d["steps"]:
        pick = np.flatnonzero(_narrow(s["path"]))
        if len(pick) == 0:
            continue
        b = MPCBatch([d["homes"][i] for i in pick], d["oat"], d["ghi"], d["tou"], 0, [0.0], seed=12,
                     home_offset=0, exact=True)
        # the same global noise keys: rebuild the picked homes' rows of the season draw
        b.vals.copy_(torch.tensor(s["prev_vals"][:, pick]))
        b.fc.copy_(torch.tensor(s["prev_fc"][:, :, pick]))
        b.step(s["t"], noise=torch.tensor(s["noise"][:, pick]))
        torch.cuda.synchronize()
        st, ob, path = b.status.cpu().numpy(), b.obj.cpu().numpy(), b.int_path.cpu().numpy()
        assert not (path & L.PATH_APPROX_MASK).any(), path
        assert (st == s["status"][pick]).all(), (st, s["status"][pick])
        # the exact mode's answers in place of the default ones, held to the exact optimum (1e-6)
        # and the reference model (violation, integrality, c.x = objective)
        ob_all, vals_all, fc_all = s["obj"].copy(), s["vals"].copy(), s["fc"].copy()
        ob_all[pick] = ob
        vals_all[:, pick] = b.vals.cpu().numpy()
        fc_all[:, :, pick] = b.fc.cpu().numpy()
        _check_sample(d["homes"], d["oat"], d["ghi"], d["tou"], [0.0], s["t"], s["prev_vals"], s["prev_fc"],
                      s["noise"], s["status"], ob_all, vals_all, fc_all, pick)
        ex = {i: ob[j] for j, i in enumerate(pick) if st[j] == L.ST_OPTIMAL}
        n_exact += len(ex)
    print(f"exact mode: {n_exact} of those solves by the step-function DP, all at the exact optimum")


NARROW_GAP_BOUND = 1e-9      # exact: the step-function DP (round 3's bucketed approximation: 8.5 %, home 7519 at t = 60)


def test_rl_bench_price_exact_on_every_chain(gpu):
    """The bench's RL workload (bench.py --workload rl: its 10,000-home community, July, H = 48, the
    smooth reward price that changes at every stage): every chain of two actions' steps solved exactly
    (no int_path approximation bit; round 4 left ~30 % of the indoor-air chains on the bucketed schedule
    there), and a sample of 20 solves per step equal to the exact optimum (oracle/thermal.py, 1e-9)."""
    import torch
    from dragg_amd import _lib as L
    from dragg_amd.aggregator import DeviceAggregator
    from dragg_amd.community import synthetic_homes, synthetic_weather
    dt, hh, steps = 4, 12, 2
    sim_hours = math.ceil(steps / dt)
    days = math.ceil((sim_hours + hh + 2) / 24) + 1
    homes = synthetic_homes(10000, seed=12, days=days, dt=dt, horizon_hours=hh)
    oat, ghi, tou = synthetic_weather(days, dt, sim_hours, seed=3, month=7)
    H = hh * dt
    off = np.random.default_rng(5).uniform(-0.02, 0.02, (steps, 1))
    prices = off + (-0.03 * np.cos(np.arange(H) / 3.0))[None, :]
    agg = DeviceAggregator(homes, oat, ghi, tou, 0, steps, reward_price=[0.0] * H, seed=12)
    b = agg.batch
    rng = np.random.default_rng(7)
    for t in range(steps):
        rp = list(prices[t])
        agg.set_reward_price(rp)
        prev_vals, prev_fc, noise = b.vals.cpu().numpy(), b.fc.cpu().numpy(), b.season_noise(t).cpu().numpy()
        agg.run_iteration()
        torch.cuda.synchronize()
        st, ob, path = b.status.cpu().numpy(), b.obj.cpu().numpy(), b.int_path.cpu().numpy()
        assert not (path & L.PATH_APPROX_MASK).any(), np.flatnonzero(path & L.PATH_APPROX_MASK)[:10]
        n_big = int(((path >> 18) & 1).sum())
        print(f"t={t}: {int((st == 0).sum())} optimal, {n_big} through the big launch, 0 approximate")
        pick = _sample(rng, st, homes, 5)
        _check_sample(homes, oat, ghi, tou, rp, t, prev_vals, prev_fc, noise, st, ob, b.vals.cpu().numpy(),
                      b.fc.cpu().numpy(), pick, path=path, fallback_gaps=[], approx_bound=1e-9)
