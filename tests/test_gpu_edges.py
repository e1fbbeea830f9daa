"""Edge cases of the device path (run_iteration over shards, mpc_calc.py:24-98 per home):

* an empty shard (more ranks than homes) is a no-op whose sums are zero;
* ragged shards (world does not divide the community, world > homes) reproduce the single
  batch bit for bit -- every home's answer depends only on its own inputs and global index;
* the longest horizon of the configs' ranges (24 h at 15-min steps, H = 96: the LDS layout
  whose battery recovery arrays no longer fit in the dead DP labels) gives answers that
  satisfy the reference model assembled by the oracle (violation <= 1e-5, integral duties,
  objective = c @ x), every home type.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _community(n, hours, steps, seed=12, month=7):
    from dragg_amd.community import synthetic_homes, synthetic_weather
    dt = 4
    sim_hours = math.ceil(steps / dt)
    days = math.ceil((sim_hours + hours + 2) / 24) + 1
    homes = synthetic_homes(n, seed=seed, days=days, dt=dt, horizon_hours=hours)
    oat, ghi, tou = synthetic_weather(days, dt, sim_hours, seed=3, month=month)
    return homes, oat, ghi, tou


def test_empty_shard_is_noop(gpu):
    import torch
    from dragg_amd.aggregator import DeviceAggregator
    homes, oat, ghi, tou = _community(2, 6, 2)
    agg = DeviceAggregator(homes, oat, ghi, tou, 0, 2, reward_price=[0.0], seed=12, rank=2, world=3)
    assert agg.batch.N == 0 and agg.batch.H == 24
    for _ in range(2):
        agg.run_iteration()
        assert agg.collect_data(defer=True).tolist() == [0.0, 0.0, 0.0]   # this shard's sums
    assert tuple(agg.batch.season_noise(0).shape) == (24, 0)
    torch.cuda.synchronize()
    assert agg.hist.shape[-1] == 0 and agg.summary()["p_grid_aggregate"] == [0.0, 0.0]


@pytest.mark.parametrize("world", [4, 16])
def test_ragged_shards_bitexact(gpu, world):
    import torch
    from dragg_amd.aggregator import DeviceAggregator
    n, steps = 13, 3
    homes, oat, ghi, tou = _community(n, 6, steps)
    full = DeviceAggregator(homes, oat, ghi, tou, 0, steps, reward_price=[0.0], seed=12)
    parts = [DeviceAggregator(homes, oat, ghi, tou, 0, steps, reward_price=[0.0], seed=12, rank=r, world=world)
             for r in range(world)]
    assert sorted(len(p.index) for p in parts)[-1] - sorted(len(p.index) for p in parts)[0] == 1
    sums = torch.zeros((steps, 3), dtype=torch.float64, device=gpu)
    for t in range(steps):
        full.run_iteration()
        for p in parts:
            p.run_iteration()
            sums[t] += p.collect_data(defer=True)
        full.collect_data()
    torch.cuda.synchronize()
    joined = torch.empty_like(full.hist)
    for r, p in enumerate(parts):
        joined[:, :, r::world] = p.hist
    assert torch.equal(torch.nan_to_num(full.hist, 7.0), torch.nan_to_num(joined, 7.0))
    # the shard sums add up to the community's (same values, a different summation order)
    assert torch.allclose(sums, full.agg_hist, rtol=1e-12, atol=1e-9)


def test_long_horizon_answers_satisfy_reference_model(gpu):
    import torch
    from oracle import mpc as M
    from dragg_amd import _lib as L
    from dragg_amd.aggregator import DeviceAggregator
    from tests.test_gpu_fullsize import _hash_dict
    from tests.test_gpu_parity import _expand
    n, hours, steps = 48, 24, 2
    homes, oat, ghi, tou = _community(n, hours, steps)
    agg = DeviceAggregator(homes, oat, ghi, tou, 0, steps, reward_price=[0.0], seed=12)
    b = agg.batch
    assert b.H == 96
    types = np.array([h["type"] for h in homes])
    seen, worst = set(), 0.0
    for t in range(steps):
        pv, pf = b.vals.cpu().numpy().copy(), b.fc.cpu().numpy().copy()
        noise = b.season_noise(t).cpu().numpy()
        agg.run_iteration()
        torch.cuda.synchronize()
        st, obj = b.status.cpu().numpy(), b.obj.cpu().numpy()
        vals, fc = b.vals.cpu().numpy(), b.fc.cpu().numpy()
        assert not np.isin(st, [L.ST_ERR_MISSING, L.ST_ERR_PARSE]).any()
        opt = np.flatnonzero(st == L.ST_OPTIMAL)
        assert len(opt) >= n // 2, np.bincount(st)
        for i in opt[::2]:
            hc = M.home_const(homes[i])
            draw, _, _ = M.water_draws(hc, t)
            T0, Tw0, E0, _ = M.initial_conditions(hc, t, _hash_dict(pv, pf, i) if t else {}, draw)
            o, g, tt = M.env_slice(oat, ghi, tou, 0, t, hc.H)
            si = M.StepInput(t=t, T0=T0, Tw0=Tw0, E0=E0, oat=o, ghi=g, price=M.total_price(tt, [0.0], hc.H),
                             draw=draw, winter=M.season_is_winter(o, noise[:, i]))
            P, x = _expand(hc, si, vals[:, i], fc[:, :, i], hc.S)
            ve = np.abs(P["A_eq"] @ x - P["b_eq"]).max()
            vu = (P["A_ub"] @ x - P["b_ub"]).max()
            worst = max(worst, ve, vu)
            assert ve <= 1e-5 and vu <= 1e-5, (t, i, types[i], ve, vu)
            duties = x[P["integrality"] == 1]
            assert np.array_equal(duties, np.round(duties)), (t, i)
            assert abs(P["c"] @ x - obj[i]) <= 1e-8 * max(1, abs(obj[i])), (t, i)
            seen.add(types[i])
    assert seen == {"base", "pv_only", "battery_only", "pv_battery"}, seen
    print(f"H = 96: worst violation {worst:.2e}")
