"""The step-function DP's capacity path (mpc_kernel.hip, DM_NARROW; reference: the MILP solve it
replaces, mpc_calc.py:447-455).  A chain whose value functions outgrow the pool (DRAGG_STEP_POOL_CAP
shrinks it here) or pass the per-chain work bound (DRAGG_STEP_WORK_CAP) keeps the bucketed schedule
the mid / big launch handed over -- a feasible schedule whose cost bounded the DP -- and is flagged
approximate (int_path reason 6) instead of silently changing the answer.  The bench community's
narrow-set home 7519 takes the step-function DP at step 36 (tests/test_gpu_overlap.py)."""
import math
import os

import numpy as np
import pytest
import torch

from dragg_amd import _lib as L
from dragg_amd.aggregator import DeviceAggregator
from dragg_amd.community import synthetic_homes, synthetic_weather

pytestmark = pytest.mark.gpu

HOME, STEP = 7519, 36


@pytest.fixture(scope="module")
def at_step():
    dt, hh, steps = 4, 12, STEP + 1
    gen = 64                                    # the community and weather of tests/test_gpu_overlap.py
    days = math.ceil((math.ceil(gen / dt) + hh + 2) / 24) + 1
    homes = synthetic_homes(10000, seed=12, days=days, dt=dt, horizon_hours=hh)
    oat, ghi, tou = synthetic_weather(days, dt, math.ceil(gen / dt), seed=3, month=7)
    agg = DeviceAggregator(homes, oat, ghi, tou, 0, steps, reward_price=[0.0], seed=12, keep_history=False)
    for _ in range(STEP):
        agg.run_iteration()
    return agg, agg.snapshot()


def _step_with(agg, snap, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    L.reload_knobs()
    try:
        agg.restore(snap)
        agg.run_iteration()
        torch.cuda.synchronize()
        b = agg.batch
        return (int(b.status[HOME]), float(b.obj[HOME]), int(b.int_path[HOME]),
                b.fc[:, :, HOME].cpu().numpy().copy(), b.params[:, HOME].cpu().numpy(),
                agg.approx_counts(STEP, STEP + 1)["approx_solves"])
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        L.reload_knobs()


@pytest.mark.parametrize("env", [{"DRAGG_STEP_POOL_CAP": "64"}, {"DRAGG_STEP_WORK_CAP": "1"}])
def test_capacity_path_keeps_the_bucketed_schedule_flagged(at_step, env, gpu):
    agg, snap = at_step
    st0, obj0, path0, _, _, n0 = _step_with(agg, snap, {})
    assert st0 == L.ST_OPTIMAL and path0 & L.PATH_STEPS and not path0 & L.PATH_APPROX_MASK   # exact by default
    assert n0 == 0                                                # the step's solves: none approximate
    st, obj, path, fc, par, n = _step_with(agg, snap, env)
    assert st == L.ST_OPTIMAL and path & L.PATH_STEPS
    assert path & 2 and (path >> 8) & 0xF == 6, hex(path)       # the tank chain: approximate, reason 6
    assert n == 1                                                 # ... and counted (DeviceAggregator.approx_counts)
    assert obj >= obj0 - 1e-9 * max(1.0, abs(obj0))               # never below the exact optimum
    assert obj <= obj0 + 0.25 * abs(obj0) + 1e-6                  # the bucketed schedule, not an arbitrary one
    # the kept schedule is feasible: integral duties in [0, S], the tank trajectory inside its box
    H = agg.batch.H
    w = fc[L.K["wh_heat_on_opt"]] * agg.batch.S
    assert np.allclose(w, np.round(w), atol=1e-9) and w.min() >= -1e-9 and w.max() <= agg.batch.S + 1e-9
    tw = fc[L.K["temp_wh_ev_opt"]]
    lo, hi = par[L.P["TWMIN"]], par[L.P["TWMAX"]]
    assert np.all(tw[1:H] >= lo - 1e-6) and np.all(tw[1:H] <= hi + 1e-6)
    # a bound of the default size solves the same step exactly again
    st2, obj2, path2, _, _, _ = _step_with(agg, snap, {"DRAGG_STEP_POOL_CAP": str(1 << 20)})
    assert (st2, obj2, path2) == (st0, obj0, path0)
