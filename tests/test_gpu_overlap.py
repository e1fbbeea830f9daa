"""Lag mode (dragg_mpc_step_main / _side, DeviceAggregator(overlap=True)): a home whose chain needs
the exact step-function DP finishes that step on a side stream while the other homes go on with
their next steps (run_rbo_mpc has no feedback between homes, aggregator.py:757-778).  Every home's
solve is the same code on the same inputs, so the run must be bit-identical to the serial one:
the history rows, statuses, collect_data sums and the final hash arrays -- on the bench community
(its narrow-set home 7519 takes the step-function DP at steps 36-60) and on the 8-way shard that
holds that home."""
import math

import numpy as np
import pytest
import torch

from dragg_amd.aggregator import DeviceAggregator
from dragg_amd.community import synthetic_homes, synthetic_weather

pytestmark = pytest.mark.gpu

STEPS = 64


def _bench_community():
    dt, hh = 4, 12
    days = math.ceil((math.ceil(STEPS / dt) + hh + 2) / 24) + 1
    homes = synthetic_homes(10000, seed=12, days=days, dt=dt, horizon_hours=hh)
    oat, ghi, tou = synthetic_weather(days, dt, math.ceil(STEPS / dt), seed=3, month=7)
    return homes, oat, ghi, tou


def _run(overlap, rank, world, com, adaptive=False, keep_history=True, steps=STEPS):
    homes, oat, ghi, tou = com
    agg = DeviceAggregator(homes, oat, ghi, tou, 0, steps, reward_price=[0.0], seed=12, rank=rank, world=world,
                           overlap=overlap, adaptive=adaptive, keep_history=keep_history)
    agg.world = 1                              # one GPU: the shard's own sums, no collectives
    assert agg.overlap == overlap and agg.adaptive == (overlap and adaptive)
    assert (agg.ring is not None) == (overlap and not keep_history)
    for _ in range(steps):
        agg.run_iteration()
        agg.collect_data(defer=True)
    agg.reduce_history()
    torch.cuda.synchronize()
    return agg


def _bits(t):
    return t.cpu().contiguous().view(torch.int64).numpy()


@pytest.fixture(scope="module")
def com():
    return _bench_community()


@pytest.mark.parametrize("rank,world", [(0, 1), (7519 % 8, 8)])
def test_overlap_is_bit_identical_to_serial(com, rank, world, gpu):
    a = _run(False, rank, world, com)
    b = _run(True, rank, world, com)
    lists = b.batch.lag["lists"].cpu().numpy()
    n = b.batch.N
    skipped, narrow = lists[:STEPS, 0, n], lists[:STEPS, 1, n]
    print(f"rank {rank} of {world}: chains to the step-function DP per step {narrow.nonzero()[0].tolist()}, "
          f"homes left to the side stream {int(skipped.sum())} home-steps")
    assert narrow.sum() > 0                    # the community has step-function chains ...
    assert skipped.sum() > 0                   # ... and the side stream ran behind (homes skipped)
    assert np.array_equal(_bits(a.hist), _bits(b.hist))
    assert np.array_equal(a.status_hist.cpu().numpy(), b.status_hist.cpu().numpy())
    assert np.array_equal(_bits(a.agg_hist), _bits(b.agg_hist))
    assert np.array_equal(_bits(a.batch.vals), _bits(b.batch.vals))
    assert np.array_equal(_bits(a.batch.fc_store), _bits(b.batch.fc_store))
    # the lagged sums are collect_data's on the final state too
    assert np.array_equal(_bits(b.agg_hist[STEPS - 1]), _bits(b.batch.aggregate()))


@pytest.mark.parametrize("adaptive,keep_history", [(True, True), (False, False), (True, False)])
def test_adaptive_start_and_history_ring_bit_identical(com, adaptive, keep_history, gpu):
    """The adaptive start (serial steps until one lists a step-function chain, then lag mode) and lag mode
    without the history (a ring of 16 history rows, the sums taken on the side stream after each step's side
    pass) give the serial run's results bit for bit, on the 8-way shard holding home 7519."""
    rank, world = 7519 % 8, 8
    a = _run(False, rank, world, com)
    b = _run(True, rank, world, com, adaptive=adaptive, keep_history=keep_history)
    if adaptive:
        assert b.lag_from is not None and 36 < b.lag_from <= 36 + b.FLAG_LAG + 1, b.lag_from
    assert np.array_equal(a.status_hist.cpu().numpy(), b.status_hist.cpu().numpy())
    assert np.array_equal(a.path_hist.cpu().numpy(), b.path_hist.cpu().numpy())
    assert np.array_equal(_bits(a.agg_hist), _bits(b.agg_hist))
    assert np.array_equal(_bits(a.batch.vals), _bits(b.batch.vals))
    assert np.array_equal(_bits(a.batch.fc_store), _bits(b.batch.fc_store))
    if keep_history:
        assert np.array_equal(_bits(a.hist), _bits(b.hist))
    c = b.approx_counts()
    assert c["approx_solves"] == 0 and c["step_dp_solves"] > 0


def test_seven_days_ring_lag_bit_identical(com, gpu):
    """configs[3]'s shape (a 7-day run at 15-min steps without the per-step history, keep_history=False) in
    lag mode on the ring, at reduced N: the 8-way shard of the bench community holding home 7519, its weather
    and water draws repeated day after day (so its step-function chains of day 1 recur), 672 steps:
    bit-identical to serial steps."""
    import copy
    steps, reps = 672, 9
    homes, oat, ghi, tou = com
    homes = copy.deepcopy(homes)
    for h in homes:
        h["wh"]["draw_sizes"] = list(h["wh"]["draw_sizes"][:24]) * (reps * len(h["wh"]["draw_sizes"]) // 24)
    day = 24 * 4
    com7 = (homes, list(oat[:day]) * reps * 2, list(ghi[:day]) * reps * 2, list(tou[:day]) * reps * 2)
    rank, world = 7519 % 8, 8
    a = _run(False, rank, world, com7, keep_history=False, steps=steps)
    b = _run(True, rank, world, com7, keep_history=False, steps=steps)
    assert b.ring is not None and b.ring.shape[0] == 16
    assert np.array_equal(a.status_hist.cpu().numpy(), b.status_hist.cpu().numpy())
    assert np.array_equal(a.path_hist.cpu().numpy(), b.path_hist.cpu().numpy())
    assert np.array_equal(_bits(a.agg_hist), _bits(b.agg_hist))
    assert np.array_equal(_bits(a.batch.vals), _bits(b.batch.vals))
    assert np.array_equal(_bits(a.batch.fc_store), _bits(b.batch.fc_store))
    steps_dp = ((a.path_hist.cpu().numpy() & (1 << 15)) != 0).sum(axis=1)
    print(f"7 days: step-function solves per day {[int(steps_dp[d * 96:(d + 1) * 96].sum()) for d in range(7)]}")
    assert steps_dp.sum() > 0
