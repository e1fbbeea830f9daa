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


def _run(overlap, rank, world, com):
    homes, oat, ghi, tou = com
    agg = DeviceAggregator(homes, oat, ghi, tou, 0, STEPS, reward_price=[0.0], seed=12, rank=rank, world=world,
                           overlap=overlap)
    agg.world = 1                              # one GPU: the shard's own sums, no collectives
    assert agg.overlap == overlap
    for _ in range(STEPS):
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
