"""Multi-rank glue of the device-resident driver on CPU with gloo (world size 2).

The solver is replaced by a stand-in batch (the HIP solver needs a GPU); what is tested is
the sharding (strided shards: rank r holds homes r, r + world, ..., keyed by the global index)
and the per-step all-reduce of [agg_load, forecast_load, agg_cost] (aggregator.py:751-753).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dragg_amd.aggregator import DeviceAggregator, shard_index


class FakeBatch:
    """Deterministic stand-in: each home contributes (index+1)*t to the three sums."""

    def __init__(self, homes, *a, home_offset=0, home_stride=1, device=None, **kw):
        self.N, self.H = len(homes), 4
        self.off, self.stride = home_offset, home_stride
        self.gidx = home_offset + home_stride * torch.arange(self.N, dtype=torch.float64)   # global indices
        self.t = 0
        self.status = torch.zeros(self.N, dtype=torch.int32)
        self.iters = torch.zeros(self.N, dtype=torch.int32)
        self.types_host = None

    def step(self, t, noise=None, hist=None):
        self.t = t
        if hist is not None:
            hist.zero_()
            hist[0] = self.gidx

    def aggregate(self):
        s = float((self.gidx + 1).sum()) * self.t
        return torch.tensor([s, 2 * s, 3 * s], dtype=torch.float64)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, steps, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    homes = [{"name": f"h{i}"} for i in range(n)]
    agg = DeviceAggregator(homes, None, None, None, 0, steps, rank=rank, world=world,
                           device=torch.device("cpu"), batch_cls=FakeBatch)
    out = []
    for _ in range(steps):
        agg.run_iteration()
        out.append(agg.collect_data().tolist())
    # run_rbo_mpc's deferred sums: local per step, community-wide after reduce_history()
    agg2 = DeviceAggregator(homes, None, None, None, 0, steps, rank=rank, world=world,
                            device=torch.device("cpu"), batch_cls=FakeBatch)
    local = []
    for _ in range(steps):
        agg2.run_iteration()
        local.append(agg2.collect_data(defer=True).tolist())
    deferred = agg2.reduce_history().tolist()
    q.put((rank, agg.index.tolist(), out, agg.hist[:, 0, :].tolist(), local, deferred))
    dist.destroy_process_group()


@pytest.mark.parametrize("n,world", [(7, 2), (10, 2), (2, 3)])
def test_two_rank_allreduce_and_sharding(n, world):
    """(2, 3): more ranks than homes, rank 2's shard is empty and still joins every collective."""
    steps = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    # strided, disjoint, covering shards
    assert sorted(sum((r[1] for r in res), [])) == list(range(n)) and res[1][1] == list(range(1, n, world))
    total = sum(range(1, n + 1))
    for rank, idx, out, hist, local, deferred in res:
        mine = sum(i + 1 for i in idx)
        for t, v in enumerate(out):
            assert v == [total * t, 2 * total * t, 3 * total * t]      # all-reduced sums, every rank
            assert local[t] == [mine * t, 2 * mine * t, 3 * mine * t]  # deferred: this shard's
            assert deferred[t] == v                                    # one reduction at the end
        assert hist[0] == list(map(float, idx))                        # global home indices


def test_shard_index_cover():
    for n in range(0, 40):
        for w in (1, 2, 3, 8):
            parts = [shard_index(n, r, w).tolist() for r in range(w)]
            assert sorted(sum(parts, [])) == list(range(n))
            assert max(map(len, parts)) - min(map(len, parts)) <= 1          # balanced counts


# ------------------------------------------------------------------ the runner over 2 ranks
class HashBatch(FakeBatch):
    """Stand-in that writes every hash field: value = global home index + 100 t."""

    def step(self, t, noise=None, hist=None):
        self.t = t
        if hist is not None:
            v = self.gidx + 100.0 * t
            hist.copy_(v.expand_as(hist))


def _runner_worker(rank, world, port, root, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dragg_amd.runner import Aggregator
    a = Aggregator(data_dir=os.path.join(root, "data"), outputs_dir=os.path.join(root, "outputs"),
                   device=torch.device("cpu"), batch_cls=StateBatch)
    path = a.run()
    q.put((rank, a.dev.index.tolist(), path))
    dist.destroy_process_group()


@pytest.mark.parametrize("checkpoint", ["daily", "hourly"])
def test_runner_two_ranks_gathers_history(tmp_path, checkpoint):
    """Two ranks each solve a strided shard; rank 0 gathers the hash history and writes
    results.json with every home's series in community order.  Hourly checkpoints (every 4
    steps) gather the history in three increments."""
    import json
    from tests import fixtures as F
    from tests.test_runner import _synthetic_data
    data = tmp_path / "data"
    data.mkdir()
    _synthetic_data(str(data))
    params = dict(n=7, batt=2, pv=2, pvb=1, start="2015-01-01 00", end="2015-01-01 03", dt=4, horizon=2,
                  action_horizon=2, seed=3)
    with open(data / "config.toml", "w") as f:
        f.write(F.config_text(params).replace('checkpoint_interval = "daily"', f'checkpoint_interval = "{checkpoint}"'))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_runner_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res[1][2] is None and res[0][1] == [0, 2, 4, 6] and res[1][1] == [1, 3, 5]
    with open(res[0][2]) as f:
        out = json.load(f)
    names = [k for k in out if k != "Summary"]
    assert len(names) == 7
    T = 12
    for i, n in enumerate(names):
        assert out[n]["p_grid_opt"] == [i + 100.0 * t for t in range(T)]
    assert out["Summary"]["p_grid_aggregate"] == [sum(i + 100.0 * t for i in range(7)) for t in range(T)]


class StateBatch(HashBatch):
    """HashBatch with the solver state a checkpoint holds (hash arrays, reward price)."""

    def __init__(self, homes, *a, **kw):
        super().__init__(homes, *a, **kw)
        self.vals = torch.zeros((19, self.N), dtype=torch.float64)
        self.fc = torch.zeros((15, 4, self.N), dtype=torch.float64)
        self.rp = torch.zeros(1, dtype=torch.float64)

    def step(self, t, noise=None, hist=None):
        super().step(t, noise, hist)
        self.vals += t + self.gidx                 # state that depends on every previous step
        self.fc[0] = self.vals[0]

    def set_reward_price(self, rp):
        self.rp = rp.clone()


def test_checkpoint_roundtrip(tmp_path):
    """save_state / load_state (CPU): a run resumed from a mid-run checkpoint ends in the state
    and histories of the uninterrupted run."""
    from dragg_amd.aggregator import DeviceAggregator
    homes = [{"name": f"h{i}"} for i in range(5)]
    kw = dict(num_timesteps=6, device=torch.device("cpu"), batch_cls=StateBatch)
    full = DeviceAggregator(homes, [0.0], [0.0], [0.0], **kw)
    full.set_reward_price([0.25])
    full.run_baseline()
    part = DeviceAggregator(homes, [0.0], [0.0], [0.0], **kw)
    part.set_reward_price([0.25])
    part.run_baseline(steps=3)
    path = part.save_state(str(tmp_path / "state.pt"))
    res = DeviceAggregator(homes, [0.0], [0.0], [0.0], **kw)
    assert res.load_state(path) == 3
    assert float(res.batch.rp[0]) == 0.25
    res.run_baseline()
    assert torch.equal(res.batch.vals, full.batch.vals) and torch.equal(res.batch.fc, full.batch.fc)
    assert torch.equal(res.hist, full.hist) and torch.equal(res.agg_hist, full.agg_hist)
    other = DeviceAggregator(homes, [0.0], [0.0], [0.0], rank=1, world=2, **kw)
    with pytest.raises(ValueError):
        other.load_state(path)


# ------------------------------------------------------------------ resume / errors over 2 ranks
class ErrBatch(StateBatch):
    """StateBatch whose global home 3 hits the reference's KeyError path at t = 2."""

    def step(self, t, noise=None, hist=None):
        super().step(t, noise, hist)
        from dragg_amd import _lib as L
        self.status = torch.where((self.gidx == 3) & (t >= 2), L.ST_ERR_MISSING, 0).to(torch.int32)


def _resume_worker(rank, world, port, root, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    homes = [{"name": f"h{i}"} for i in range(6)]
    kw = dict(num_timesteps=6, rank=rank, world=world, device=torch.device("cpu"), batch_cls=StateBatch)
    out = {}
    # a crash between the two ranks' saves: rank 0 checkpointed step 3, rank 1 still holds step 2
    a = DeviceAggregator(homes, [0.0], [0.0], [0.0], **kw)
    for _ in range(2 + (rank == 0)):             # (no reduce_history: the ranks never met)
        a.run_iteration()
        a.collect_data(defer=True)
    path = os.path.join(root, f"state-{rank}.pt")
    a.save_state(path)
    b = DeviceAggregator(homes, [0.0], [0.0], [0.0], **kw)
    try:
        b.agree(b.load_state(path), "the checkpoint timestep")
        out["resume"] = "ok"
    except RuntimeError as e:
        out["resume"] = str(e)
    # the same checkpoint under another seed is another run's
    c = DeviceAggregator(homes, [0.0], [0.0], [0.0], seed=99, **kw)
    try:
        c.load_state(path)
        out["seed"] = "ok"
    except ValueError as e:
        out["seed"] = "refused"
    # rank 1's checkpoint is another run's (refused) while rank 0's loads: both raise, none hangs
    # in the collective (resume agrees on -1 for a refused checkpoint)
    e = DeviceAggregator(homes, [0.0], [0.0], [0.0], **(kw | {"seed": 99 if rank == 1 else 0}))
    try:
        e.resume(path)
        out["foreign"] = "ok"
    except ValueError as ex:
        out["foreign"] = "own: " + str(ex)
    except RuntimeError as ex:
        out["foreign"] = str(ex)
    # rank 0's checkpoint file is garbage (torch.load(weights_only=True) raises
    # pickle.UnpicklingError): rank 0 raises that, rank 1 the disagreement -- neither hangs
    junk = os.path.join(root, f"junk-{rank}.pt")
    with open(junk, "wb") as f:
        f.write(b"not a checkpoint" if rank == 0 else open(path, "rb").read())
    g = DeviceAggregator(homes, [0.0], [0.0], [0.0], **kw)
    try:
        g.resume(junk)
        out["garbage"] = "ok"
    except RuntimeError as ex:
        out["garbage"] = str(ex)
    except Exception as ex:
        out["garbage"] = "own: " + type(ex).__name__
    # a crashing home on rank 1 only: both ranks raise the same KeyError together
    kw["batch_cls"] = ErrBatch
    d = DeviceAggregator(homes, [0.0], [0.0], [0.0], **kw)
    d.run_baseline(steps=4)
    try:
        d.check_errors()
        out["err"] = "ok"
    except KeyError as e:
        out["err"] = str(e)
    q.put((rank, out))
    dist.destroy_process_group()


def test_two_ranks_resume_disagreement_and_errors_raise_on_every_rank(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_resume_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for rank in (0, 1):
        assert "ranks disagree" in res[rank]["resume"] and "from 2 to 3" in res[rank]["resume"]
        assert res[rank]["seed"] == "refused"
        assert "home h3 at timestep 2" in res[rank]["err"]
    assert res[1]["foreign"].startswith("own: ") and "another run" in res[1]["foreign"]
    assert "ranks disagree" in res[0]["foreign"]
    assert res[0]["garbage"] == "own: UnpicklingError", res[0]["garbage"]
    assert "ranks disagree" in res[1]["garbage"]
