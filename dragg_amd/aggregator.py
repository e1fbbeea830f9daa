"""Device-resident replacement of the aggregator's per-timestep loop.

Reference: `Aggregator.run_baseline / run_iteration / collect_data`
(aggregator.py:711-778).  There, every timestep forks a process pool, pickles each
MPCCalc to a worker, round-trips ~400 redis fields per home and sums three fields per
home on the host.  Here the community's state never leaves the GPU:

* one `dragg_mpc_step` launch solves and advances every home of this rank's shard;
* `dragg_mpc_aggregate` reduces agg_load / forecast_load / agg_cost on device and, with
  more than one rank, a single 24-byte RCCL all-reduce (torch.distributed, backend
  "nccl" = RCCL over xGMI) combines the shards -- the only cross-GPU traffic;
* the per-step hash fields are appended to an on-device history (the
  `collected_data` lists), converted to the results.json layout only on request.

Homes are sharded by stride (rank r solves global homes r, r + world, r + 2 world, ...: every
shard carries the community's type mix); the season-noise stream is keyed by the GLOBAL home
index, so results do not depend on the shard layout.
"""
import os
import zlib

import numpy as np
import torch

from . import _lib as L
from .mpc import MPCBatch


def shard_index(n, rank, world):
    """Global indices of the homes a rank solves: every world-th home from `rank`.  Strided
    rather than contiguous so that every shard carries the community's type mix (the
    reference lists homes grouped by type, aggregator.py:425-587, and battery homes cost more
    per solve): the ranks finish a step together."""
    return np.arange(rank, n, world)


class DeviceAggregator:
    def __init__(self, homes, oat, ghi, tou, start_index=0, num_timesteps=96, reward_price=(0.0,),
                 int_mode="round", seed=0, rank=0, world=1, group=None, keep_history=True,
                 max_iter=4000, check_every=10, device=None, batch_cls=MPCBatch, exact=False, overlap=False,
                 adaptive=False, ring=16):
        self.rank, self.world, self.group = rank, world, group
        self.seed = int(seed)
        # identifies the community a checkpoint belongs to (load_state refuses another one's)
        self.names_crc = zlib.crc32("\x00".join(str(h.get("name", i)) for i, h in enumerate(homes)).encode())
        self.index = shard_index(len(homes), rank, world)
        self.all_homes = homes
        self.homes = [homes[i] for i in self.index]
        dev = device or torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        # batch_cls is injectable only so the multi-rank glue can be exercised with gloo on
        # CPU (tests/test_distributed.py); the solver itself is MPCBatch (HIP, no fallback).
        self.batch = batch_cls(self.homes, oat, ghi, tou, start_index, reward_price, int_mode=int_mode,
                              seed=seed, home_offset=rank, home_stride=world, max_iter=max_iter, check_every=check_every,
                              device=dev, template_home=homes[0] if homes else None,
                              **({"exact": True} if exact else {}))
        self.num_timesteps = num_timesteps
        self.timestep = 0
        n = self.batch.N
        self.hist = (torch.full((num_timesteps, L.NVAL, n), float("nan"), dtype=torch.float64, device=dev)
                     if keep_history else None)
        self.agg_hist = torch.zeros((num_timesteps, 3), dtype=torch.float64, device=dev)
        self.status_hist = torch.zeros((num_timesteps, n), dtype=torch.int32, device=dev)
        # every solve's int_path bits (dragg_mpc_out.int_path): which solves kept an approximate schedule
        # (bits 0-11, approx_counts) -- the reference's solve is exact up to GLPK's gap (mpc_calc.py:447-451)
        self.path_hist = torch.zeros((num_timesteps, n), dtype=torch.int32, device=dev)
        self._deferred = []          # steps whose agg_hist row holds this rank's sums only
        # overlap (lag mode, MPCBatch.enable_lag): a home whose chain needs the slow step-function DP
        # finishes that step on a side stream while the others go on (run_rbo_mpc has no feedback
        # between homes, aggregator.py:757-778); its results land in the step's own history rows later,
        # so the deferred sums are taken from those rows once the side stream has drained.  Without the
        # history (keep_history=False, configs[3]: 100k homes x 672 steps) the steps write a ring of
        # `ring` history rows instead, and the side stream sums row t right after step t's side pass (the
        # main pass of step t + ring waits for that).  Keyed season noise; int_mode round.
        self.overlap = (bool(overlap) and int_mode in ("round", "fail") and n > 0 and hasattr(self.batch, "enable_lag"))
        self.ring = None
        if self.overlap:
            if self.hist is None:
                R = max(2, min(int(ring), num_timesteps))
                self.ring = torch.full((R, L.NVAL, n), float("nan"), dtype=torch.float64, device=dev)
                self.batch.enable_lag(ring=R)
            else:
                self.batch.enable_lag()
        self._unsummed = []          # lag-mode steps whose agg_hist row is not computed yet
        # adaptive start (overlap): serial steps -- no side-stream launches at all -- until a step hands a
        # chain to the step-function DP (int_path bit 15, read back asynchronously, the host kept at most
        # FLAG_LAG steps ahead of the GPU), lag mode from the next step the host enqueues
        self.adaptive = self.overlap and bool(adaptive)
        self._lagging = self.overlap and not self.adaptive
        if self.adaptive:
            K = self.FLAG_LAG + 2
            pin = torch.cuda.is_available() and dev.type == "cuda"
            self._flag_host = torch.zeros(K, dtype=torch.int32, pin_memory=pin)
            self._flag_ev = [torch.cuda.Event() if pin else None for _ in range(K)]
            self._flag_step = [-1] * K
            # the flag of a step is reduced and copied on a stream of its own, from the step's path_hist row
            # (written once): the main stream's steps go on with no reduction kernels or device-to-host copy
            # between them (on the main stream those cost +3.8 % per step against serial steps, round 6)
            self._flag_stream = torch.cuda.Stream(device=dev) if pin else None
            self._flag_src = [torch.cuda.Event() if pin else None for _ in range(K)]
            self.lag_from = None             # the first step run in lag mode

    FLAG_LAG = 2                 # adaptive start: steps the host may run ahead of the last flag it reads

    def _lag_now(self, t):
        """Adaptive start: has a step the host can see (<= t - FLAG_LAG, waited for) listed a step-function
        chain?  Then this and every later step runs in lag mode."""
        if self._lagging:
            return True
        K = len(self._flag_step)
        s = t - self.FLAG_LAG
        if s >= 0 and self._flag_step[s % K] == s:
            ev = self._flag_ev[s % K]
            if ev is not None:
                ev.synchronize()
            if int(self._flag_host[s % K]):
                self._lagging = True
                self.lag_from = t
        return self._lagging

    def _flag(self, t):
        """After a serial step t: did it hand a chain to the step-function DP?  (device -> pinned host, async,
        on the flag stream after the step's path_hist row is written)"""
        K = len(self._flag_step)
        if self._flag_stream is None:
            f = ((self.path_hist[t] & L.PATH_STEPS) != 0).any().to(torch.int32)
            self._flag_host[t % K:t % K + 1].copy_(f.reshape(1))
        else:
            src = self._flag_src[t % K]
            src.record()                                   # the main stream, after the path_hist[t] copy
            with torch.cuda.stream(self._flag_stream):
                self._flag_stream.wait_event(src)
                f = ((self.path_hist[t] & L.PATH_STEPS) != 0).any().to(torch.int32)
                self._flag_host[t % K:t % K + 1].copy_(f.reshape(1), non_blocking=True)
                self._flag_ev[t % K].record(self._flag_stream)
        self._flag_step[t % K] = t

    # aggregator.py:711-726
    def run_iteration(self, noise=None):
        t = self.timestep
        hist = self.hist[t] if self.hist is not None else None
        if self.overlap and noise is None and self._lag_now(t):
            ring = self.ring is not None
            self.batch.step_lagged(t, self.ring[t % self.ring.shape[0]] if ring else hist, self.status_hist[t],
                                   path_row=self.path_hist[t], sums_row=self.agg_hist[t] if ring else None)
        else:
            self.batch.step(t, noise=noise, hist=hist)
            self.status_hist[t].copy_(self.batch.status, non_blocking=True)
            if hasattr(self.batch, "int_path"):
                self.path_hist[t].copy_(self.batch.int_path, non_blocking=True)
            if self.adaptive and noise is None:
                self._flag(t)
        self.timestep += 1

    def approx_counts(self, lo=0, hi=None):
        """Solves of steps [lo, hi) (default: all so far) by int_path: {"approx_solves": solves that
        kept an approximate integer schedule (int_path bits 0-11: reason 3, an RL-priced front past
        2,048 labels without DRAGG_FLAG_EXACT; reason 6, the step-function DP past its pool or work
        bound), "step_dp_solves": solves by the exact step-function DP (bit 15), "later_launch_solves":
        solves finished by the mid / big / step-function launches (bit 12)}, over every rank."""
        self.drain()
        hi = self.timestep if hi is None else hi
        p = self.path_hist[lo:hi]
        v = torch.stack([((p & L.PATH_APPROX_MASK) != 0).sum(), ((p & L.PATH_STEPS) != 0).sum(),
                         ((p & L.PATH_SECOND) != 0).sum()]).to(torch.int64)
        if self.world > 1:
            torch.distributed.all_reduce(v, group=self.group)
        a, s, m = (int(x) for x in v.cpu().tolist())
        return {"approx_solves": a, "step_dp_solves": s, "later_launch_solves": m}

    def approx_solves(self):
        """[(timestep, global home index, int_path)] of this shard's approximate solves so far."""
        self.drain()
        p = self.path_hist[:self.timestep].cpu().numpy()
        return [(int(t), int(self.index[i]), int(p[t, i])) for t, i in np.argwhere((p & L.PATH_APPROX_MASK) != 0)]

    def drain(self):
        """Overlap mode: wait (in stream order) for the side stream, then fill the sums of the steps
        that were deferred from their history rows.  Everything a step wrote is readable after this."""
        d = getattr(self.batch, "drain", None)     # (stand-in batches of the CPU tests have none)
        if d is not None:
            d()
        if self._unsummed:
            lo, hi = self._unsummed[0], self._unsummed[-1] + 1
            assert self._unsummed == list(range(lo, hi))
            self.agg_hist[lo:hi].copy_(self.batch.aggregate_rows(self.hist[lo:hi]))
            self._unsummed = []

    # aggregator.py:728-755 (sums only; the per-home series stay in self.hist)
    def collect_data(self, defer=False):
        """The step's [agg_load, forecast_load, agg_cost].  defer=True: nothing reads the
        community sums before the run ends (run_rbo_mpc has no feedback, aggregator.py:757-778),
        so this rank keeps its own sums and reduce_history() all-reduces every deferred step in
        one collective; the ranks then need not meet at every step."""
        t = self.timestep - 1
        if self.overlap and defer and self.batch.lag["next"] == self.timestep:
            # (lag mode: the lagging homes' fields of step t are not written yet; drain() sums the row --
            # with the history ring, the side stream already does, after the step's side pass)
            if self.ring is None:
                self._unsummed.append(t)
            if self.world > 1:
                self._deferred.append(t)
            return None
        self.drain()
        agg = self.batch.aggregate()
        if self.world > 1:
            if defer:
                self._deferred.append(t)
            else:
                torch.distributed.all_reduce(agg, group=self.group)
        self.agg_hist[t].copy_(agg)
        return agg

    def reduce_history(self):
        """All-reduce the deferred steps' sums (one RCCL call); agg_hist is then community-wide."""
        self.drain()
        if self._deferred:
            idx = torch.tensor(self._deferred, dtype=torch.long, device=self.agg_hist.device)
            rows = self.agg_hist.index_select(0, idx)
            torch.distributed.all_reduce(rows, group=self.group)
            self.agg_hist.index_copy_(0, idx, rows)
            self._deferred = []
        return self.agg_hist[:self.timestep]

    # aggregator.py:757-778
    def run_baseline(self, steps=None, noise_fn=None):
        steps = self.num_timesteps - self.timestep if steps is None else steps
        for _ in range(steps):
            self.run_iteration(noise_fn(self.timestep) if noise_fn else None)
            self.collect_data(defer=True)
        return self.reduce_history()

    # ------------------------------------------------------------------ RL reward-price path
    # (aggregator.py:664-675, 876-896).  A step reads exactly three things
    # that change between steps: the timestep, the hash arrays (vals, fc: the previous
    # solve, mpc_calc.py:264-289, 527-595) and the reward-price list.  A forecast rollout
    # therefore snapshots the hash arrays on device, solves ahead and puts them back.
    def set_reward_price(self, rp, src=0):
        """Broadcast the reward-price list decided on rank `src` (the RL agent's host) to every
        rank (one RCCL broadcast of action_horizon*dt fp64) and hand it to the solver."""
        t = torch.as_tensor(np.asarray(rp, dtype=float) if not torch.is_tensor(rp) else rp,
                            dtype=torch.float64).to(self.device).reshape(-1).contiguous()
        if self.world > 1:
            torch.distributed.broadcast(t, src=src, group=self.group)
        self.batch.set_reward_price(t)
        return t

    def snapshot(self):
        self.drain()
        return self.timestep, self.batch.vals.clone(), self.batch.fc.clone()

    def restore(self, snap):
        self.drain()
        t, vals, fc = snap
        self.timestep = t
        self.batch.vals.copy_(vals)
        self.batch.fc.copy_(fc)

    def forecast(self, steps, noise_fn=None):
        """Solve every home `steps` timesteps ahead under the current reward price without
        committing anything (no history, state restored): the community's [steps][agg_load,
        forecast_load, agg_cost], all-reduced once over the ranks.  The season-noise stream
        is keyed by (seed, home, t), so a rollout sees the draws the committed steps will."""
        snap = self.snapshot()
        out = torch.empty((steps, 3), dtype=torch.float64, device=self.device)
        try:
            for s in range(steps):
                t = self.timestep + s
                self.batch.step(t, noise=noise_fn(t) if noise_fn else None, hist=None)
                out[s].copy_(self.batch.aggregate())
        finally:
            self.restore(snap)
        if self.world > 1:
            torch.distributed.all_reduce(out, group=self.group)
        return out

    # ------------------------------------------------------------------ checkpoint / resume
    # The reference has no resume (aggregator.py:265-267, 768: a stopped run starts over); here a
    # checkpoint is the device state a step reads -- the hash arrays, the timestep, the reward
    # price -- plus the histories, one file per rank.  The season-noise stream is keyed by
    # (seed, home, t), so a resumed run continues bit for bit as if it had not stopped.
    def save_state(self, path):
        self.drain()
        t = self.timestep
        state = {"timestep": t, "rank": self.rank, "world": self.world, "n_local": int(self.batch.N),
                 "seed": self.seed, "num_timesteps": int(self.num_timesteps), "n_all": len(self.all_homes),
                 "names_crc": int(self.names_crc),
                 "vals": self.batch.vals.cpu(), "fc": self.batch.fc.cpu(),
                 "reward_price": self.batch.rp.cpu(),
                 "agg_hist": self.agg_hist[:t].cpu(), "status_hist": self.status_hist[:t].cpu(),
                 "path_hist": self.path_hist[:t].cpu(),
                 "deferred": torch.as_tensor(self._deferred, dtype=torch.long),
                 "hist": self.hist[:t].cpu() if self.hist is not None else None}
        tmp = path + ".tmp"
        torch.save(state, tmp)
        os.replace(tmp, path)                 # a crash mid-write leaves the previous checkpoint
        return path

    def load_state(self, path):
        """Resume from save_state's file (tensors only: loaded with weights_only=True)."""
        self.drain()
        st = torch.load(path, map_location="cpu", weights_only=True)
        if (st["rank"], st["world"], st["n_local"]) != (self.rank, self.world, int(self.batch.N)):
            raise ValueError(f"checkpoint {path} is for rank {st['rank']} of {st['world']} with "
                             f"{st['n_local']} homes, not rank {self.rank} of {self.world} with {self.batch.N}")
        want = {"seed": self.seed, "num_timesteps": int(self.num_timesteps), "n_all": len(self.all_homes),
                "names_crc": int(self.names_crc)}
        diff = {k: (st.get(k), v) for k, v in want.items() if st.get(k) != v}
        if diff:
            raise ValueError(f"checkpoint {path} belongs to another run (saved vs this run: {diff})")
        t = int(st["timestep"])
        if not 0 <= t <= self.num_timesteps:
            raise ValueError(f"checkpoint {path} holds timestep {t} of a {self.num_timesteps}-step run")
        self.batch.vals.copy_(st["vals"])
        self.batch.fc.copy_(st["fc"])
        self.batch.set_reward_price(st["reward_price"].to(self.device))
        self.agg_hist[:t].copy_(st["agg_hist"])
        self.status_hist[:t].copy_(st["status_hist"])
        if st.get("path_hist") is not None:
            self.path_hist[:t].copy_(st["path_hist"])
        self._deferred = st["deferred"].tolist()
        if self.hist is not None and st["hist"] is not None:
            self.hist[:t].copy_(st["hist"])
        self.timestep = t
        return t

    def resume(self, path):
        """load_state(path) on every rank together (path None or absent: step 0), then agree on the
        timestep.  A rank whose checkpoint is refused (another run's, corrupt, out of range) does not
        raise before the collective -- the other ranks would wait in it forever -- but agrees on -1,
        so that every rank raises together: the refused rank its own error, the others the
        disagreement (or, when every rank refused, each its own error)."""
        err, t = None, 0
        if path is not None and os.path.isfile(path):
            try:
                t = self.load_state(path)
            except Exception as e:      # any refusal (incl. pickle.UnpicklingError from a garbage
                err, t = e, -1          # file under weights_only=True) must reach the collective
        try:
            t = self.agree(t, "the checkpoint timestep to resume from")
        except RuntimeError as e:
            if err is not None:
                raise err from e
            raise
        if err is not None:
            raise err
        return t

    def agree(self, value, what):
        """Every rank's `value` (an int) must be the same; raises on every rank otherwise (one
        min and one max all-reduce), so that no rank goes on into a collective the others skip."""
        if self.world == 1:
            return int(value)
        v = torch.tensor([int(value), -int(value)], dtype=torch.int64, device=self.agg_hist.device)
        torch.distributed.all_reduce(v, op=torch.distributed.ReduceOp.MIN, group=self.group)
        lo, hi = int(v[0]), -int(v[1])
        if lo != hi:
            raise RuntimeError(f"ranks disagree on {what}: from {lo} to {hi} (this rank: {int(value)})")
        return lo

    def check_errors(self):
        """Raise as the reference would if a home hit a crashing path (KeyError / ValueError):
        the first such (timestep, home) over EVERY rank, raised on every rank together (one
        all-reduce), so a multi-rank run stops instead of leaving the other ranks in a gather."""
        self.drain()
        st = self.status_hist[:self.timestep].cpu().numpy()
        n_all = max(1, len(self.all_homes))
        first = np.iinfo(np.int64).max
        for code in (L.ST_ERR_MISSING, L.ST_ERR_PARSE):
            bad = np.argwhere(st == code)
            if len(bad):
                t, i = bad[0]
                first = min(first, (int(t) * n_all + int(self.index[i])) * 8 + code)
        if self.world > 1:
            v = torch.tensor([first], dtype=torch.int64, device=self.agg_hist.device)
            torch.distributed.all_reduce(v, op=torch.distributed.ReduceOp.MIN, group=self.group)
            first = int(v[0])
        if first == np.iinfo(np.int64).max:
            return
        code = first % 8
        t, g = divmod(first // 8, n_all)
        exc = KeyError if code == L.ST_ERR_MISSING else ValueError
        raise exc(f"home {self.all_homes[g]['name']} at timestep {t}: {L.STATUS_NAMES[code]} "
                  "(the reference raises here, mpc_calc.py:280-289 / 537-539)")

    def collected_data(self):
        """This shard's `collected_data` dict (aggregator.py:589-615, 737-748): the initial
        entries plus every step's hash fields, in the reference's key order."""
        from . import results as R
        self.drain()
        hist = self.hist[:self.timestep].cpu().numpy()
        return R.append_history(R.new_collected(self.homes), self.homes, hist)

    def summary(self):
        self.drain()
        agg = self.agg_hist[:self.timestep].cpu().numpy()
        return {"p_grid_aggregate": agg[:, 0].tolist(), "forecast_load": agg[:, 1].tolist(),
                "agg_cost": agg[:, 2].tolist(), "p_max_aggregate": float(agg[:, 0].max()) if len(agg) else None}
