"""Drop-in for `dragg.aggregator.Aggregator` on its run_rbo_mpc path, solved on MI355X.

Reference: aggregator.py:28-970 (+ `dragg/main.py`: `Aggregator().run()`).  The same
environment variables, config.toml, NSRDB weather csv and water-draw profiles go in; the
same outputs come out (outputs/all_homes-<N>-config.json and
outputs/<run dir>/baseline/results.json, checkpointed at the configured cadence).  In between,
nothing of the reference's per-step machinery is left: no process pool, no pickled MPCCalc,
no redis round trips.  The community's state stays on the GPU (`DeviceAggregator`), one
kernel launch per timestep solves every home of this rank's shard, and the hash history is
brought to the host only when an output file is written.

    python -m dragg_amd.runner            # like `python -m dragg.main`, DATA_DIR / CONFIG_FILE honoured

Multi-GPU: start one process per GPU (torchrun) with torch.distributed initialised
(backend "nccl" = RCCL); homes are sharded by stride (shard_index), the three per-step sums are
all-reduced, rank 0 gathers the history and writes the files.

Scope: run_rbo_mpc (the baseline case) and the RL-aggregator hooks (SURVEY.md §8 F4:
`setup_rl_agg_run`, `redis_set_current_values`, `gen_setpoint`, `test_response`, plus
`rl_step` / `rl_forecast` / `run_rl_agg`, the reward-price loop the reference leaves to an
external driver).  SPP prices (`agg.spp_enabled`, an ERCOT xlsx absent from the reference)
raise.
"""
import json
import os
import time
import warnings
from contextlib import contextmanager
from datetime import datetime

import numpy as np

from . import inputs as I
from . import results as R


class Aggregator:
    def __init__(self, data_dir=None, config_file=None, outputs_dir="outputs", int_mode="round", device=None,
                 group=None, first_name=None, batch_cls=None):
        # wall seconds per phase of the run (tools/e2e.py): {phase: seconds}, accumulated
        self.timings = {}
        with self._phase("config_and_weather"):
            self._init(data_dir, config_file, outputs_dir, int_mode, device, group, first_name, batch_cls)

    @contextmanager
    def _phase(self, name):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.timings[name] = self.timings.get(name, 0.0) + time.perf_counter() - t0

    def _init(self, data_dir, config_file, outputs_dir, int_mode, device, group, first_name, batch_cls):
        env = os.environ
        self.data_dir = os.path.expanduser(env.get("DATA_DIR", "data")) if data_dir is None else data_dir
        self.outputs_dir = outputs_dir
        self.config_file = config_file or os.path.join(self.data_dir, env.get("CONFIG_FILE", "config.toml"))
        self.ts_data_file = os.path.join(self.data_dir, env.get("SOLAR_TEMPERATURE_DATA_FILE", "nsrdb.csv"))
        self.config = I.read_config(self.config_file)
        self.check_type = self.config["simulation"]["check_type"]
        self.dt = int(self.config["agg"]["subhourly_steps"])
        self.dt_interval = 60 // self.dt
        self.ts_data = I.load_weather(self.ts_data_file, self.dt)
        self.start_dt, self.end_dt, self.hours = I.run_window(self.config)
        self.num_timesteps = int(np.ceil(self.hours * self.dt))
        if self.config["agg"]["spp_enabled"]:
            raise I.ConfigError("SPP prices (agg.spp_enabled) are not supported by this build")
        self.tou_data = I.tou_prices(self.start_dt, self.hours, self.config["agg"])
        self.all_data, self.mask = I.join_series(self.ts_data, self.tou_data, self.start_dt, self.end_dt)
        self.all_rps = np.zeros(self.num_timesteps)
        self.all_sps = np.zeros(self.num_timesteps)
        self.case = "baseline"
        self.int_mode, self.device, self.group = int_mode, device, group
        self.first_name = first_name
        self.batch_cls = batch_cls          # injectable only for the CPU tests of the multi-rank glue
        self.rank, self.world = 0, 1
        try:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized():
                self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        except ImportError:
            pass
        self.agg_load = 0                   # aggregator.py:55-57
        self.baseline_agg_load_list = []
        self.max_agg_load_list = []
        self.dev = None
        if self.rank == 0:
            os.makedirs(self.outputs_dir, exist_ok=True)

    # aggregator.py:913-925 (flush_redis: the checks, the start index and initial values)
    def flush(self):
        I.check_series(self.all_data, self.start_dt, self.end_dt, self.config["home"]["hems"]["prediction_horizon"])
        self.start_hour_index = I.start_hour_index(self.all_data, self.start_dt)
        self.timestep = 0
        self.reward_price = np.zeros(self.config["agg"]["rl"]["action_horizon"] * self.dt)

    # aggregator.py:263-271
    def get_homes(self):
        n = self.config["community"]["total_number_homes"]
        path = os.path.join(self.outputs_dir, f"all_homes-{n}-config.json")
        with self._phase("create_homes"):
            if not self.config["community"]["overwrite_existing"] and os.path.isfile(path):
                with open(path) as f:
                    self.all_homes = json.load(f)
            else:
                draws = os.path.join(self.data_dir, self.config["home"]["wh"]["waterdraw_file"])
                self.all_homes = I.create_homes(self.config, self.num_timesteps, self.dt, draws, self.first_name)
            I.check_home_counts(self.all_homes, self.config)
        if self.rank == 0:
            with self._phase("write_home_configs"):
                R.write_home_configs(self.outputs_dir, self.all_homes, n)
        self.max_poss_load = sum(I.max_load(h) for h in self.all_homes)

    def _device_community(self):
        """The checked homes (aggregator.py:762-765 / 879-882) as this rank's device shard."""
        from .aggregator import DeviceAggregator
        self.checked = [h for h in self.all_homes if self.check_type == "all" or h["type"] == self.check_type]
        self._hist_rows = 0                 # steps of the history already on rank 0 (_history)
        col = lambda c: self.all_data[c].to_numpy(dtype=float)  # noqa: E731
        self.dev = DeviceAggregator(self.checked, col("OAT"), col("GHI"), col("tou"), self.start_hour_index,
                                    self.num_timesteps, reward_price=self.reward_price, int_mode=self.int_mode,
                                    seed=int(self.config["simulation"]["random_seed"]), rank=self.rank,
                                    world=self.world, group=self.group, device=self.device,
                                    # run_rbo_mpc: a home in its step-function DP does not hold up the
                                    # others (lag mode, DeviceAggregator); results are bit-identical
                                    overlap=getattr(self, "case", None) == "baseline",
                                    **({"batch_cls": self.batch_cls} if self.batch_cls else {}))
        return self.dev

    def state_path(self):
        """This rank's device-state checkpoint, next to results.json (<run dir>/<case>/)."""
        d = os.path.join(self.run_dir, self.case)
        os.makedirs(d, exist_ok=True)
        return os.path.join(d, f"state-rank{self.rank}-of-{self.world}.pt")

    # aggregator.py:757-778
    def run_baseline(self, noise_fn=None, resume=False, stop_after=None):
        """`noise_fn(t)`, optional: the season draw [H][homes checked] of step t (replaces the
        keyed on-device stream, e.g. to replay a recorded run).  Every checkpoint also saves
        each rank's device state; `resume=True` continues from it (the reference has no resume:
        aggregator.py:265-267, 768) and finishes with the results an uninterrupted run writes.
        Every rank must resume from the same timestep (a crash between two ranks' saves leaves
        them apart): they check that together and all raise otherwise.  `stop_after`: return
        after the first checkpoint at or past that many steps (an interrupted run)."""
        self.start_time = datetime.now()
        with self._phase("upload"):
            self._device_community()
            self._sync()
        t0 = 0
        if resume:                                 # every rank loads, then all agree (or all raise)
            t0 = self.dev.resume(self.state_path())
            self.timestep = t0
        loop_t0 = time.perf_counter()
        ckpt = self.timings.get("checkpoints", 0.0)
        for t in range(t0, self.num_timesteps):
            noise = noise_fn(t)[:, self.dev.index] if noise_fn is not None else None
            self.dev.run_iteration(noise)
            self.dev.collect_data(defer=True)      # no feedback: the sums are reduced at the end
            self.timestep = t + 1
            if (t + 1) % self.checkpoint_interval == 0:
                with self._phase("checkpoints"):
                    # the reference raises inside the step that fails (mpc_calc.py:280-289,
                    # 537-539); checking at each checkpoint (one host sync) keeps post-error data
                    # out of every results.json written
                    self.dev.check_errors()
                    self.write_outputs()
                    self.dev.save_state(self.state_path())
                if stop_after is not None and t + 1 >= stop_after:
                    return                         # an interrupted run
        self.dev.reduce_history()
        self.dev.check_errors()
        self.check_solve_paths()
        # the step loop: launches and device time of every step, without the checkpoint writes
        self.timings["step_loop"] = (self.timings.get("step_loop", 0.0) + time.perf_counter() - loop_t0
                                     - (self.timings.get("checkpoints", 0.0) - ckpt))

    def _sync(self):
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize()
        except ImportError:
            pass

    def check_solve_paths(self):
        """The run's solve-path counts over every rank (`self.solve_paths`: approximate solves, solves by
        the step-function DP, solves finished by a later launch); warns when a solve kept an approximate
        integer schedule -- the reference's GLPK_MI solve is exact up to its gap (mpc_calc.py:447-451),
        so such a run is not the reference's to that tolerance (int_path reasons 3 and 6)."""
        self.solve_paths = self.dev.approx_counts()
        n = self.solve_paths["approx_solves"]
        if n:
            where = self.dev.approx_solves()[:5]
            warnings.warn(f"{n} solve(s) kept an approximate integer schedule (int_path reason 3 / 6; first on "
                          f"this rank as (timestep, home, int_path): {where}); rerun with a larger "
                          "DRAGG_STEP_WORK_CAP / DRAGG_STEP_POOL_CAP or dims.flags DRAGG_FLAG_EXACT", RuntimeWarning)
        return self.solve_paths

    # ------------------------------------------------------------------ RL aggregator (§8 F4)
    # aggregator.py:677-696
    def gen_setpoint(self):
        if self.timestep < 2:
            self.tracked_loads = [0.5 * self.max_poss_load] * self.config["agg"]["rl"]["prev_timesteps"]
            self.max_load = -float("inf")
            self.min_load = float("inf")
        else:
            self.tracked_loads[:-1] = self.tracked_loads[1:]
            self.tracked_loads[-1] = self.agg_load
        self.avg_load = np.average(self.tracked_loads)
        if self.agg_load > self.max_load or self.timestep % 24 == 0:
            self.max_load = self.agg_load
        if self.agg_load < self.min_load or self.timestep % 24 == 0:
            self.min_load = self.agg_load
        return self.avg_load

    # aggregator.py:664-675: the reward price goes to every rank's solver (RCCL broadcast from
    # rank 0) instead of the redis 'reward_price' list
    def redis_set_current_values(self):
        if "rl" in self.case:
            self.all_sps[self.timestep] = self.agg_setpoint
            self.all_rps[self.timestep] = self.reward_price[0]
            self.dev.set_reward_price(self.reward_price)

    # aggregator.py:876-896
    def setup_rl_agg_run(self, noise_fn=None):
        """Needs the community (`get_homes`) like the reference's (it reads all_homes_obj)."""
        self.flush()
        self._device_community()
        self.noise_fn = noise_fn
        self.start_time = datetime.now()
        self.baseline_agg_load_list = [0]
        self.all_rewards = []
        self.forecast_load = 3 * len(self.all_homes)
        self.prev_forecast_load = self.forecast_load
        self.forecast_setpoint = self.gen_setpoint()
        self.agg_load = self.forecast_load  # approximate load for initial timestep
        self.agg_setpoint = self.gen_setpoint()
        self.redis_set_current_values()

    def _noise(self, t):
        fn = getattr(self, "noise_fn", None)
        return fn(t)[:, self.dev.index] if fn is not None else None

    # aggregator.py:728-755 on the RL path: the three community sums come to the host (the
    # agent needs them) and feed the setpoint
    def collect_data(self):
        agg = self.dev.collect_data().tolist()
        self.agg_load, self.forecast_load, self.agg_cost = agg
        self.baseline_agg_load_list.append(self.agg_load)
        self.agg_setpoint = self.gen_setpoint()
        return agg

    def _set_price(self, reward_price):
        rp = np.asarray(reward_price, dtype=float).reshape(-1)
        if len(rp) == 1:
            rp = np.full(len(self.reward_price), rp[0])
        if len(rp) != len(self.reward_price):
            raise ValueError(f"reward price has {len(rp)} entries, the action horizon holds "
                             f"{len(self.reward_price)} (agg.rl.action_horizon * dt)")
        self.reward_price = rp

    def rl_step(self, reward_price):
        """One RL-aggregator timestep under `reward_price` (a scalar, or action_horizon*dt
        values): publish the price, solve every home, collect, new setpoint -- the order of
        the reference's step loop (aggregator.py:768-771)."""
        self._set_price(reward_price)
        self.redis_set_current_values()
        self.dev.run_iteration(self._noise(self.dev.timestep))
        self.timestep = self.dev.timestep
        return self.collect_data()

    def rl_forecast(self, reward_price, steps=None):
        """The community's response to a candidate price over `rl.forecast_horizon` timesteps
        (README.md:67, `rl_agg_forecast_horizon`): every home re-solved ahead on device,
        nothing committed.  -> [steps][agg_load, forecast_load, agg_cost] on the host."""
        steps = int(self.config["agg"]["rl"]["forecast_horizon"]) if steps is None else int(steps)
        steps = min(steps, self.num_timesteps - self.dev.timestep)
        prev = self.reward_price
        self._set_price(reward_price)
        self.dev.set_reward_price(self.reward_price)
        try:
            out = self.dev.forecast(steps, noise_fn=self._noise if getattr(self, "noise_fn", None) else None)
        finally:
            self.reward_price = prev
            self.dev.set_reward_price(prev)
        return out.cpu().numpy()

    # aggregator.py:898-911
    def test_response(self):
        c = self.config["agg"]["simplified"]["response_rate"]
        if self.timestep == 0:
            self.agg_load = self.agg_setpoint + 0.1 * self.agg_setpoint
        self.agg_load = self.agg_load - c * self.reward_price[0] * (self.agg_setpoint - self.agg_load)
        self.agg_cost = self.agg_load * self.reward_price[0]
        self.timestep += 1

    def run_rl_agg(self, policy, noise_fn=None):
        """The `run_rl_agg` case (README.md:55): MPC homes under an RL-designed reward price.
        `policy(aggregator) -> reward price` is called once per timestep (e.g. an
        `dragg_amd.rl.SetpointAgent.act`, or the reference's agent via `rl.policy_from_agent`);
        it may call `rl_forecast` to try candidate prices.
        Writes `<run dir>/rl_agg/results.json` with the Summary's RP and p_grid_setpoint."""
        self.case = "rl_agg"
        self.get_homes()
        self.setup_rl_agg_run(noise_fn)
        for t in range(self.num_timesteps):
            self.rl_step(policy(self))
            if (t + 1) % self.checkpoint_interval == 0:
                # the reference raises inside the step that fails (mpc_calc.py:280-289,
                # 537-539); checking at each checkpoint (one host sync) keeps post-error data
                # out of every results.json written
                self.dev.check_errors()
                self.write_outputs()
        self.dev.check_errors()
        self.check_solve_paths()
        return self.write_outputs()

    def _history(self):
        """The checked homes' hash history [T][19][N] on rank 0.

        Incremental: each call brings over only the steps since the previous one (a checkpoint
        then costs its own rows, not the whole run again), as one tensor gather of the shards
        padded to a common width (NCCL on the device, gloo on the host) -- no pickling."""
        self.dev.drain()
        T = self.dev.timestep
        t0 = getattr(self, "_hist_rows", 0)
        if t0 == 0:
            self._hist_host = []
        if T > t0:
            new = self.dev.hist[t0:T]                      # [dT][19][n_local]
            if self.world == 1:
                self._hist_host.append(new.cpu().numpy())
            else:
                import torch
                import torch.distributed as dist
                n_all = len(self.checked)
                width = -(-n_all // self.world)            # the widest strided shard
                on_dev = dist.get_backend(self.group) == "nccl"
                src = new if on_dev else new.cpu()
                pad = torch.full(src.shape[:2] + (width,), float("nan"), dtype=src.dtype, device=src.device)
                pad[:, :, :src.shape[2]] = src
                parts = [torch.empty_like(pad) for _ in range(self.world)] if self.rank == 0 else None
                dist.gather(pad, parts, dst=0, group=self.group)
                if self.rank == 0:
                    out = np.empty(src.shape[:2] + (n_all,), dtype=np.float64)
                    for r, p in enumerate(parts):          # rank r holds homes r, r + world, ... (shard_index)
                        k = len(range(r, n_all, self.world))
                        out[:, :, r::self.world] = p[:, :, :k].cpu().numpy()
                    self._hist_host.append(out)
            self._hist_rows = T
        if self.rank != 0:
            return None
        if not self._hist_host:
            return np.empty((0, self.dev.hist.shape[1], len(self.checked)))
        if len(self._hist_host) > 1:
            self._hist_host = [np.concatenate(self._hist_host, axis=0)]
        return self._hist_host[0]

    # aggregator.py:783-844 (summarize_baseline + write_outputs)
    def write_outputs(self):
        with self._phase("history_gather"):
            hist = self._history()
        if self.rank != 0:
            return None
        t_diff = datetime.now() - self.start_time
        with self._phase("results_build"):
            # the RL case's list starts with setup_rl_agg_run's 0 (aggregator.py:887)
            loads = self.baseline_agg_load_list if "rl" in self.case else R.aggregate_loads(hist)
            self.max_agg_load = max(loads)
            self.max_agg_load_list.append(self.max_agg_load)
            summary = R.summary(
                self.case, self.start_dt, self.end_dt, t_diff.total_seconds(),
                self.config["home"]["hems"]["prediction_horizon"], self.config["community"]["total_number_homes"],
                loads, self.all_data.loc[self.mask, "OAT"].values.tolist(),
                self.all_data.loc[self.mask, "GHI"].values.tolist(), self.all_rps.tolist(), self.all_sps.tolist(),
                tou=self.all_data.loc[self.mask, "tou"].values.tolist())
            # the reference's collected_data dict (aggregator.py:589-615, 737-748) is built when read
            self._collected_src = (self.all_homes, self.checked, hist, summary)
            self._collected = None
        with self._phase("results_write"):
            # the same bytes as json.dump(collected_data, indent=4), straight from the history array
            if not hasattr(self, "_results_cache"):
                self._results_cache = {}
            return R.write_results_history(self.run_dir, self.case, self.all_homes, self.checked, hist, summary,
                                           cache=self._results_cache)

    @property
    def collected_data(self):
        """The reference's `collected_data` (per-home series + "Summary"), as of the last write_outputs."""
        if getattr(self, "_collected", None) is None and getattr(self, "_collected_src", None) is not None:
            homes, checked, hist, summary = self._collected_src
            c = R.new_collected(homes)
            R.append_history(c, checked, hist)
            c["Summary"] = summary
            self._collected = c
        return getattr(self, "_collected", None)

    # aggregator.py:941-970
    def run(self, noise_fn=None, resume=False, stop_after=None):
        sim = self.config["simulation"]
        self.checkpoint_interval = R.checkpoint_interval(sim["checkpoint_interval"], self.dt)
        self.version = sim["named_version"]
        hems = self.config["home"]["hems"]
        self.run_dir = R.run_dir(self.outputs_dir, self.start_dt, self.end_dt, self.check_type,
                                 self.config["community"]["total_number_homes"], hems["prediction_horizon"],
                                 self.dt_interval, hems["sub_subhourly_steps"], hems["solver"], self.version)
        if sim["run_rbo_mpc"]:
            self.case = "baseline"
            with self._phase("flush"):
                self.flush()
            self.get_homes()
            self.run_baseline(noise_fn, resume=resume, stop_after=stop_after)
            if stop_after is not None and self.timestep < self.num_timesteps:
                return None
            return self.write_outputs()
        if sim.get("run_rl_agg"):
            if resume or stop_after is not None:
                # the RL loop's state (the agent, the setpoint history, all_rps / all_sps) is not
                # checkpointed: a resumed RL run would silently start over
                raise ValueError("resume / stop_after are supported on the run_rbo_mpc case only")
            from .rl import agent_policy
            return self.run_rl_agg(agent_policy(self), noise_fn)
        return None


def main():
    """`python -m dragg_amd.runner`; under torchrun (WORLD_SIZE > 1) one rank per GPU over RCCL."""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("nccl")
        try:
            Aggregator().run()
        finally:
            dist.destroy_process_group()
    else:
        Aggregator().run()


if __name__ == "__main__":
    main()
