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
(backend "nccl" = RCCL); homes are sharded in contiguous blocks, the three per-step sums are
all-reduced, rank 0 gathers the history and writes the files.

Scope: run_rbo_mpc (the baseline case).  SPP prices (`agg.spp_enabled`, an ERCOT xlsx) and
the RL-aggregator case are not part of this build and raise.
"""
import json
import os
from datetime import datetime

import numpy as np

from . import inputs as I
from . import results as R


class Aggregator:
    def __init__(self, data_dir=None, config_file=None, outputs_dir="outputs", int_mode="round", device=None,
                 group=None, first_name=None, batch_cls=None):
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
        if not self.config["community"]["overwrite_existing"] and os.path.isfile(path):
            with open(path) as f:
                self.all_homes = json.load(f)
        else:
            draws = os.path.join(self.data_dir, self.config["home"]["wh"]["waterdraw_file"])
            self.all_homes = I.create_homes(self.config, self.num_timesteps, self.dt, draws, self.first_name)
        I.check_home_counts(self.all_homes, self.config)
        if self.rank == 0:
            R.write_home_configs(self.outputs_dir, self.all_homes, n)
        self.max_poss_load = sum(I.max_load(h) for h in self.all_homes)

    # aggregator.py:757-778
    def run_baseline(self, noise_fn=None):
        """`noise_fn(t)`, optional: the season draw [H][homes checked] of step t (replaces the
        keyed on-device stream, e.g. to replay a recorded run)."""
        from .aggregator import DeviceAggregator
        self.start_time = datetime.now()
        self.checked = [h for h in self.all_homes if self.check_type == "all" or h["type"] == self.check_type]
        col = lambda c: self.all_data[c].to_numpy(dtype=float)  # noqa: E731
        self.dev = DeviceAggregator(self.checked, col("OAT"), col("GHI"), col("tou"), self.start_hour_index,
                                    self.num_timesteps, reward_price=self.reward_price, int_mode=self.int_mode,
                                    seed=int(self.config["simulation"]["random_seed"]), rank=self.rank,
                                    world=self.world, group=self.group, device=self.device,
                                    **({"batch_cls": self.batch_cls} if self.batch_cls else {}))
        for t in range(self.num_timesteps):
            noise = noise_fn(t)[:, self.dev.lo:self.dev.hi] if noise_fn is not None else None
            self.dev.run_iteration(noise)
            self.dev.collect_data()
            self.timestep = t + 1
            if (t + 1) % self.checkpoint_interval == 0:
                self.write_outputs()
        self.dev.check_errors()

    def _history(self):
        """The checked homes' hash history [T][19][N] on rank 0 (gathered from every rank)."""
        hist = self.dev.hist[:self.dev.timestep].cpu().numpy()
        if self.world == 1:
            return hist
        import torch.distributed as dist
        parts = [None] * self.world if self.rank == 0 else None
        dist.gather_object(hist, parts, dst=0, group=self.group)
        return np.concatenate(parts, axis=2) if self.rank == 0 else None

    # aggregator.py:783-844 (summarize_baseline + write_outputs)
    def write_outputs(self):
        hist = self._history()
        if self.rank != 0:
            return None
        t_diff = datetime.now() - self.start_time
        collected = R.new_collected(self.all_homes)
        R.append_history(collected, self.checked, hist)
        loads = R.aggregate_loads(hist)
        self.max_agg_load = max(loads)
        self.max_agg_load_list.append(self.max_agg_load)
        collected["Summary"] = R.summary(
            self.case, self.start_dt, self.end_dt, t_diff.total_seconds(),
            self.config["home"]["hems"]["prediction_horizon"], self.config["community"]["total_number_homes"],
            loads, self.all_data.loc[self.mask, "OAT"].values.tolist(),
            self.all_data.loc[self.mask, "GHI"].values.tolist(), self.all_rps.tolist(), self.all_sps.tolist(),
            tou=self.all_data.loc[self.mask, "tou"].values.tolist())
        self.collected_data = collected
        return R.write_results(self.run_dir, self.case, collected)

    # aggregator.py:941-970
    def run(self, noise_fn=None):
        sim = self.config["simulation"]
        self.checkpoint_interval = R.checkpoint_interval(sim["checkpoint_interval"], self.dt)
        self.version = sim["named_version"]
        hems = self.config["home"]["hems"]
        self.run_dir = R.run_dir(self.outputs_dir, self.start_dt, self.end_dt, self.check_type,
                                 self.config["community"]["total_number_homes"], hems["prediction_horizon"],
                                 self.dt_interval, hems["sub_subhourly_steps"], hems["solver"], self.version)
        if sim["run_rbo_mpc"]:
            self.case = "baseline"
            self.flush()
            self.get_homes()
            self.run_baseline(noise_fn)
            return self.write_outputs()
        raise NotImplementedError("only run_rbo_mpc (the baseline case) is part of this build")


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
