#!/usr/bin/env python3
"""Generate golden fixtures by running the REFERENCE's own code (this container only).

TEST INFRASTRUCTURE.  Never shipped, never run on the GPU box; the GPU box only
sees the committed fixture files this script writes under tests/golden/.

What it does
------------
* Imports the unmodified reference package from /root/reference (`dragg.aggregator`,
  `dragg.mpc_calc`) with stand-ins for its absent third-party dependencies
  (tests/golden/refshim: cvxpy-subset over scipy HiGHS, in-memory redis with
  str values, tomli-backed toml, sequential deep-copying pathos pool, names).
* Replaces ONLY the forecast-noise source: `mpc_calc.py:222` draws
  `np.random.randn(H)` from the worker's global RNG (not reproducible).
  Here that call returns a keyed draw `default_rng([seed, home_index, t])`, and the
  draw is recorded in the fixture so every consumer can replay it.
* Runs `Aggregator().run()` (run_rbo_mpc) end to end and records, per solve
  (home, t): the inputs the solve saw, the HiGHS MILP status / objective, the
  LP-relaxation objective and solution, and every field written to the home's
  redis hash.  Also dumps results.json (collected data) and the community
  (all_homes-N-config.json).

Usage:  python tests/golden/make_golden.py [scenario ...]
"""
import copy
import gzip
import inspect
import json
import os
import shutil
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

SCENARIOS = {
    # BASELINE config 1: 20-home mixed community, 24 h at 15-min steps, 6 h horizon.
    "c1_h24": dict(n=20, batt=4, pv=4, pvb=4, start="2015-01-01 00", end="2015-01-02 00",
                   dt=4, horizon=6, action_horizon=6, seed=12, record_t=range(0, 96)),
    # the same run with every MILP proven optimal (GOLDEN_MIP_REL_GAP=0, long GOLDEN_MILP_TIME_LIMIT);
    # a record whose milp_status is still 1 (time limit, incumbent kept) is unpinned
    "c1_h24_proven": dict(n=20, batt=4, pv=4, pvb=4, start="2015-01-01 00", end="2015-01-02 00",
                          dt=4, horizon=6, action_horizon=6, seed=12, record_t=range(0, 96)),
    # 12 h horizon (H=48): season noise sigma reaches 1.1^47 -> mostly 'summer' -> fallback.
    "c3_h48": dict(n=6, batt=0, pv=2, pvb=0, start="2015-01-01 00", end="2015-01-01 04",
                   dt=4, horizon=12, action_horizon=12, seed=7, record_t=range(0, 16)),
    # hourly steps (dt=1), different season/time of year: exercises summer mode and tou.
    "summer_dt1": dict(n=6, batt=0, pv=3, pvb=0, start="2015-07-10 00", end="2015-07-11 00",
                       dt=1, horizon=6, action_horizon=6, seed=3, record_t=range(0, 24)),
    # spring, hourly steps, all four types (battery homes must not fail at t=0: the reference
    # then raises KeyError('e_batt_opt') at t=1, mpc_calc.py:285)
    "spring_dt1": dict(n=8, batt=2, pv=2, pvb=2, start="2015-04-02 00", end="2015-04-03 00",
                       dt=1, horizon=4, action_horizon=4, seed=5, record_t=range(0, 24)),
    # negative total prices (an RL reward price, broadcast through the redis 'reward_price'
    # list as aggregator.py:671-675 does): battery charge-while-discharge edge, PV curtailment
    "negprice_dt1": dict(n=8, batt=2, pv=2, pvb=2, start="2015-04-02 00", end="2015-04-03 00",
                         dt=1, horizon=4, action_horizon=4, seed=11, record_t=range(0, 24),
                         rp=[-0.12, 0.03, -0.2, 0.0]),
    "negprice_dt2": dict(n=4, batt=1, pv=1, pvb=1, start="2015-01-01 00", end="2015-01-01 12",
                         dt=2, horizon=6, action_horizon=6, seed=13, record_t=range(0, 24),
                         rp=[round(0.11 * np.sin(0.5 * k) - 0.04, 4) for k in range(12)]),
}

# the reference config.toml of every scenario (str.format fields: n, batt, pv, pvb, start, end, seed,
# dt, action_horizon, horizon); shared with the tests, which build the same configs
with open(os.path.join(HERE, "config_template.toml")) as _f:
    CONFIG_TMPL = _f.read()



class _NoiseRandom:
    """Stands in for `np.random` inside dragg.mpc_calc only; randn is keyed by (seed, home, t)."""

    def __init__(self, seed, index_of, log):
        self.seed, self.index_of, self.log = seed, index_of, log
        self.cp = None

    def randn(self, *shape):
        me = inspect.currentframe().f_back.f_locals["self"]
        hidx = self.index_of[me.name]
        if self.cp is not None:
            self.cp.CURRENT_HOME[0] = hidx          # (GOLDEN_OWN runs: the shim's solve limits)
        draw = np.random.default_rng([self.seed, hidx, int(me.timestep)]).standard_normal(shape)
        self.log[(me.name, int(me.timestep))] = draw.copy()
        return draw

    def __getattr__(self, k):
        return getattr(np.random, k)


class _NumpyProxy(types.ModuleType):
    def __init__(self, rnd):
        super().__init__("numpy_proxy")
        self.random = rnd

    def __getattr__(self, k):
        return getattr(np, k)


def _f(x):
    return None if x is None else float(x)


def run(name, sc, hook=None):
    work = tempfile.mkdtemp(prefix=f"golden_{name}_")
    data = os.path.join(work, "data")
    os.makedirs(data)
    with open(os.path.join(data, "config.toml"), "w") as f:
        f.write(CONFIG_TMPL.format(**sc))
    os.symlink(os.path.join(REF, "dragg/data/nsrdb.csv"), os.path.join(data, "nsrdb.csv"))
    os.symlink(os.path.join(REF, "dragg/data/waterdraw_profiles.csv"),
               os.path.join(data, "waterdraw_profiles.csv"))
    os.environ["DATA_DIR"] = data
    os.environ["LOGLEVEL"] = "ERROR"
    cwd = os.getcwd()
    os.chdir(work)
    sys.path.insert(0, os.path.join(HERE, "refshim"))
    sys.path.insert(1, REF)
    for m in [m for m in sys.modules if m.startswith("dragg") or m in ("redis", "cvxpy", "toml", "names")
              or m.startswith("pathos")]:
        del sys.modules[m]
    import redis  # refshim
    redis._STORE.clear()
    import cvxpy as cp  # refshim
    if hook is not None:
        hook(cp)
    import dragg.mpc_calc as mc
    import dragg.aggregator as ag

    import pathos.pools as pp  # refshim
    del pp.EXTRA[:]
    index_of, noise_log, records = {}, {}, pp.EXTRA
    rnd = _NoiseRandom(sc["seed"], index_of, noise_log)
    rnd.cp = cp
    mc.np = _NumpyProxy(rnd)
    record_t = set(sc["record_t"])

    orig_cleanup = mc.MPCCalc.cleanup_and_finish

    def cleanup(self):
        t = int(self.timestep)
        rec_in = None
        if t in record_t:
            lr = cp.Problem.last_record
            prev = dict(self.prev_optimal_vals) if (t > 0 and self.prev_optimal_vals is not None) else {}
            rec_in = dict(
                name=self.name, home=index_of[self.name], type=self.type, t=t,
                T0=_f(self.temp_in_init.value), Tw0=_f(self.temp_wh_init.value),
                E0=_f(self.e_batt_init.value) if "battery" in self.type else None,
                counter_in=int(self.counter),
                draw_size=[float(v) for v in self.draw_size],
                oat=[float(v) for v in self.oat_current], ghi=[float(v) for v in self.ghi_current],
                tou=[float(v) for v in self.base_price],
                reward_price=[float(v) for v in self.reward_price],
                total_price=[float(v) for v in self.total_price.value],
                noise=noise_log[(self.name, t)].tolist(),
                season="winter" if self.hvac_heat_max > 0 else "summer",
                status=self.prob.status,
                milp_obj=lr["obj"] if lr else None,
                milp_status=lr["milp_status"] if lr else None,
                milp_gap=_f(lr["mip_gap"]) if lr else None,
                milp_seconds=_f(lr.get("milp_seconds")) if lr else None,
                lp_status=int(lr["relax_status"]) if lr else None,
                lp_obj=lr["relax_obj"] if lr else None,
                prev_hash=prev if self.prob.status != "optimal" else {},
            )
            if lr and lr["relax_x"] is not None:
                relax = {}
                for v, off in lr["order"]:
                    relax[v.id] = lr["relax_x"][off:off + v.n].tolist()
                names_ = {"p_grid": self.p_grid, "p_load": self.p_load, "temp_in_ev": self.temp_in_ev,
                          "temp_wh_ev": self.temp_wh_ev, "temp_in": self.temp_in, "temp_wh": self.temp_wh,
                          "hvac_cool_on": self.hvac_cool_on, "hvac_heat_on": self.hvac_heat_on,
                          "wh_heat_on": self.wh_heat_on, "cost": self.cost}
                if "battery" in self.type:
                    names_.update(p_batt_ch=self.p_batt_ch, p_batt_disch=self.p_batt_disch, e_batt=self.e_batt)
                if "pv" in self.type:
                    names_.update(p_pv=self.p_pv, u_pv_curt=self.u_pv_curt)
                rec_in["lp"] = {k: relax.get(v.id) for k, v in names_.items()}
            if lr and lr["x"] is not None:
                mil = {}
                for v, off in lr["order"]:
                    mil[v.id] = lr["x"][off:off + v.n].tolist()
                rec_in["milp_x"] = {k: mil.get(getattr(self, k).id) for k in
                                    ["hvac_cool_on", "hvac_heat_on", "wh_heat_on", "temp_in_ev", "temp_wh_ev"]}
        orig_cleanup(self)
        if rec_in is not None:
            out = {}
            for k, v in self.optimal_vals.items():
                out[k] = v if isinstance(v, str) else float(v)
            rec_in["optimal_vals"] = out
            rec_in["counter_out"] = int(self.counter)
            records.append(rec_in)

    mc.MPCCalc.cleanup_and_finish = cleanup

    agg = ag.Aggregator()
    if sc.get("rp") is not None:            # the RL agent's reward-price broadcast, fixed
        orig_init = agg.redis_set_initial_values

        def init_vals():
            orig_init()
            agg.reward_price = np.array(sc["rp"], dtype=float)
            agg.redis_client.conn.delete("reward_price")
            agg.redis_client.conn.rpush("reward_price", *agg.reward_price.tolist())

        agg.redis_set_initial_values = init_vals
    orig_create = agg.create_homes

    def create_homes():
        orig_create()
        for i, h in enumerate(agg.all_homes):
            index_of[h["name"]] = i

    agg.create_homes = create_homes
    agg.run()

    res_path = None
    for root, _, files in os.walk(os.path.join(work, "outputs")):
        if "results.json" in files:
            res_path = os.path.join(root, "results.json")
    with open(res_path) as f:
        results = json.load(f)
    env = dict(
        oat=agg.all_data["OAT"].values[:24 * 8 * sc["dt"]].tolist(),
        ghi=agg.all_data["GHI"].values[:24 * 8 * sc["dt"]].tolist(),
        tou_window=agg.all_data["tou"].values[agg.start_hour_index:agg.start_hour_index
                                              + agg.num_timesteps + 60 * sc["dt"]].tolist(),
        start_hour_index=agg.start_hour_index, num_timesteps=agg.num_timesteps,
    )
    out = dict(scenario=name, params=sc | {"record_t": [min(record_t), max(record_t)]},
               homes=agg.all_homes, records=records, results=results, env=env)
    os.chdir(cwd)
    shutil.rmtree(work, ignore_errors=True)
    sys.path.remove(os.path.join(HERE, "refshim"))
    sys.path.remove(REF)
    if cp.OWN is not None:                  # a part of a run split by home: only its homes' records
        records[:] = [r for r in records if r["home"] in cp.OWN]
        out["params"]["own"] = sorted(cp.OWN)
    path = os.path.join(os.environ.get("GOLDEN_OUT_DIR", HERE), f"{name}{os.environ.get('GOLDEN_PART', '')}.json.gz")
    with gzip.open(path, "wt") as f:
        json.dump(out, f, separators=(",", ":"))
    nst = {}
    for r in records:
        nst[r["status"]] = nst.get(r["status"], 0) + 1
    print(f"{name}: {len(records)} records, statuses {nst}, file {os.path.getsize(path)/1e6:.2f} MB")


if __name__ == "__main__":
    for name in (sys.argv[1:] or list(SCENARIOS)):
        run(name, SCENARIOS[name])
