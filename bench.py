#!/usr/bin/env python3
"""Benchmark: home-MPC solves/sec (homes x timesteps) of the batched MI355X solver.

Workload (BASELINE.json configs[2], the configuration its metric is quoted on, "at 10k
homes"): a 10,000-home community (40 % base, 20 % pv_only, 20 % battery_only, 20 %
pv_battery), run_rbo_mpc closed loop at 15-min steps (dt = 4) with a 12 h horizon (H = 48),
S = 6, discount 0.92, TOU prices, int_mode round (the reference's MILP).  Inputs are
synthetic: NSRDB-shaped July weather (Houston-like) and homes drawn from the config.toml
ranges (no network for the reference data).  July, because with the reference's season
draw (1.1^k-scaled OAT noise, mpc_calc.py:222, 303-309) a 12 h horizon in January sends
nearly every home to the cooling-only mode and the fallback thermostat (tests/golden/c3_h48:
96/96), which would benchmark the fallback, not the solver; `--month 1` runs it anyway.

A "step" is one closed-loop timestep of the whole community: one solver launch per rank
(every home's MPC solve + state advance), the aggregate reduction and, with N > 1 GPUs, the
24-byte RCCL all-reduce.  The community is sharded over the ranks (strong scaling: --homes
is the community size).  `value` = homes x timed steps / max-over-ranks wall time.

Ranks: under torch.distributed.run (WORLD_SIZE set) each process is one rank and --gpus must
equal WORLD_SIZE; a plain `python bench.py --gpus N` starts the N rank processes itself (child
processes, before any GPU use) and exits with their status.  DRAGG_BENCH_BACKEND=gloo rehearses
N ranks on fewer GPUs (ranks share devices round-robin).

Also reported (rank 0): `roofline` of the solver kernel (algorithmic HBM bytes per launch
over the launch time measured with HIP events on the launch stream), `cpu_baseline` (N = 1
only): the repo's CPU restatement of the reference solve (oracle/, HiGHS MILP in place of
GLPK_MI) on this host's cores -- the committed >= 1,000-home-step run of the same workload
(`bench.py --cpu-only`, profiles/*/cpu_baseline_*.json, labelled as committed) with this run's
own bounded sample beside it (`in_run_sample`).
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=96)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--homes", type=int, default=10000, help="community size (sharded over the ranks)")
    ap.add_argument("--horizon-hours", type=int, default=12)
    ap.add_argument("--dt", type=int, default=4)
    ap.add_argument("--month", type=int, default=7, choices=[1, 4, 7, 10])
    ap.add_argument("--int-mode", default="round", choices=["round", "relax", "round_lp"])
    ap.add_argument("--cpu-seconds", type=float, default=60.0,
                    help="CPU baseline wall budget (0 = skip; with --cpu-only, 0 = no limit)")
    ap.add_argument("--cpu-workers", type=int, default=0, help="0 = the host cores this job may use")
    ap.add_argument("--cpu-home-steps", type=int, default=1000,
                    help="CPU baseline sample size (home-steps; stopped early at --cpu-seconds of wall time)")
    ap.add_argument("--cpu-steps-per-home", type=int, default=4,
                    help="CPU baseline: closed-loop steps per sampled home from t = 0 (configs[0] in full: 96 "
                         "with --homes 20 --cpu-home-steps 1920)")
    ap.add_argument("--cpu-milp-limit", type=float, default=300.0,
                    help="HiGHS time limit per CPU solve; solves that reach it are counted separately")
    ap.add_argument("--cpu-home-range", default=None,
                    help="CPU baseline: only the sampled homes [a:b) of the sample (a workload split by home over "
                         "several runs, e.g. configs[0] in full over two GPU-box calls; tools/merge_cpu_parts.py)")
    ap.add_argument("--cpu-only", action="store_true",
                    help="run only the CPU baseline (no GPU) and print its JSON (the committed full run)")
    ap.add_argument("--workload", default="rbo", choices=["rbo", "rl"],
                    help="rbo: run_rbo_mpc closed loop (configs[2], default); rl: configs[4], every step "
                         "is one RL reward-price action: price broadcast, --forecast-horizon rollout "
                         "re-solves of the community, the committed step, the sums to the host")
    ap.add_argument("--forecast-horizon", type=int, default=1, help="rl: rollout timesteps per action")
    ap.add_argument("--rl-price", default="smooth", choices=["smooth", "flat"],
                    help="rl: the agent's reward price per action: 'smooth' varies over the horizon "
                         "(-0.03 cos(k/3) + a per-action offset, the shape of test_gpu_configs.py's "
                         "configs[4] test: the price changes at every stage); 'flat' "
                         "is one constant per action (round 2's RL line)")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="diagnostic: time rank 0's strided shard of the community sharded this many ways, on "
                         "one GPU without the collectives (the per-GPU load of an N-GPU strong-scaling run)")
    ap.add_argument("--shard-rank", type=int, default=0,
                    help="with --shard-of N: which rank's shard to time (0..N-1)")
    ap.add_argument("--shard-max", action="store_true",
                    help="with --shard-of N: time EVERY rank's shard in turn (same steps each) and report the "
                         "slowest one -- the step time of an N-GPU strong-scaling run is its slowest rank's")
    ap.add_argument("--exact", action="store_true",
                    help="DRAGG_FLAG_EXACT (diagnostic): every chain the front DPs cannot take goes to the step-function DP")
    ap.add_argument("--no-overlap", action="store_true",
                    help="rbo: serial steps (no lag mode: every home's step t completes before step t + 1 starts); "
                         "= --steps-mode serial")
    ap.add_argument("--steps-mode", default="lag", choices=["lag", "adaptive", "serial"],
                    help="rbo: lag (lag mode from the first step), adaptive (serial steps until a step hands a chain "
                         "to the step-function DP, lag mode after), serial")
    ap.add_argument("--no-history", action="store_true",
                    help="skip the per-step history write (collected_data); a configs[2] run keeps it")
    ap.add_argument("--keep-crashing-homes", action="store_true",
                    help="keep battery homes whose t = 0 solve fails (the reference raises KeyError at t = 1)")
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------- CPU baseline
def host_cores():
    """The host cores this job may use: the affinity mask, the cgroup CPU quota and the job's
    worker cap (MAX_JOBS: the GPU box grants one GPU's job a share of the host's cores and sets it
    to that share) -- the smallest of them, and each of them for the record."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = float(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = float(f.read())
            quota = q / per if q > 0 else None
        except (OSError, ValueError):
            pass
    cap = int(os.environ["MAX_JOBS"]) if os.environ.get("MAX_JOBS", "").isdigit() else None
    n = min(x for x in (aff, math.ceil(quota) if quota else None, cap) if x)
    return max(1, n), {"affinity": aff, "cgroup_quota": quota, "max_jobs": cap, "os_cpu_count": os.cpu_count()}


def _cpu_worker(args):
    """Closed-loop oracle solves of a few homes (t = 0, 1, ...), each the reference's MILP solved by
    HiGHS, until the deadline or the home-step quota (runs before any GPU use).
    -> (home-steps, per-solve seconds, solves that reached the time limit)"""
    homes, env, deadline, milp_limit, steps_per_home, quota = args
    from oracle import mpc as M
    from scipy.optimize import milp, LinearConstraint, Bounds
    import numpy as np
    n, times, limited = 0, [], [0]

    def solver(P):
        """solve_problem's HiGHS call, recording whether the time limit cut it (HiGHS status 1)"""
        # the per-solve limit, cut to what is left of the sample's wall budget (a solve in flight
        # at the deadline ends there with its incumbent and is counted as time-limited)
        lim = milp_limit if not deadline else max(1.0, min(milp_limit, deadline - time.time()))
        res = milp(P["c"], constraints=[LinearConstraint(P["A_eq"], P["b_eq"], P["b_eq"]),
                                        LinearConstraint(P["A_ub"], -np.inf, P["b_ub"])],
                   integrality=P["integrality"], bounds=Bounds(-np.inf, np.inf),
                   options={"time_limit": lim, "mip_rel_gap": 1e-6, "presolve": True})
        if res.status == 1:
            limited[0] += 1
        if res.x is None:
            return ({2: "infeasible", 3: "unbounded"}.get(res.status, "solver_error"), None, None)
        x = res.x.copy()
        ii = P["integrality"] == 1
        x[ii] = np.floor(x[ii] + 0.5)
        return "optimal", x, float(P["c"] @ x)
    for home in homes:
        hc = M.home_const(home)
        hsh = {}
        rng = np.random.default_rng(1234)
        for t in range(steps_per_home):
            if (deadline and time.time() >= deadline) or n >= quota:
                return n, times, limited[0]
            t0 = time.time()
            # (RL workload: the reward price of action t, redis_set_current_values aggregator.py:671-675)
            env_t = dict(env, reward_price=env["rp_steps"][t]) if env.get("rp_steps") is not None else env
            try:
                M.run_home_step(hc, t, hsh, env_t, rng.standard_normal(hc.H), solver=solver)
            except Exception:
                break
            times.append(time.time() - t0)
            n += 1
    return n, times, limited[0]


def cpu_baseline(homes, env, seconds, workers, home_steps, milp_limit=300.0, steps_per_home=4, home_range=None):
    """The reference's per-home solve restated on the host (oracle/mpc.py: the reference's problem
    build, HiGHS MILP standing in for GLPK_MI, cleanup/fallback), one process per host core this
    job may use (one process per core), on `home_steps` home-steps of this workload
    (homes spread over the community, steps_per_home closed-loop steps each from t = 0), stopped
    early at `seconds` of wall time (0: no limit).  The rate is extrapolated to the whole workload
    (solves are independent across homes)."""
    import multiprocessing as mp
    import numpy as np
    cores, info = host_cores()
    workers = workers or cores
    deadline = time.time() + seconds if seconds > 0 else 0.0
    n_homes = max(workers, -(-home_steps // steps_per_home))
    picks = [homes[(i * 7919) % len(homes)] for i in range(n_homes)]
    if home_range:
        a_, b_ = (int(x) for x in home_range.split(":"))
        picks = picks[a_:b_]
        home_steps = min(home_steps, len(picks) * steps_per_home)
        workers = min(workers, len(picks))
    per = [picks[w::workers] for w in range(workers)]
    # a sample covering every step of every home (configs[0] in full) runs each home's whole loop
    quota = -(-home_steps // workers) if n_homes * steps_per_home > home_steps else 1 << 40
    t0 = time.time()
    with mp.get_context("fork").Pool(workers) as pool:
        res = pool.map(_cpu_worker, [(p, env, deadline, milp_limit, steps_per_home, quota) for p in per])
    wall = time.time() - t0
    n = sum(r[0] for r in res)
    times = [x for r in res for x in r[1]]
    limited = sum(r[2] for r in res)
    # the rate counts only solves that ran to their end: a solve cut by the per-solve limit or by the
    # sample's wall budget (its incumbent kept) is excluded from the count but its time is not
    done = n - limited
    return {"value": done / wall if wall > 0 else 0.0, "unit": "solves/s", "cores": workers, "host_cores": info,
            "home_range": home_range, "solve_cpu_s": float(np.sum(times)) if times else 0.0,
            "done_home_steps": done,
            "value_incl_cut_solves": n / wall if wall > 0 else 0.0,
            "kind": "port", "home_steps": n, "target_home_steps": home_steps, "time_limited_solves": limited,
            "extrapolated": True, "wall_s": wall,
            "median_solve_s": float(np.median(times)) if times else None,
            "mean_solve_s": float(np.mean(times)) if times else None,
            "sample": f"{n} home-steps of this workload ({len(picks)} homes spread over the community, up to "
                      f"{steps_per_home} closed-loop steps each from t = 0) on {workers} worker processes, one per "
                      f"host core this job may use (affinity {info['affinity']}, cgroup quota {info['cgroup_quota']}, "
                      f"MAX_JOBS {info['max_jobs']}), solved by oracle/mpc.py (the reference's problem build, "
                      f"HiGHS MILP with mip_rel_gap 1e-6 in place of GLPK_MI, time limit {milp_limit:.0f} s per "
                      f"solve, cut to the sample's remaining wall budget: {limited} solves reached a limit; the rate "
                      f"counts the {done} that ran to their end) in {wall:.1f} s wall; "
                      f"median {np.median(times) if times else float('nan'):.2f} s per solve; extrapolated to the "
                      f"whole workload (home solves are independent)"}


def cpu_workload_key(n_total, Hh, dt, month, rl_price=None):
    """The identity of a CPU-baseline workload (bench.py --cpu-only writes it into its JSON)."""
    w = f"{n_total} homes, H={Hh * dt} ({Hh} h), {60 // dt}-min steps, month {month}, "
    if rl_price:
        return w + f"run_rl_agg reward price ({rl_price}), closed loop from t = 0"
    return w + "run_rbo_mpc closed loop from t = 0"


def committed_cpu_baseline(workload=None):
    """The committed full CPU-baseline run of this workload (bench.py --cpu-only on the GPU box,
    >= 1,000 home-steps): profiles/*/cpu_baseline_*.json whose `workload` is this one,
    newest round first."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "cpu_baseline_*.json")), reverse=True):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        if workload is not None and d.get("workload") != workload:
            continue
        if (d.get("home_steps") or 0) < 1000:
            continue
        return {k: d.get(k) for k in ("value", "unit", "cores", "kind", "home_steps", "time_limited_solves",
                                     "median_solve_s", "wall_s", "workload", "sample")} | {"source": os.path.relpath(f, ROOT)}
    return None


def headline_cpu_baseline(full, sample):
    """`cpu_baseline` of the line: the committed >= 1,000-home-step run of this workload (BASELINE.md:
    35-37; a bounded in-run sample over-represents short solves), labelled as committed, with this run's
    own bounded sample beside it; without a committed run, the in-run sample."""
    if full is None:
        return sample
    out = dict(full)
    out["measured_in_this_run"] = False
    out["sample"] = (f"COMMITTED run ({full['source']}, bench.py --cpu-only on a GPU box of this pool): "
                     + (full.get("sample") or ""))
    out["in_run_sample"] = sample
    return out


# ----------------------------------------------------------------------------- roofline
def bytes_per_launch(batch, success_frac):
    """Algorithmic HBM bytes of one solver launch: per home the parameters,
    type, the hourly draw rows of the window and the hash state read; the hash fields,
    status/objective outputs and (on success) the forecast fields written."""
    import numpy as np
    H, dt = batch.H, batch.dt
    types = batch.types_host
    n = len(types)
    rd = n * (22 * 8 + 4 + ((H + 1) // dt + 2) * 8 + 6 * 8)
    nfc = 10 + 2 * ((types & 1) != 0) + 3 * ((types & 2) != 0)   # forecast keys per home type
    wr = n * (19 * 8 + 4 + 4 + 8 + 8) + success_frac * float(np.sum(nfc)) * H * 8
    env = 3 * (H + 1) * 8
    return rd + wr + env


def measured_pmc(workload_key):
    """The committed rocprofv3 passes of EXACTLY this command's workload and timed window
    (profiles/*/traffic.json, written by tools/make_traffic.py from the kernel trace and the PMC
    passes of the same bench command): HBM bytes per step (FETCH_SIZE x 2 + WRITE_SIZE,
    MI355X_MICROARCH.md HBM section), SQ counters per step and the profiled kernel time per
    step, all over the timed steps only."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic*.json")), reverse=True):
        try:
            with open(f) as fh:
                tj = json.load(fh)
        except (OSError, ValueError):
            continue
        if tj.get("workload") == workload_key:
            return tj, os.path.relpath(f, ROOT)
    return {}, None


# Issue model of the VALU bound (MI355X_MICROARCH.md "Wave scheduling": a SIMD-32 issues a
# wave64 VALU instruction over 2 cycles; fp64 add/mul/fma run at half the fp32 rate (78.6 vs
# 157.3 TFLOPS): 4 cycles; fp64 transcendental (v_rcp_f64) a quarter of that: 8).  The rest
# (int32/int64, conversions, moves, compares, lane ops) is priced at 2 cycles.  Peak: 256 CUs x
# 4 SIMDs x 2.4 GHz SIMD-cycles per second.
N_SIMD, CLOCK = 256 * 4, 2.4e9
LDS_PEAK_TBS = 150.0      # ds_read_b64/b128 with every CU streaming (MI355X_MICROARCH.md, LDS)


def valu_cycles(sq):
    f64 = sq.get("SQ_INSTS_VALU_ADD_F64", 0) + sq.get("SQ_INSTS_VALU_MUL_F64", 0) + sq.get("SQ_INSTS_VALU_FMA_F64", 0)
    trans = sq.get("SQ_INSTS_VALU_TRANS_F64", 0)
    return 2.0 * (sq["SQ_INSTS_VALU"] - f64 - trans) + 4.0 * f64 + 8.0 * trans


def extra_rooflines(pmc, src):
    """The bounds that do limit the kernel, from the committed profile of
    this very command (counters per step over the timed steps, divided by the kernel time per step
    of the SAME profiled run, so each number recomputes from profiles/).  Without such a profile:
    none (no borrowed or window-mismatched counters)."""
    sq = pmc.get("sq_per_step", {})
    ks_ms = pmc.get("kernel_ms_per_step")
    if "SQ_INSTS_VALU" not in sq or not ks_ms:
        return {}
    ks = ks_ms * 1e-3
    out = {}
    if "SQ_INSTS_VALU_FMA_F64" in sq:
        cyc = valu_cycles(sq)
        out["roofline_valu"] = {
            "bound": "valu-issue", "achieved": cyc / ks / 1e12, "peak": N_SIMD * CLOCK / 1e12,
            "unit": "T SIMD-cycles/s", "frac": cyc / ks / (N_SIMD * CLOCK),
            "valu_per_step": sq["SQ_INSTS_VALU"],
            "fp64_valu_per_step": sum(sq.get(f"SQ_INSTS_VALU_{c}_F64", 0) for c in ("ADD", "MUL", "FMA", "TRANS")),
            "profiled_kernel_ms_per_step": ks_ms,
            "model": "2 cycles per wave64 VALU instruction, 4 per fp64 add/mul/fma, 8 per fp64 transcendental",
            "source": src}
    if "SQ_ACTIVE_INST_VALU" in sq and "SQ_WAVE_CYCLES" in sq:
        out["valu_busy_per_wave"] = sq["SQ_ACTIVE_INST_VALU"] / sq["SQ_WAVE_CYCLES"]
    if "SQ_INSTS_LDS" in sq:
        # upper estimate of LDS bytes: every LDS instruction moving 8 B for all 64 lanes
        b = sq["SQ_INSTS_LDS"] * 64 * 8
        out["roofline_lds"] = {
            "bound": "lds", "achieved": b / ks / 1e12, "peak": LDS_PEAK_TBS, "unit": "TB/s",
            "frac": b / ks / 1e12 / LDS_PEAK_TBS, "lds_instr_per_step": sq["SQ_INSTS_LDS"],
            "bank_conflict_share": (sq["SQ_LDS_BANK_CONFLICT"] / sq["SQ_LDS_IDX_ACTIVE"]
                                    if sq.get("SQ_LDS_IDX_ACTIVE") else None),
            "profiled_kernel_ms_per_step": ks_ms,
            "assumption": "8 B x 64 lanes per LDS instruction (an upper estimate; most are b64)", "source": src}
    if "SQ_WAIT_ANY" in sq and "SQ_WAVE_CYCLES" in sq:
        out["wave_cycle_shares"] = {"wait_any": sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"],
                                    "issue_any": (sq["SQ_ACTIVE_INST_ANY"] / sq["SQ_WAVE_CYCLES"]
                                                  if "SQ_ACTIVE_INST_ANY" in sq else None), "source": src}
    fs = pmc.get("front_stats")
    if fs and fs.get("children_per_step"):
        out["dp_work"] = {"unit": "G label relaxations/s", "achieved": fs["children_per_step"] / ks / 1e9,
                          "children_per_step": fs["children_per_step"],
                          "front_mean": [fs["front_mean_T"], fs["front_mean_W"]],
                          "profiled_kernel_ms_per_step": ks_ms,
                          "definition": "one label relaxation = one child (parent label, duty) of a front DP stage: "
                                        "state and cost update, box test, bucket positions, dominance tests",
                          "source": src}
    return out


def occupancy(batch):
    """Registers, spills, LDS and resident homes per CU of the step's launches, as the code object
    and the runtime report them on this device (dragg_mpc_kernel_info_get)."""
    from dragg_amd import _lib as L
    info = L.kernel_info(batch.dims)
    info["hot"]["waves_per_simd"] = info["hot"]["blocks_per_cu"] * info["hot"]["threads"] / 64 / 4.0
    return info | {"source": "hipFuncGetAttributes + hipOccupancyMaxActiveBlocksPerMultiprocessor (live, this device)"}


def traffic_key(n_total, H, dt, month, int_mode, world, workload="rbo", steps=None, warmup=None, rl_price=None,
                fh=0, shard_of=0, shard_rank=None, steps_mode=None):
    """The identity of a profiled command: workload, community, horizon, the timed window, and (since
    round 6) the shard a --shard-of line times (`shard_rank`: its rank, or "max" for --shard-max) and
    how the steps run (`steps_mode`: "lag", "serial" or "adaptive").  A line takes counters only from
    a pass whose key is its own; keys without the last two parts are the profiles of rounds <= 5."""
    w = f"{n_total} homes, H={H}, dt={dt}, month {month}, int_mode={int_mode}, {world} rank(s)"
    if workload == "rl":
        w += f", rl ({rl_price} price, forecast_horizon {fh})"
    w += f", timed steps {warmup}..{(warmup or 0) + (steps or 0) - 1}"
    if shard_of and shard_of > 1:
        w += f", shard {shard_rank} of {shard_of}"
    if steps_mode:
        w += f", {steps_mode} steps"
    return w


def steps_mode(agg):
    """How the timed steps ran: "lag" (lag mode from the first step), "adaptive" (serial steps until a
    step hands a chain to the step-function DP, lag mode after), "serial"."""
    if not agg.overlap:
        return "serial"
    return "adaptive" if getattr(agg, "adaptive", False) else "lag"


def window(warmup, steps, dt, month, rl):
    """The simulated time the timed steps cover (the per-step cost varies over a day)."""
    def clock(k):
        m = k * 60 // dt
        return f"day {m // 1440 + 1} {m // 60 % 24:02d}:{m % 60:02d}"
    return {"steps": [warmup, warmup + steps], "sim_hours": [warmup / dt, (warmup + steps) / dt],
            "clock": f"{clock(warmup)} to {clock(warmup + steps)} (month {month}; step k starts at k x {60 // dt} min)",
            "note": "timed steps k in [warmup, warmup + steps); the step cost varies with the time of day (tariff "
                    "boundaries, daylight), so a window is not the full-day average" +
                    ("; rl: every step is one action = rollout solves + the committed step" if rl else "")}


from dragg_amd.community import reference_completable  # noqa: E402  (re-exported for the tools)


def bench_community(args):
    """The bench's synthetic community and weather (seeded; the same for every rank and tool)."""
    from dragg_amd.community import synthetic_homes, synthetic_weather
    dt, Hh = args.dt, args.horizon_hours
    sim_hours = math.ceil((args.warmup + args.steps) / dt)
    days = math.ceil((sim_hours + Hh + 2) / 24) + 1
    homes = synthetic_homes(args.homes, seed=12, days=days, dt=dt, horizon_hours=Hh)
    oat, ghi, tou = synthetic_weather(days, dt, sim_hours, seed=3, month=args.month)
    return homes, oat, ghi, tou


def spawn_ranks(args):
    """`bench.py --gpus N` without a launcher: start N rank processes of this same command, one per
    GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run sets them), wait
    for all of them and return the first failing exit code (0 when every rank succeeded).  Called
    before anything touches the GPU; the ranks are child processes (no exec), rank 0 prints the
    line.  One rank failing ends the others (their own process ids)."""
    import socket
    import subprocess
    backend = os.environ.get("DRAGG_BENCH_BACKEND", "nccl")
    if backend == "nccl":
        import torch                       # device_count() does not initialise the GPU on this image
        n_dev = torch.cuda.device_count()
        if n_dev < args.gpus:
            print(f"bench.py: --gpus {args.gpus} but {n_dev} GPU(s) visible (DRAGG_BENCH_BACKEND=gloo rehearses "
                  f"several ranks on fewer GPUs)", file=sys.stderr)
            return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:            # the others would wait for the failed rank forever
                    q.kill()
        if live:
            time.sleep(0.2)
    return rc


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and not args.cpu_only:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and not args.cpu_only:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were launched")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dt, Hh = args.dt, args.horizon_hours
    total_steps = args.warmup + args.steps
    n_total = args.homes
    homes, oat, ghi, tou = bench_community(args)

    rl = args.workload == "rl"
    import numpy as np
    H_ = Hh * dt
    off = np.random.default_rng(5).uniform(-0.02, 0.02, (max(total_steps, args.cpu_steps_per_home), 1))
    if args.rl_price == "smooth":       # changes at every stage (test_gpu_configs.py configs[4])
        prices = off + (-0.03 * np.cos(np.arange(H_) / 3.0))[None, :]
    else:
        prices = off * np.ones((1, H_))

    cpu = None
    env = {"oat": oat, "ghi": ghi, "tou": tou, "start_hour_index": 0, "reward_price": [0.0],
           "rp_steps": [list(map(float, prices[t])) for t in range(args.cpu_steps_per_home)] if rl else None}
    cpu_args = (args.cpu_seconds, args.cpu_workers, args.cpu_home_steps, args.cpu_milp_limit, args.cpu_steps_per_home)
    if args.cpu_only:
        out = cpu_baseline(homes, env, *cpu_args, home_range=args.cpu_home_range)
        out["workload"] = cpu_workload_key(n_total, Hh, dt, args.month, args.rl_price if rl else None)
        print(json.dumps(out))
        return
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(homes, env, *cpu_args)

    import torch
    from dragg_amd.aggregator import DeviceAggregator
    # one rank per GPU over RCCL (backend "nccl").  DRAGG_BENCH_BACKEND=gloo rehearses the
    # multi-rank path with several ranks on fewer GPUs (ranks share devices round-robin)
    backend = os.environ.get("DRAGG_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    # (after the CPU leg: its worker processes fork before anything touches the GPU)
    replaced = None
    if not args.keep_crashing_homes:
        homes, replaced = reference_completable(homes, oat, ghi, tou, seed=12)
    if world > 1:
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.distributed.init_process_group(backend)
    # keep_history: the per-step hash history (collected_data, aggregator.py:737-748) is written
    # inside the timed steps, as a configs[2] run does
    shard = args.shard_of > 1 and world == 1
    fh = args.forecast_horizon if rl else 0

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
            torch.cuda.synchronize()

    def timed(shard_rank):
        """Build the aggregator (this rank's shard, or shard `shard_rank` of --shard-of on one GPU),
        run the warmup steps, then time exactly --steps steps between barriers."""
        agg = DeviceAggregator(homes, oat, ghi, tou, 0, total_steps, reward_price=[0.0],
                               int_mode=args.int_mode, seed=12, rank=shard_rank if shard else rank,
                               world=args.shard_of if shard else world,
                               keep_history=not args.no_history, exact=args.exact,
                               overlap=not (rl or args.no_overlap or args.steps_mode == "serial"),
                               adaptive=args.steps_mode == "adaptive")
        if shard:
            agg.world = 1                     # one GPU: no collectives (the shard's own sums)
        stream = torch.cuda.current_stream()

        def action(k):
            """rl: one reward-price action (random stand-in for the host agent's choice)."""
            agg.set_reward_price(prices[k])
            agg.forecast(fh)

        for k in range(args.warmup):
            if rl:
                action(k)
            agg.run_iteration()
            agg.collect_data(defer=not rl)
        if not rl:
            agg.reduce_history()
        barrier()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        t0 = time.perf_counter()
        for k in range(args.steps):
            evs[k][0].record(stream)            # rl: the action's rollout solves are timed with its step
            if rl:
                action(args.warmup + k)
            agg.run_iteration()
            evs[k][1].record(stream)
            if rl:
                agg.collect_data().tolist()         # the agent reads the community sums on the host
            else:
                agg.collect_data(defer=True)        # run_rbo_mpc: no feedback, one reduction at the end
        if not rl:
            agg.reduce_history()
        barrier()
        return agg, time.perf_counter() - t0, evs

    shard_times = None
    if shard and args.shard_max:
        # every shard in turn; the slowest one is what an N-GPU run waits for (its aggregator is kept)
        runs = []
        for r in range(args.shard_of):
            agg, el, evs = timed(r)
            runs.append((el, r))
            if el >= max(x[0] for x in runs):
                keep = (agg, el, evs, r)
            del agg
            torch.cuda.empty_cache()
        agg, elapsed, evs, slow_rank = keep
        shard_times = {"ms_per_step": [round(el / args.steps * 1e3, 4) for el, _ in sorted(runs, key=lambda x: x[1])],
                       "slowest_rank": slow_rank}
    else:
        slow_rank = args.shard_rank if shard else rank
        agg, elapsed, evs = timed(slow_rank)
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        torch.distributed.all_reduce(e, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(e.item())
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    # per-status counts of the timed steps over EVERY rank (one small all-reduce after timing)
    st = agg.status_hist[args.warmup:total_steps]
    from dragg_amd import _lib as L
    names = L.STATUS_NAMES
    counts = torch.stack([(st == i).sum() for i in range(len(names))]).to(torch.float64)
    if world > 1:
        torch.distributed.all_reduce(counts)
    counts = counts.cpu().tolist()
    # the timed solves' integer paths over every rank (int_path): approximate schedules (bits 0-11), the
    # step-function DP (bit 15)
    paths = agg.approx_counts(args.warmup, total_steps)
    # the homes every rank solved (strided shards: the rank's share of the community)
    per_rank = torch.tensor([agg.batch.N], dtype=torch.int64, device="cuda" if backend == "nccl" else "cpu")
    if world > 1:
        got = [torch.zeros_like(per_rank) for _ in range(world)]
        torch.distributed.all_gather(got, per_rank)
        homes_per_rank = [int(x.item()) for x in got]
        dist_world = torch.distributed.get_world_size()
    else:
        homes_per_rank, dist_world = [int(agg.batch.N)], 1
    stat_counts = {name: int(c) for name, c in zip(names, counts)}
    success = stat_counts["optimal"] / max(1, sum(stat_counts.values()))
    stat_counts.update(paths)
    solves = (agg.batch.N if shard else n_total) * args.steps * (1 + fh)
    value = solves / elapsed
    if rank == 0:
        H = agg.batch.H
        workload = (f"{n_total} homes x {args.steps} closed-loop {60 // dt}-min steps, H={H} "
                    f"({Hh} h), month {args.month}, run_rbo_mpc, int_mode={args.int_mode}")
        if rl:
            workload = (f"{n_total} homes x {args.steps} RL reward-price actions ({args.rl_price} price), each "
                        f"{fh} rollout timestep(s) + the committed {60 // dt}-min step, H={H} ({Hh} h), month "
                        f"{args.month}, run_rl_agg, int_mode={args.int_mode}")
        alg_bytes = bytes_per_launch(agg.batch, success) * (1 + fh)     # rl: per action (rollouts + commit)
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        key = traffic_key(n_total, H, dt, args.month, args.int_mode, world, args.workload, args.steps, args.warmup,
                          args.rl_price if rl else None, fh, args.shard_of if shard else 0,
                          ("max" if shard_times else slow_rank) if shard else None, steps_mode(agg))
        pmc, traffic_src = measured_pmc(key)
        traffic = pmc.get("bytes_per_step")
        out = {
            "metric": "home-MPC solves/sec (homes x steps)", "value": value, "unit": "solves/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (NSRDB-shaped weather, config.toml-range homes, seeded)",
            "community": {"battery_home_swaps": replaced,
                          "note": "battery homes whose t = 0 solve fails (the reference raises KeyError at "
                                  "t = 1, mpc_calc.py:280-289; the failure follows the index-keyed season "
                                  "draw) swapped with homes without a battery, so the run is one the "
                                  "reference completes; null = kept (--keep-crashing-homes)"},
            "config": {"workload": workload, "baseline_config": "BASELINE.json configs[4]" if rl else "BASELINE.json configs[2]",
                       "homes_total": n_total, "homes_per_gpu": agg.batch.N, "homes_per_rank": homes_per_rank,
                       "dist_world_size": dist_world, "dist_backend": backend if world > 1 else None,
                       "timing": "max over ranks of each rank's wall time between barriers" if world > 1
                                 else "wall time between barriers",
                       "global_batch": n_total,
                       "horizon": H, "mix": "40/20/20/20 base/pv/battery/pv_battery",
                       "parallelism": f"homes sharded x{world}"},
            "shard_emulation": ({"shard_of": args.shard_of, "shard_rank": slow_rank, "homes": agg.batch.N,
                                 "max_over_shards": shard_times,
                                 "note": ("diagnostic: EVERY rank's strided shard in turn on one GPU, no collectives; "
                                          "the line is the slowest shard's (an N-GPU strong-scaling step waits for its "
                                          "slowest rank); value counts that shard's solves" if shard_times else
                                          f"diagnostic: rank {slow_rank}'s strided shard alone on one GPU (the per-GPU "
                                          "load of an N-GPU strong-scaling run), no collectives; value counts the "
                                          "shard's solves")} if shard else None),
            "window": window(args.warmup, args.steps, dt, args.month, rl),
            "history_written": not args.no_history,
            "lag_mode": bool(agg.overlap),
            "steps_mode": steps_mode(agg),
            "lag_from_step": getattr(agg, "lag_from", None),
            "sim_wall_s": elapsed,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": 8000.0, "unit": "GB/s",
                         "frac": achieved / 8000.0,
                         "traffic": (traffic / (kern_ms * 1e-3) / 1e9) if traffic else None,
                         "traffic_bytes_per_step": traffic, "traffic_source": traffic_src,
                         "profile_key": key,
                         "profiled_kernel_ms_per_step": pmc.get("kernel_ms_per_step"),
                         "kernel": (f"mpc_direct_kernel (DM_FRONT + DM_BUCKET launches of a step)"
                                    if args.int_mode == "round" else "mpc_home_kernel"),
                         "kernel_ms": kern_ms,
                         "algorithmic_bytes_per_step": alg_bytes,
                         "unit_note": "one step = the hot launch + the second launch of one timestep; HIP events "
                                      "on the launch stream around run_iteration (lag mode: the main pass; the "
                                      "side stream's step-function DP runs beside it and is in the wall time)"},
            "cpu_baseline": (headline_cpu_baseline(committed_cpu_baseline(cpu_workload_key(n_total, Hh, dt, args.month,
                                                                                            args.rl_price if rl else None)), cpu)
                             if rank == 0 else None),       # (world > 1: the committed run only)
            "status_counts": stat_counts,
            # RL: the headline counts the rollout re-solves too; the committed steps alone:
            "committed_solves_per_s": n_total * args.steps / elapsed,
        }
        out.update(extra_rooflines(pmc, traffic_src))
        out["occupancy"] = occupancy(agg.batch) | (
            {"wave_cycle_shares": out.pop("wave_cycle_shares")} if "wave_cycle_shares" in out else {})
        print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
