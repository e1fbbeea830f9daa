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

Also reported (rank 0): `roofline` of the solver kernel (algorithmic HBM bytes per launch
over the launch time measured with HIP events on the launch stream), `cpu_baseline` (N = 1
only): the repo's CPU restatement of the reference solve (oracle/, HiGHS MILP in place of
GLPK_MI) timed on this host's cores on a bounded sample of the same workload.
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=96)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--homes", type=int, default=10000, help="community size (sharded over the ranks)")
    ap.add_argument("--horizon-hours", type=int, default=12)
    ap.add_argument("--dt", type=int, default=4)
    ap.add_argument("--month", type=int, default=7, choices=[1, 4, 7, 10])
    ap.add_argument("--int-mode", default="round", choices=["round", "relax", "round_lp"])
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--cpu-workers", type=int, default=0)
    ap.add_argument("--cpu-home-steps", type=int, default=1000,
                    help="CPU baseline sample size (home-steps; stopped at --cpu-seconds of wall time)")
    ap.add_argument("--workload", default="rbo", choices=["rbo", "rl"],
                    help="rbo: run_rbo_mpc closed loop (configs[2], default); rl: configs[4], every step "
                         "is one RL reward-price action: price broadcast, --forecast-horizon rollout "
                         "re-solves of the community, the committed step, the sums to the host")
    ap.add_argument("--forecast-horizon", type=int, default=1, help="rl: rollout timesteps per action")
    ap.add_argument("--keep-crashing-homes", action="store_true",
                    help="keep battery homes whose t = 0 solve fails (the reference raises KeyError at t = 1)")
    return ap.parse_args()


def reference_completable(homes, oat, ghi, tou, rounds=8):
    """A community the reference completes.  A battery home whose t = 0 solve fails leaves no
    e_batt_opt in its hash, and the reference raises KeyError('e_batt_opt') at t = 1
    (mpc_calc.py:280-289).  The failures come from the season draw (keyed by the home's index:
    a "winter" draw on a hot day leaves the cooling duty at zero), not from the home's
    parameters, so each such battery home swaps places with a home without a battery (whose
    failed t = 0 solve the reference survives) until the t = 0 step solves every battery home.
    Deterministic: every rank builds the same community.  -> (homes, swaps)"""
    import torch
    from dragg_amd import _lib as L
    from dragg_amd.mpc import MPCBatch
    homes, swaps = list(homes), 0
    donors = [j for j in range(len(homes) - 1, -1, -1) if "battery" not in homes[j]["type"]]
    for _ in range(rounds):
        b = MPCBatch(homes, oat, ghi, tou, 0, [0.0], int_mode="round", seed=12)
        b.step(0)
        st = b.status.cpu().numpy()
        del b
        torch.cuda.empty_cache()
        bad = [i for i, h in enumerate(homes) if "battery" in h["type"] and st[i] != L.ST_OPTIMAL]
        if not bad or not donors:
            break
        for i in bad:
            if not donors:
                break
            j = donors.pop(0)
            homes[i], homes[j] = homes[j], homes[i]
            swaps += 1
    return homes, swaps


# ----------------------------------------------------------------------------- CPU baseline
def _cpu_worker(args):
    """Closed-loop oracle solves of a few homes (t = 0, 1, ...), each solve a HiGHS MILP to the
    reference's stopping rule, until the deadline or the home-step quota (runs before any GPU use)."""
    homes, env, deadline, milp_limit, steps_per_home, quota = args
    from oracle import mpc as M
    import numpy as np
    n, times = 0, []
    for home in homes:
        hc = M.home_const(home)
        hsh = {}
        rng = np.random.default_rng(1234)

        def solver(P):
            return M.solve_problem(P, integer=True, time_limit=milp_limit)
        for t in range(steps_per_home):
            if time.time() >= deadline or n >= quota:
                return n, times
            t0 = time.time()
            try:
                M.run_home_step(hc, t, hsh, env, rng.standard_normal(hc.H), solver=solver)
            except Exception:
                break
            times.append(time.time() - t0)
            n += 1
    return n, times


def cpu_baseline(homes, env, seconds, workers, home_steps, steps_per_home=4):
    """The reference's per-home solve restated on the host (oracle/mpc.py: the reference's
    problem build, HiGHS MILP standing in for GLPK_MI, cleanup/fallback), one process per worker,
    on a sample of this workload's home-steps: `home_steps` of them (homes spread over the
    community, steps_per_home closed-loop steps each), stopped at `seconds` of wall time.  The
    rate is extrapolated to the whole workload (solves are independent across homes)."""
    import multiprocessing as mp
    import numpy as np
    cores = len(os.sched_getaffinity(0))
    workers = workers or max(1, min(16, cores))
    milp_limit = 10.0
    deadline = time.time() + seconds
    n_homes = max(workers, -(-home_steps // steps_per_home))
    picks = [homes[(i * 7919) % len(homes)] for i in range(n_homes)]
    per = [picks[w::workers] for w in range(workers)]
    quota = -(-home_steps // workers)
    t0 = time.time()
    with mp.get_context("fork").Pool(workers) as pool:
        res = pool.map(_cpu_worker, [(p, env, deadline, milp_limit, steps_per_home, quota) for p in per])
    wall = time.time() - t0
    n = sum(r[0] for r in res)
    times = [x for r in res for x in r[1]]
    return {"value": n / wall if wall > 0 else 0.0, "unit": "solves/s", "cores": workers, "host_cores": cores,
            "kind": "port", "home_steps": n, "extrapolated": True,
            "sample": f"{n} home-steps of this workload ({len(picks)} homes spread over the community, up to "
                      f"{steps_per_home} closed-loop steps each from t = 0, {workers} worker processes on "
                      f"{cores} host cores) solved by oracle/mpc.py (the reference's problem build, HiGHS MILP in "
                      f"place of GLPK_MI, time_limit {milp_limit:.0f}s/solve) in {wall:.1f}s wall; median "
                      f"{np.median(times) if times else float('nan'):.2f}s per solve; the rate is extrapolated to "
                      f"the whole workload (home solves are independent)"}


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
    """The committed rocprofv3 PMC passes of this workload (profiles/*/traffic.json): HBM
    bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE, MI355X_MICROARCH.md §HBM) and the SQ
    counters per launch."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic.json")), reverse=True):
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


def extra_rooflines(pmc, kern_ms, lds_bytes_per_home, src):
    """The bounds that do limit the kernel, from the committed PMC passes of
    this workload (per solver step) and the step's kernel time measured in this run."""
    sq = pmc.get("sq_per_launch", {})
    if "SQ_INSTS_VALU" not in sq:
        return {}
    ks = kern_ms * 1e-3
    out = {}
    if "SQ_INSTS_VALU_FMA_F64" in sq:
        cyc = valu_cycles(sq)
        out["roofline_valu"] = {
            "bound": "valu-issue", "achieved": cyc / ks / 1e12, "peak": N_SIMD * CLOCK / 1e12,
            "unit": "T SIMD-cycles/s", "frac": cyc / ks / (N_SIMD * CLOCK),
            "valu_per_launch": sq["SQ_INSTS_VALU"],
            "fp64_valu_per_launch": sum(sq.get(f"SQ_INSTS_VALU_{c}_F64", 0) for c in ("ADD", "MUL", "FMA", "TRANS")),
            "model": "2 cycles per wave64 VALU instruction, 4 per fp64 add/mul/fma, 8 per fp64 transcendental",
            "source": src}
    if "SQ_ACTIVE_INST_VALU" in sq and "SQ_WAVE_CYCLES" in sq:
        out["valu_busy_per_wave"] = sq["SQ_ACTIVE_INST_VALU"] / sq["SQ_WAVE_CYCLES"]
    if "SQ_INSTS_LDS" in sq:
        # upper estimate of LDS bytes: every LDS instruction moving 8 B for all 64 lanes
        b = sq["SQ_INSTS_LDS"] * 64 * 8
        out["roofline_lds"] = {
            "bound": "lds", "achieved": b / ks / 1e12, "peak": LDS_PEAK_TBS, "unit": "TB/s",
            "frac": b / ks / 1e12 / LDS_PEAK_TBS, "lds_instr_per_launch": sq["SQ_INSTS_LDS"],
            "bank_conflict_share": (sq["SQ_LDS_BANK_CONFLICT"] / sq["SQ_LDS_IDX_ACTIVE"]
                                    if sq.get("SQ_LDS_IDX_ACTIVE") else None),
            "assumption": "8 B x 64 lanes per LDS instruction (an upper estimate; most are b64)", "source": src}
    homes_per_cu = (160 * 1024) // max(1, lds_bytes_per_home)
    out["occupancy"] = {"lds_bytes_per_home": lds_bytes_per_home, "homes_per_cu_lds": homes_per_cu,
                        "waves_per_simd": min(homes_per_cu / 4.0, 3.0),
                        "limit": (f"LDS: {homes_per_cu} one-wave workgroups (homes) per CU; 168 VGPRs allow 3 waves "
                                  "per SIMD (12 per CU)"),
                        "wait_share": (sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"] if "SQ_WAIT_ANY" in sq else None),
                        "issue_share": (sq["SQ_ACTIVE_INST_ANY"] / sq["SQ_WAVE_CYCLES"]
                                        if "SQ_ACTIVE_INST_ANY" in sq else None)}
    fs = pmc.get("front_stats")
    if fs:
        out["dp_work"] = {"unit": "G label relaxations/s", "achieved": fs["children_per_launch"] / ks / 1e9,
                          "children_per_launch": fs["children_per_launch"],
                          "front_mean": [fs["front_mean_T"], fs["front_mean_W"]],
                          "definition": "one label relaxation = one child (parent label, duty) of a front DP stage: "
                                        "state and cost update, box test, bucket positions, dominance tests",
                          "source": src}
    return out


def traffic_key(n_total, H, dt, month, int_mode, world):
    return f"{n_total} homes, H={H}, dt={dt}, month {month}, int_mode={int_mode}, {world} rank(s)"


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    from dragg_amd.community import synthetic_homes, synthetic_weather
    dt, Hh = args.dt, args.horizon_hours
    total_steps = args.warmup + args.steps
    sim_hours = math.ceil(total_steps / dt)
    days = math.ceil((sim_hours + Hh + 2) / 24) + 1
    n_total = args.homes
    homes = synthetic_homes(n_total, seed=12, days=days, dt=dt, horizon_hours=Hh)
    oat, ghi, tou = synthetic_weather(days, dt, sim_hours, seed=3, month=args.month)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        env = {"oat": oat, "ghi": ghi, "tou": tou, "start_hour_index": 0, "reward_price": [0.0]}
        cpu = cpu_baseline(homes, env, args.cpu_seconds, args.cpu_workers, args.cpu_home_steps)

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
        homes, replaced = reference_completable(homes, oat, ghi, tou)
    if world > 1:
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.distributed.init_process_group(backend)
    agg = DeviceAggregator(homes, oat, ghi, tou, 0, total_steps, reward_price=[0.0],
                           int_mode=args.int_mode, seed=12, rank=rank, world=world, keep_history=False)
    stream = torch.cuda.current_stream()

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
            torch.cuda.synchronize()

    rl = args.workload == "rl"
    fh = args.forecast_horizon if rl else 0
    import numpy as np
    prices = np.random.default_rng(5).uniform(-0.02, 0.02, (total_steps, 1)) * np.ones((1, Hh * dt))

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
        if rl:
            action(args.warmup + k)
        evs[k][0].record(stream)
        agg.run_iteration()
        evs[k][1].record(stream)
        if rl:
            agg.collect_data().tolist()         # the agent reads the community sums on the host
        else:
            agg.collect_data(defer=True)        # run_rbo_mpc: no feedback, one reduction at the end
    if not rl:
        agg.reduce_history()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        torch.distributed.all_reduce(e, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(e.item())
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    # per-status counts of the timed steps over EVERY rank (one small all-reduce after timing)
    st = agg.status_hist[args.warmup:total_steps]
    names = ["optimal", "infeasible", "infeasible_cert", "max_iter", "round_fail", "err_parse", "err_missing"]
    counts = torch.stack([(st == i).sum() for i in range(len(names))]).to(torch.float64)
    if world > 1:
        torch.distributed.all_reduce(counts)
    counts = counts.cpu().tolist()
    stat_counts = {name: int(c) for name, c in zip(names, counts)}
    success = stat_counts["optimal"] / max(1, sum(stat_counts.values()))
    solves = n_total * args.steps * (1 + fh)
    value = solves / elapsed
    if rank == 0:
        H = agg.batch.H
        workload = (f"{n_total} homes x {args.steps} closed-loop {60 // dt}-min steps, H={H} "
                    f"({Hh} h), month {args.month}, run_rbo_mpc, int_mode={args.int_mode}")
        if rl:
            workload = (f"{n_total} homes x {args.steps} RL reward-price actions, each {fh} rollout "
                        f"timestep(s) + the committed {60 // dt}-min step, H={H} ({Hh} h), month {args.month}, "
                        f"run_rl_agg, int_mode={args.int_mode}")
        achieved = bytes_per_launch(agg.batch, success) / (kern_ms * 1e-3) / 1e9
        pmc, traffic_src = measured_pmc(traffic_key(n_total, H, dt, args.month, args.int_mode, world))
        traffic = pmc.get("bytes_per_launch")
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
                       "homes_total": n_total, "homes_per_gpu": agg.batch.N, "global_batch": n_total,
                       "horizon": H, "mix": "40/20/20/20 base/pv/battery/pv_battery",
                       "parallelism": f"homes sharded x{world}"},
            "sim_wall_s": elapsed,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": 8000.0, "unit": "GB/s",
                         "frac": achieved / 8000.0,
                         "traffic": (traffic / (kern_ms * 1e-3) / 1e9) if traffic else None,
                         "traffic_bytes_per_launch": traffic, "traffic_source": traffic_src,
                         "kernel": (f"mpc_direct_kernel (DM_FRONT + DM_BUCKET launches of a step)"
                                    if args.int_mode == "round" else "mpc_home_kernel"),
                         "kernel_ms": kern_ms},
            "cpu_baseline": cpu,
            "status_counts": stat_counts,
            # RL: the headline counts the rollout re-solves too; the committed steps alone:
            "committed_solves_per_s": n_total * args.steps / elapsed,
        }
        out.update(extra_rooflines(pmc, kern_ms, agg.batch.lib.dragg_mpc_lds_bytes(ctypes.byref(agg.batch.dims)),
                                   traffic_src))
        print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
