#!/usr/bin/env python3
"""Benchmark: home-MPC solves/sec (homes x timesteps) of the batched MI355X solver.

Workload (BASELINE.json configs[1]): 1,000 homes (40 % base,
20 % pv_only, 20 % battery_only, 20 % pv_battery), run_rbo_mpc closed loop at 15-min
steps (dt = 4), 6 h horizon (H = 24), S = 6, discount 0.92, TOU prices; synthetic
NSRDB-shaped January weather and synthetic homes (no network for the reference data).
A "step" is one closed-loop timestep of the whole community: one launch of the
batched solver (every home's MPC solve + state advance) plus the aggregate reduction
(and, with N > 1 GPUs, the 24-byte RCCL all-reduce).  Homes shard across ranks
(weak scaling: --homes is per GPU).

Default: warmup 4 timesteps, then 96 timed timesteps (the full 24 h day) on 1 GPU.

Also reported (rank 0, N = 1 only): `cpu_baseline`, the repo's CPU restatement of the
reference solve (oracle/, HiGHS MILP in place of GLPK_MI) timed on this host's cores
on a bounded sample of the same workload, and `roofline` for the solver kernel.
"""
import argparse
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
    ap.add_argument("--homes", type=int, default=1000, help="homes per GPU")
    ap.add_argument("--horizon-hours", type=int, default=6)
    ap.add_argument("--dt", type=int, default=4)
    ap.add_argument("--int-mode", default="round", choices=["round", "relax", "round_lp"])
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--cpu-workers", type=int, default=0)
    return ap.parse_args()


# ----------------------------------------------------------------------------- CPU baseline
def _cpu_worker(args):
    """Closed-loop oracle solves for one home until the deadline (runs before any GPU use)."""
    home, env, deadline, milp_limit = args
    from oracle import mpc as M
    import numpy as np
    hc = M.home_const(home)
    hsh, n, t, times = {}, 0, 0, []
    rng = np.random.default_rng(1234)

    def solver(P):
        return M.solve_problem(P, integer=True, time_limit=milp_limit)
    while time.time() < deadline:
        t0 = time.time()
        try:
            M.run_home_step(hc, t, hsh, env, rng.standard_normal(hc.H), solver=solver)
        except Exception:
            break
        if time.time() > deadline + milp_limit:
            break
        times.append(time.time() - t0)
        n += 1
        t += 1
    return n, times


def cpu_baseline(homes, env, seconds, workers):
    import multiprocessing as mp
    import numpy as np
    cores = len(os.sched_getaffinity(0))
    workers = workers or max(1, min(16, cores))
    milp_limit = 10.0
    deadline = time.time() + seconds
    sample = [homes[(i * 7919) % len(homes)] for i in range(workers)]
    t0 = time.time()
    with mp.get_context("fork").Pool(workers) as pool:
        res = pool.map(_cpu_worker, [(h, env, deadline, milp_limit) for h in sample])
    wall = time.time() - t0
    n = sum(r[0] for r in res)
    times = [x for r in res for x in r[1]]
    return {"value": n / wall if wall > 0 else 0.0, "unit": "solves/s", "cores": workers, "kind": "port",
            "sample": f"{n} closed-loop home-steps of this workload ({workers} homes of the mix, one per "
                      f"process, t=0..) solved by oracle/mpc.py (reference problem build + HiGHS MILP "
                      f"standing in for GLPK_MI, time_limit {milp_limit:.0f}s/solve) in {wall:.1f}s wall; "
                      f"median {np.median(times) if times else float('nan'):.2f}s per solve"}


# ----------------------------------------------------------------------------- roofline
def bytes_per_step(batch, success_frac):
    """Algorithmic HBM bytes of one solver launch."""
    import numpy as np
    H, dt = batch.H, batch.dt
    types = batch.types_host
    n = len(types)
    rd = n * (22 * 8 + 4 + (H // dt + 1) * 8 + 6 * 8)            # params, type, draw window, hash state
    nfc = 10 + 2 * ((types & 1) != 0) + 3 * ((types & 2) != 0)   # forecast keys per home type
    wr = n * (19 * 8 + 4 + 4 + 8 + 8) + success_frac * float(np.sum(nfc)) * H * 8
    env = 3 * (H + 1) * 8
    return rd + wr + env


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
    n_total = args.homes * world
    homes = synthetic_homes(n_total, seed=12, days=days, dt=dt, horizon_hours=Hh)
    oat, ghi, tou = synthetic_weather(days, dt, sim_hours, seed=3)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        env = {"oat": oat, "ghi": ghi, "tou": tou, "start_hour_index": 0, "reward_price": [0.0]}
        cpu = cpu_baseline(homes, env, args.cpu_seconds, args.cpu_workers)

    import torch
    from dragg_amd.aggregator import DeviceAggregator
    torch.cuda.set_device(local)
    if world > 1:
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    agg = DeviceAggregator(homes, oat, ghi, tou, 0, total_steps, reward_price=[0.0],
                           int_mode=args.int_mode, seed=12, rank=rank, world=world, keep_history=False)
    stream = torch.cuda.current_stream()

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        agg.run_iteration()
        agg.collect_data()
    barrier()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        evs[k][0].record(stream)
        agg.run_iteration()
        evs[k][1].record(stream)
        agg.collect_data()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        torch.distributed.all_reduce(e, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(e.item())
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    st = agg.status_hist[args.warmup:total_steps].cpu()
    success = float((st == 0).float().mean())
    stat_counts = {name: int((st == i).sum()) for i, name in enumerate(
        ["optimal", "infeasible", "infeasible_cert", "max_iter", "round_fail", "err_parse", "err_missing"])}
    solves = n_total * args.steps
    value = solves / elapsed
    if rank == 0:
        achieved = bytes_per_step(agg.batch, success) / (kern_ms * 1e-3) / 1e9
        traffic = None
        tf = os.path.join(ROOT, "profiles", "traffic.json")
        if os.path.exists(tf):
            with open(tf) as f:
                tj = json.load(f)
            if tj.get("homes") == args.homes and tj.get("horizon") == agg.batch.H:
                traffic = tj.get("bytes_per_launch")
        out = {
            "metric": "home-MPC solves/sec (homes x steps)", "value": value, "unit": "solves/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic (NSRDB-shaped weather, config.toml-range homes)",
            "config": {"workload": f"{args.homes} homes/GPU x {args.steps} closed-loop 15-min steps, "
                                   f"H={agg.batch.H} (6 h), run_rbo_mpc, int_mode={args.int_mode}",
                       "homes_total": n_total, "global_batch": n_total, "horizon": agg.batch.H,
                       "mix": "40/20/20/20 base/pv/battery/pv_battery", "parallelism": f"homes sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": 8000.0, "unit": "GB/s",
                         "frac": achieved / 8000.0, "traffic": traffic,
                         "kernel": "mpc_home_kernel<false>", "kernel_ms": kern_ms},
            "cpu_baseline": cpu,
            "status_counts": stat_counts,
            "mean_admm_iters": float(agg.batch.iters.float().mean()),
        }
        print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
