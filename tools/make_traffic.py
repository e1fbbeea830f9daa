#!/usr/bin/env python3
"""profiles/<round>/traffic*.json from the rocprofv3 passes of ONE bench command (tools/gpu_profile.sh):
the kernel trace and the PMC passes (each counter group in its own run of the same command).

Only the TIMED steps count: the last `--steps` step groups of every pass (a step group = the hot
launch `mpc_direct_kernel<false, 0>` and the launches after it up to the next one, i.e. the
second launch of the same timestep; for the RL workload one action = forecast_horizon rollout
steps + the committed step).  Per step (per action for RL):
* kernel_ms_per_step: summed durations of the step group's launches (kernel trace);
* bytes_per_step: HBM bytes (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (MI355X_MICROARCH.md HBM section:
  FETCH_SIZE counts half of a streaming read on gfx950; our reads are narrow, so the factor is an
  upper estimate);
* sq_per_step: the SQ counters of the sq* passes;
* front_stats (optional, tools/front_stats.py on the same window): label relaxations per step.
bench.py uses the file only when its key names the same workload and timed window."""
import argparse
import csv
import gzip
import re
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _hot(name):
    """the hot launch (any waves-per-home instance) or the LP kernel"""
    return re.search(r"mpc_direct_kernel<false, 0[,>]", name) is not None or "mpc_home_kernel<false>" in name


def _ours(name):
    """the solver's launches: mpc_* kernels, the RL cell bound (cell_kernel), the lag mode's side hot launch"""
    return "mpc_" in name or "cell_kernel" in name or "side_front_kernel" in name


def step_groups(rows, n_units, per_unit):
    """rows: (dispatch_id, kernel_name, payload) of one pass.  -> the last n_units units, each a list
    of payloads (a unit = per_unit consecutive step groups)."""
    rows = sorted((r for r in rows if _ours(r[1])), key=lambda r: r[0])
    groups = []
    for d, name, pay in rows:
        if _hot(name) or not groups:
            groups.append([])
        groups[-1].append(pay)
    need = n_units * per_unit
    if len(groups) < need:
        raise SystemExit(f"only {len(groups)} step groups in the pass, {need} needed")
    groups = groups[-need:]
    return [sum(groups[u * per_unit:(u + 1) * per_unit], []) for u in range(n_units)]


def _open(path):
    """A raw pass CSV, or its gzipped copy (the committed raw passes of older rounds are gzipped)."""
    if not os.path.exists(path) and os.path.exists(path + ".gz"):
        return gzip.open(path + ".gz", "rt")
    return open(path)


def trace_ms(path, n_units, per_unit):
    """(mean, per-unit) kernel ms of the launches on the hot launch's stream, and the mean per unit of
    those on other streams (lag mode's side pass: it runs beside the main pass, so it is reported apart
    and not added; bench.py's HIP events time the main stream)"""
    rows = list(csv.DictReader(_open(path)))
    hot_streams = {r.get("Stream_Id") for r in rows if _hot(r["Kernel_Name"])}
    main, side = [], []
    for r in rows:
        t = (int(r["Dispatch_Id"]), r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
        (main if r.get("Stream_Id") in hot_streams else side).append(t)
    units = step_groups(main, n_units, per_unit)
    per = [sum(u) for u in units]
    side_ms = sum(t[2] for t in side if _ours(t[1])) / max(1, len(units))
    if side and not any(_ours(t[1]) for t in side):
        side_ms = 0.0
    return sum(per) / len(per), per, side_ms


def counters(path, n_units, per_unit):
    """{counter: mean per unit} over the last n_units units of a PMC pass."""
    by = {}
    for r in csv.DictReader(_open(path)):
        by.setdefault(r["Counter_Name"], []).append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    out = {}
    for c, rows in by.items():
        # a dispatch may report several rows of one counter (per XCD/instance): sum them first
        agg = {}
        for d, name, v in rows:
            agg.setdefault((d, name), 0.0)
            agg[(d, name)] += v
        units = step_groups([(d, n, v) for (d, n), v in agg.items()], n_units, per_unit)
        out[c] = sum(sum(u) for u in units) / len(units)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prof", default=os.path.join(ROOT, "gpurun_out", "prof"))
    ap.add_argument("--out", required=True)
    ap.add_argument("--homes", type=int, default=10000)
    ap.add_argument("--horizon", type=int, default=48)
    ap.add_argument("--dt", type=int, default=4)
    ap.add_argument("--month", type=int, default=7)
    ap.add_argument("--int-mode", default="round")
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--workload", default="rbo")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--rl-price", default="smooth")
    ap.add_argument("--forecast-horizon", type=int, default=1)
    ap.add_argument("--shard-of", type=int, default=0)
    ap.add_argument("--shard-rank", default=None, help="the rank of a --shard-of line, or max (--shard-max)")
    ap.add_argument("--steps-mode", default=None, choices=["lag", "serial", "adaptive"],
                    help="how the profiled command's steps ran (since round 6; unset: the key of rounds <= 5)")
    ap.add_argument("--command", default="")
    a = ap.parse_args()
    from bench import traffic_key
    rl = a.workload == "rl"
    fh = a.forecast_horizon if rl else 0
    per_unit = 1 + fh
    key = traffic_key(a.homes, a.horizon, a.dt, a.month, a.int_mode, a.world, a.workload, a.steps, a.warmup,
                      a.rl_price if rl else None, fh, a.shard_of,
                      (a.shard_rank if a.shard_rank == "max" else int(a.shard_rank)) if a.shard_of > 1 else None,
                      a.steps_mode)
    ms, per, side_ms = trace_ms(os.path.join(a.prof, "trace", "trace_kernel_trace.csv"), a.steps, per_unit)
    out = {"workload": key, "command": a.command, "unit": "action" if rl else "step",
           "kernel_ms_per_step": ms, "kernel_ms_per_step_min_max": [min(per), max(per)],
           "side_stream_kernel_span_ms_per_step": side_ms,
           "side_stream_note": "lag mode: summed start-to-end spans of the side pass launches, which run beside the main pass (a span includes the wait for dispatch slots), not added to kernel_ms_per_step"}
    f = counters(os.path.join(a.prof, "fetch", "fetch_counter_collection.csv"), a.steps, per_unit)["FETCH_SIZE"]
    w = counters(os.path.join(a.prof, "write", "write_counter_collection.csv"), a.steps, per_unit)["WRITE_SIZE"]
    out.update({"fetch_size_kb_per_step": f, "write_size_kb_per_step": w, "bytes_per_step": (2.0 * f + w) * 1024.0,
                "formula": "(2 x FETCH_SIZE + WRITE_SIZE) x 1024, rocprofv3 --pmc, separate passes"})
    sq = {}
    for p in ("sq1", "sq2", "sq3", "sq4"):
        fp = os.path.join(a.prof, p, f"{p}_counter_collection.csv")
        if os.path.exists(fp) or os.path.exists(fp + ".gz"):
            sq.update(counters(fp, a.steps, per_unit))
    if sq:
        out["sq_per_step"] = sq
    fs = os.path.join(a.prof, "front_stats.json")
    if os.path.exists(fs):
        with open(fs) as fh_:
            st = json.load(fh_)
        if st.get("window") == [a.warmup, a.warmup + a.steps]:
            out["front_stats"] = st
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as fh_:
        json.dump(out, fh_, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
