#!/usr/bin/env python3
"""profiles/<round>/traffic.json from the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of
tools/gpu_profile.sh: HBM bytes per launch of the solver kernel = (2 x FETCH_SIZE +
WRITE_SIZE) x 1024 (MI355X_MICROARCH.md §HBM: FETCH_SIZE counts half of a streaming read on
gfx950; our reads are narrow, so the factor is an upper estimate).  Also the SQ counters of
the sq1 / sq2 passes per launch (VALU/LDS/SALU instruction counts, wave cycles in quad-cycles),
from which bench.py prices the kernel against the VALU issue rate."""
import argparse
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def per_dispatch(path, counter, kernel_sub):
    """Per solver STEP: the step's launches (DM_FRONT and the DM_BUCKET second launch, both named
    mpc_direct_kernel) summed, averaged over the steps (= the DM_FRONT dispatches) -- the unit
    bench.py times with its events around run_iteration."""
    vals, first = {}, set()
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and kernel_sub in r["Kernel_Name"]:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
            if "<false, 0>" in r["Kernel_Name"] or "<true, 0>" in r["Kernel_Name"] or "direct" not in kernel_sub:
                first.add(r["Dispatch_Id"])
    steps = max(1, len(first) or len(vals))
    return sum(vals.values()) / steps, steps


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
    ap.add_argument("--kernel", default="mpc_direct_kernel")
    a = ap.parse_args()
    from bench import traffic_key
    fetch, nf = per_dispatch(os.path.join(a.prof, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE", a.kernel)
    write, nw = per_dispatch(os.path.join(a.prof, "write", "write_counter_collection.csv"), "WRITE_SIZE", a.kernel)
    out = {"workload": traffic_key(a.homes, a.horizon, a.dt, a.month, a.int_mode, a.world),
           "kernel": a.kernel, "dispatches": [nf, nw],
           "fetch_size_kb_per_launch": fetch, "write_size_kb_per_launch": write,
           "bytes_per_launch": (2.0 * fetch + write) * 1024.0,
           "formula": "(2 x FETCH_SIZE + WRITE_SIZE) x 1024, rocprofv3 --pmc, separate passes"}
    sq = {}
    for p in ("sq1", "sq2", "sq3", "sq4"):
        f = os.path.join(a.prof, p, f"{p}_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for c in sorted({r["Counter_Name"] for r in csv.DictReader(open(f))}):
            sq[c] = per_dispatch(f, c, a.kernel)[0]
    if sq:
        out["sq_per_launch"] = sq
    fs = os.path.join(a.prof, "front_stats.json")
    if os.path.exists(fs):
        with open(fs) as f:
            out["front_stats"] = json.load(f)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
