#!/usr/bin/env python3
"""Exact thermal optima of every golden-fixture solve -- TEST INFRASTRUCTURE (this container).

For every record of tests/golden/*.json.gz and tests/golden/proven/*.json.gz, solves the
reference's thermal integer programme with oracle/thermal.py (assumption-free backward
step-function DP, itself pinned by tests/test_oracle_thermal.py against enumeration and HiGHS)
and writes tests/golden/proven/thermal_exact.json.gz: per scenario and record the exact
indoor-air and tank chain costs (None where a chain has no integer schedule), whether the
record's duty prices have one sign (where the GPU's Pareto-front DP applies), and the EXACT
optimum of the whole MILP ("opt_obj"): the reference model (oracle/mpc.py build_problem) with its
integer columns fixed to the exact thermal schedule, the rest (battery, PV, grid, cost) solved as
an LP by HiGHS (oracle/thermal.py exact_milp).  The MILP is separable (the battery and PV columns share
no row with the duty columns, only the linear objective), so this LP optimum is the MILP optimum;
tests/test_oracle_thermal.py checks that claim against every record HiGHS proved optimal.  The GPU test
tests/test_gpu_exact.py compares the kernel's integer solutions with these numbers, so the GPU
box needs neither the oracle run nor scipy.

Usage:  python tests/golden/make_thermal_exact.py [FIXTURE ...]
(FIXTURE: e.g. proven/c1_h24_proven -- only those fixtures are (re)computed and merged into the
existing output; records are solved in parallel, one process per host core)
"""
import glob
import gzip
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import mpc as M          # noqa: E402
from oracle import thermal as TH     # noqa: E402


def si_of(r):
    return M.StepInput(t=r["t"], T0=r["T0"], Tw0=r["Tw0"], E0=r["E0"], oat=np.array(r["oat"]),
                       ghi=np.array(r["ghi"]), price=np.array(r["total_price"]), draw=np.array(r["draw_size"]),
                       winter=r["season"] == "winter")


def solve_record(args):
    home, r = args
    hc = M.home_const(home)
    si = si_of(r)
    chT = TH.chain_T(hc, si)
    uniform = bool(np.all(chT["q"] >= 0) or np.all(chT["q"] <= 0))
    T = TH.solve_chain(chT)
    W = TH.solve_chain(TH.chain_W(hc, si, T[2])) if T is not None else None
    th = None if W is None else dict(u_T=T[1], u_W=W[1])
    return dict(uniform=uniform, cost_T=None if T is None else T[0], cost_W=None if W is None else W[0],
                opt_obj=TH.exact_milp(hc, si, th))


def main():
    import multiprocessing as mp
    files = sorted(glob.glob(os.path.join(HERE, "*.json.gz"))) + sorted(glob.glob(os.path.join(HERE, "proven", "h48_*.json.gz")))
    out = {}
    path = os.path.join(HERE, "proven", "thermal_exact.json.gz")
    if sys.argv[1:]:
        files = [os.path.join(HERE, f"{n}.json.gz") for n in sys.argv[1:]]
        with gzip.open(path, "rt") as f:
            out = json.load(f)
    pool = mp.get_context("fork").Pool(os.cpu_count())
    for path_in in files:
        path = path_in
        with gzip.open(path, "rt") as f:
            d = json.load(f)
        name = os.path.basename(path)[:-8]
        if path.startswith(os.path.join(HERE, "proven")):
            name = "proven/" + name
        homes = {h["name"]: h for h in d["homes"]}
        rows = pool.map(solve_record, [(homes[r["name"]], r) for r in d["records"]], chunksize=4)
        out[name] = rows
        n_ok = sum(1 for x in rows if x["cost_W"] is not None)
        print(f"{name}: {len(rows)} records, {n_ok} with an integer schedule", flush=True)
    path = os.path.join(HERE, "proven", "thermal_exact.json.gz")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with gzip.open(path, "wt") as f:
        json.dump(out, f, separators=(",", ":"))
    print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
