#!/usr/bin/env python3
"""Joint-model verdicts for the solves the kernel declares ROUND_FAIL or solves approximately
(narrow feasible sets) -- TEST INFRASTRUCTURE, run in this container only.

Input: the cases tools/dump_cases.py dumped on the GPU box (every ROUND_FAIL solve of 100 steps of
the bench workload and of the configs[3] run, and every solve whose integer path used the bucketed
approximation because of a narrow feasible set), each with the inputs the oracle restates for it.

For each case the reference's FULL model (oracle/mpc.py build_problem: the reference's variables and
rows, `mpc_calc.py:291-446`, T and Tw coupled through e T_{k+1}) is given to HiGHS
(scipy.optimize.milp), nothing decomposed:
  * ROUND_FAIL: a FEASIBILITY problem (zero objective, integrality kept): HiGHS either finds an
    integer point (the joint MILP is feasible: the kernel's sequential T-then-Tw verdict would be
    wrong) or proves there is none -- independent of the sequential decomposition the kernel and
    oracle/thermal.py share;
  * narrow: the MILP with its objective to proven optimality (mip_rel_gap 0): the joint optimum
    the kernel's answer is compared with.
Verdicts whose HiGHS run hit the time limit are recorded as undecided (None).
Output: tests/golden/proven/round_fail_joint.json.gz (inputs + verdicts).

Usage: python tests/golden/make_round_fail_verdicts.py CASES.json [workers] [rf_time_limit] [narrow_time_limit]
       python tests/golden/make_round_fail_verdicts.py --from-journal [rf_time_limit] [narrow_time_limit]
         (writes the fixture from the verdicts journalled so far, e.g. after a run was cut short)"""
import gzip
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)


def decide(args):
    case, limits = args
    from scipy.optimize import milp, LinearConstraint, Bounds
    from oracle import mpc as M
    from oracle import thermal as TH
    hc = M.home_const(case["home"])
    si = M.StepInput(t=case["t"], T0=case["T0"], Tw0=case["Tw0"], E0=case["E0"], oat=np.asarray(case["oat"]),
                     ghi=np.asarray(case["ghi"]), price=np.asarray(case["price"]), draw=np.asarray(case["draw"]),
                     winter=case["winter"])
    P = M.build_problem(hc, si)
    cons = [LinearConstraint(P["A_eq"], P["b_eq"], P["b_eq"]), LinearConstraint(P["A_ub"], -np.inf, P["b_ub"])]
    rf = case["status"] == "round_fail"
    limit = limits[0] if rf else limits[1]
    c = np.zeros_like(P["c"]) if rf else P["c"]
    t0 = time.time()
    res = milp(c, constraints=cons, integrality=P["integrality"], bounds=Bounds(-np.inf, np.inf),
               options={"time_limit": limit, "mip_rel_gap": 0.0, "presolve": True})
    sec = time.time() - t0
    out = dict(case, highs_status=int(res.status), highs_seconds=sec)
    # 0 optimal (feasible point found / proven optimum), 2 infeasible (proven), 1 time limit
    if res.status == 2:
        out["joint_feasible"] = False
    elif res.status == 0:
        out["joint_feasible"] = True
    elif res.x is not None:
        out["joint_feasible"] = True                    # an integer point exists (incumbent)
    else:
        out["joint_feasible"] = None
    if res.x is not None:
        ii = P["integrality"] == 1
        x = res.x.copy()
        x[ii] = np.floor(x[ii] + 0.5)
        viol = max(float(np.abs(P["A_eq"] @ x - P["b_eq"]).max()), float((P["A_ub"] @ x - P["b_ub"]).max()))
        out["highs_violation"] = viol
        if not rf:
            out["joint_opt"] = float(P["c"] @ x) if res.status == 0 else None
            out["joint_bound"] = float(getattr(res, "mip_dual_bound", np.nan) or np.nan)
    seq = TH.thermal_optimum(hc, si)
    out["sequential_feasible"] = seq is not None
    out["sequential_opt"] = TH.exact_milp(hc, si, seq) if seq is not None else None
    return out


def write_fixture(res, limit, nlimit):
    res.sort(key=lambda r: (r["source"], r["t"], r["i"]))
    path = os.path.join(HERE, "proven", "round_fail_joint.json.gz")
    with gzip.open(path, "wt") as f:
        json.dump({"cases": res, "time_limit": limit, "narrow_time_limit": nlimit,
                   "note": "HiGHS on the reference's full model: round_fail = feasibility (zero objective), "
                           "narrow = proven optimum; joint_feasible None = undecided within the limit"}, f)
    n_rf = [r for r in res if r["status"] == "round_fail"]
    print(f"{len(res)} cases; round_fail: {sum(r['joint_feasible'] is False for r in n_rf)} jointly infeasible, "
          f"{sum(r['joint_feasible'] is True for r in n_rf)} jointly FEASIBLE, "
          f"{sum(r['joint_feasible'] is None for r in n_rf)} undecided -> {path}")


def main():
    if sys.argv[1] == "--from-journal":
        with open(os.path.join(HERE, "proven", "round_fail_joint.partial.jsonl")) as f:
            res = list({(r["source"], r["t"], r["i"]): r for r in map(json.loads, f)}.values())
        write_fixture(res, float(sys.argv[2]) if len(sys.argv) > 2 else 900.0,
                      float(sys.argv[3]) if len(sys.argv) > 3 else 120.0)
        return
    cases = json.load(open(sys.argv[1]))
    workers = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    limit = float(sys.argv[3]) if len(sys.argv) > 3 else 1800.0
    nlimit = float(sys.argv[4]) if len(sys.argv) > 4 else limit
    # every verdict is also appended to a journal as it arrives (a long run can be cut short)
    journal = open(os.path.join(HERE, "proven", "round_fail_joint.partial.jsonl"), "a")
    with mp.get_context("fork").Pool(workers) as pool:
        res = []
        for r in pool.imap_unordered(decide, [(c, (limit, nlimit)) for c in cases]):
            res.append(r)
            journal.write(json.dumps(r) + "\n")
            journal.flush()
            print(f"{r['source']} t={r['t']} i={r['i']} {r['status']}: joint feasible {r['joint_feasible']} "
                  f"(HiGHS {r['highs_status']}, {r['highs_seconds']:.1f}s), sequential {r['sequential_feasible']}",
                  flush=True)
    write_fixture(res, limit, nlimit)


if __name__ == "__main__":
    main()
