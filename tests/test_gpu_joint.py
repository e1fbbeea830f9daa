"""ROUND_FAIL and narrow-set solves against the reference's FULL model, decided without the
sequential T-then-Tw decomposition the kernel and oracle/thermal.py share.

tests/golden/proven/round_fail_joint.json.gz holds every ROUND_FAIL solve of 100 steps of the bench
workload (BASELINE configs[2]) and of the configs[3] run, and every solve whose integer path used
the bucketed approximation (narrow feasible set), with the inputs the oracle restated for them on
the GPU box (tools/dump_cases.py) and HiGHS's verdict on the reference's whole MILP
(tests/golden/make_round_fail_verdicts.py: a zero-objective feasibility problem for ROUND_FAIL,
the proven optimum for the narrow cases).  The kernel re-solves each case from those explicit
inputs:
* status parity: ROUND_FAIL iff HiGHS proved the joint model infeasible, optimal iff it found an
  integer point (undecided cases are reported, not counted);
* narrow cases, solved with DRAGG_FLAG_EXACT (the step-function DP): the kernel's objective against
  HiGHS's proven joint optimum where HiGHS proved one within its limit."""
import gzip
import json
import os

import numpy as np
import pytest

from tests import fixtures as F

pytestmark = pytest.mark.gpu

PATH = os.path.join(F.GOLDEN, "proven", "round_fail_joint.json.gz")


def _cases():
    if not os.path.exists(PATH):
        pytest.skip("no joint-verdict fixture")
    with gzip.open(PATH, "rt") as f:
        return json.load(f)["cases"]


def _solve(cases, exact=False):
    """solve_explicit over the cases (one batch per horizon)."""
    import torch
    from dragg_amd.mpc import MPCBatch
    out = {}
    by_h = {}
    for j, c in enumerate(cases):
        by_h.setdefault(len(c["price"]), []).append(j)
    for H, idx in by_h.items():
        cs = [cases[j] for j in idx]
        b = MPCBatch([c["home"] for c in cs], int_mode="round", exact=exact)
        col = lambda k, n: np.array([np.asarray(c[k], float)[:n] for c in cs]).T  # noqa: E731
        b.solve_explicit(t=np.array([c["t"] for c in cs], np.int32), T0=[c["T0"] for c in cs],
                         Tw0=[c["Tw0"] for c in cs], E0=[np.nan if c["E0"] is None else c["E0"] for c in cs],
                         counter=np.array([c["counter"] for c in cs], np.int32),
                         winter=np.array([int(c["winter"]) for c in cs], np.int32), draw=col("draw", H + 1),
                         oat=col("oat", H + 1), ghi=col("ghi", H + 1), price=col("price", H))
        torch.cuda.synchronize()
        st, obj, path = b.status.cpu().numpy(), b.obj.cpu().numpy(), b.int_path.cpu().numpy()
        for k, j in enumerate(idx):
            out[j] = (int(st[k]), float(obj[k]), int(path[k]))
    return out


def test_round_fail_status_matches_the_joint_model(gpu):
    from dragg_amd import _lib as L
    cases = _cases()
    res = _solve(cases)
    n_inf = n_feas = n_und = 0
    for j, c in enumerate(cases):
        if c["status"] != "round_fail":
            continue
        st, obj, path = res[j]
        jf = c["joint_feasible"]
        if jf is None:
            n_und += 1
            continue
        if jf:
            n_feas += 1
            assert st == L.ST_OPTIMAL, (c["source"], c["t"], c["i"], L.STATUS_NAMES[st])
        else:
            n_inf += 1
            assert st == L.ST_ROUND_FAIL, (c["source"], c["t"], c["i"], L.STATUS_NAMES[st])
    print(f"ROUND_FAIL cases: {n_inf} proven jointly infeasible (kernel: ROUND_FAIL), {n_feas} jointly feasible "
          f"(kernel: optimal), {n_und} undecided by HiGHS within its limit")
    assert n_inf + n_feas > 0


def test_narrow_set_solves_against_the_joint_optimum(gpu):
    from dragg_amd import _lib as L
    cases = [c for c in _cases() if c["status"] != "round_fail"]
    if not cases:
        pytest.skip("no narrow-set case")
    res = _solve(cases, exact=True)            # DRAGG_FLAG_EXACT: the step-function DP
    gaps = []
    for j, c in enumerate(cases):
        st, obj, path = res[j]
        if c["joint_feasible"] is None:
            continue
        assert (st == L.ST_OPTIMAL) == bool(c["joint_feasible"]), (c["source"], c["t"], c["i"])
        if st == L.ST_OPTIMAL and c.get("joint_opt") is not None:
            g = (obj - c["joint_opt"]) / max(1.0, abs(c["joint_opt"]))
            assert g >= -1e-6, (c["source"], c["t"], c["i"], obj, c["joint_opt"])   # never below the optimum
            gaps.append(g)
    g = np.array(gaps)
    print(f"narrow-set cases: {len(cases)}; gap to HiGHS's proven joint optimum: max {g.max() if len(g) else 0:.2e}, "
          f"{int((g > 1e-6).sum())} above 1e-6")
    assert len(g) == 0 or g.max() <= 1e-6
