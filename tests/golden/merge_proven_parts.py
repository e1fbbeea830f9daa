#!/usr/bin/env python3
"""Merge the parts of a proven-optimum reference run split by home -- TEST INFRASTRUCTURE, this
container only.

tests/golden/make_golden.py c1_h24_proven can run as K processes (GOLDEN_OWN = the home indices a
process proves, GOLDEN_PART = its file suffix): every process runs the reference's unmodified
Aggregator over the whole community, solving its own homes' MILPs to proven optimality (HiGHS,
mip_rel_gap 0) and the other homes' fast.  In run_rbo_mpc a home's closed loop depends on its own
solves only (aggregator.py:757-778: nothing flows back from the community sums), so each home's
records and results.json series are taken from the process that proved it, and the community
sums of the Summary (p_grid_aggregate = the sum of the homes' p_grid_opt, p_max_aggregate its
maximum; aggregator.py:751-753) are recomputed from the merged series.

Usage: python tests/golden/merge_proven_parts.py [--partial] NAME PART_FILE ...  -> tests/golden/proven/NAME.json.gz
(--partial: some parts did not finish; the fixture holds the homes of the parts given, and no
community sums)"""
import gzip
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    args = sys.argv[1:]
    partial = args[0] == "--partial"
    if partial:
        args = args[1:]
    name, files = args[0], args[1:]
    parts = [json.load(gzip.open(f, "rt")) for f in files]
    base = parts[0]
    names = [h["name"] for h in base["homes"]]
    for p in parts[1:]:
        assert [h["name"] for h in p["homes"]] == names and p["env"] == base["env"], "parts of different runs"
    owner = {}
    for k, p in enumerate(parts):
        for i in p["params"]["own"]:
            assert i not in owner, f"home {i} proven twice"
            owner[i] = k
    assert partial or sorted(owner) == list(range(len(names))), "every home must be proven by one part"
    records = sorted((r for k, p in enumerate(parts) for r in p["records"] if owner[r["home"]] == k),
                     key=lambda r: (r["t"], r["home"]))
    results = {names[i]: parts[owner[i]]["results"][names[i]] for i in sorted(owner)}
    summary = dict(base["results"]["Summary"])
    if partial:
        summary["p_grid_aggregate"] = summary["p_max_aggregate"] = None
    else:
        agg = np.sum([results[n]["p_grid_opt"] for n in names], axis=0)
        summary["p_grid_aggregate"] = agg.tolist()
        summary["p_max_aggregate"] = float(np.max(agg))
    summary["solve_time"] = None                    # (the parts ran concurrently)
    results["Summary"] = summary
    params = {k: v for k, v in base["params"].items() if k != "own"}
    params["parts"] = [p["params"]["own"] for p in parts]
    params["homes_proven"] = sorted(owner)
    out = dict(scenario=name, params=params, homes=base["homes"], records=records, results=results, env=base["env"])
    path = os.path.join(HERE, "proven", f"{name}.json.gz")
    with gzip.open(path, "wt") as f:
        json.dump(out, f, separators=(",", ":"))
    ms = [r["milp_status"] for r in records]
    print(f"{name}: {len(records)} records from {len(parts)} parts; HiGHS proven optimal {ms.count(0)}, "
          f"time-limited incumbents {ms.count(1)}, other {len(ms) - ms.count(0) - ms.count(1)} -> {path}")


if __name__ == "__main__":
    main()
