#!/usr/bin/env python3
"""Merge CPU-baseline parts of one workload run split by home over several GPU-box calls
(bench.py --cpu-only --cpu-home-range a:b, each part one call on the box's cores) into one record.

value = completed solves / (summed solve seconds / cores): the workload's throughput on `cores`
host cores when its solves are spread evenly over them (each part ran on the same core share).
Usage: python tools/merge_cpu_parts.py OUT.json PART.json ..."""
import json
import sys


def main(out, parts):
    P = [json.load(open(p)) for p in parts]
    cores = max(p["host_cores"]["max_jobs"] or p["cores"] for p in P)
    done = sum(p["done_home_steps"] for p in P)
    n = sum(p["home_steps"] for p in P)
    cpu_s = sum(p["solve_cpu_s"] for p in P)
    lim = sum(p["time_limited_solves"] for p in P)
    rec = {"value": done / (cpu_s / cores), "unit": "solves/s", "cores": cores, "kind": "port",
           "home_steps": n, "done_home_steps": done, "time_limited_solves": lim, "solve_cpu_s": cpu_s,
           "target_home_steps": sum(p["target_home_steps"] for p in P), "workload": P[0]["workload"],
           "extrapolated": True, "wall_s": sum(p["wall_s"] for p in P),
           "parts": [{k: p.get(k) for k in ("home_range", "home_steps", "done_home_steps", "time_limited_solves",
                                            "wall_s", "solve_cpu_s", "cores", "value")} for p in P],
           "median_solve_s": None,
           "sample": (f"{n} home-steps (the workload in full when they equal its target) split by home over "
                      f"{len(P)} GPU-box calls (bench.py --cpu-only --cpu-home-range), each on the box's "
                      f"{cores}-core share, solved by oracle/mpc.py (the reference's problem build, HiGHS MILP in "
                      f"place of GLPK_MI); {lim} solves reached the per-solve time limit and are not counted; "
                      f"value = {done} completed solves / ({cpu_s:.0f} solve-seconds / {cores} cores)")}
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps({k: rec[k] for k in ("value", "home_steps", "done_home_steps", "time_limited_solves")}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
