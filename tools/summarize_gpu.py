#!/usr/bin/env python3
"""Print a short summary of the files tools/gpu_check.sh leaves in gpurun_out/."""
import glob
import json
import os
import re

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")


def last_json(path):
    for line in reversed(open(path).read().strip().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return None


log = os.path.join(OUT, "pytest_gpu.log")
if os.path.exists(log):
    txt = open(log).read()
    print([l for l in txt.splitlines() if re.search(r"passed|failed", l)][-1:])
    for l in txt.splitlines():
        if re.search(r"gap|bit-exact|battery LP|LP-optimal|worst violation|within 1e-3", l):
            print("  ", l.strip())
for f in sorted(glob.glob(os.path.join(OUT, "phase_*.json"))):
    d = json.load(open(f))
    print(os.path.basename(f), "kernel ms mean/max %.3f/%.3f" % (d["kernel_ms_mean"], d["kernel_ms_max"]),
          {k: int(v) for k, v in d["phase_mean_cycles"].items() if v}, "p50/max cycles",
          d["home_total_cycles_pct"]["50"], d["home_total_cycles_pct"]["100"], d["status_counts"])
for f in sorted(glob.glob(os.path.join(OUT, "bench*.log"))):
    d = last_json(f)
    if d:
        print(os.path.basename(f), "value %.0f ms/step %.3f kernel ms %.3f" % (d["value"], d["ms_per_step"],
              d["roofline"]["kernel_ms"]), d.get("status_counts"), "cpu", (d.get("cpu_baseline") or {}).get("value"))
