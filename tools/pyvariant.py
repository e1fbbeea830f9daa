"""Build an experimental library variant from (old, new) text replacements (experiments only).
python tools/pyvariant.py NAME repl.py  -- repl.py defines R = [(old, new), ...]"""
import os
import runpy
import subprocess
import sys

name, spec = sys.argv[1], sys.argv[2]
SCHED = ["-mllvm", "-amdgpu-sched-strategy=" + (sys.argv[3] if len(sys.argv) > 3 else "iterative-ilp")]
R = runpy.run_path(spec)["R"]
src = open("dragg_amd/csrc/mpc_kernel.hip").read()
for o, n in R:
    assert o in src, o[:80]
    src = src.replace(o, n)
tmp = f"dragg_amd/csrc/_var_{name}.hip"
open(tmp, "w").write(src)
os.makedirs("varlib", exist_ok=True)
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC", "-Wno-unused-function",
       "-Wno-unused-variable", *SCHED, "-o", f"varlib/{name}.so", tmp]
r = subprocess.run(cmd, capture_output=True, text=True)
os.remove(tmp)
print(r.stderr[-2000:] if r.returncode else f"varlib/{name}.so")
