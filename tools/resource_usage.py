#!/usr/bin/env python3
"""Per-kernel VGPRs / scratch / occupancy of the library as the compiler reports them
(-Rpass-analysis=kernel-resource-usage on a throwaway build).  Usage: python tools/resource_usage.py [src]"""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "dragg_amd/csrc/mpc_kernel.hip"
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC", "-Wno-unused-function",
       "-Wno-unused-variable", "-mllvm", "-amdgpu-sched-strategy=iterative-ilp", "-Rpass-analysis=kernel-resource-usage",
       "-o", "/tmp/_ru.so", src]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in err.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|SGPRs): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split()[0]] = int(m.group(2))
for k, v in rows.items():
    if "kernel" in k:
        name = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", k)
        print(f"{name[:60]:60s} VGPR {v.get('VGPRs')} AGPR {v.get('AGPRs')} scratch {v.get('ScratchSize')} occ {v.get('Occupancy')}")
