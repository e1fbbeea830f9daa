"""Diagnostic: with a build that marks DM_FRONT front overflows in the S_PAD slots
(1e7 + nn at the overflowing stage) and skips the second launch, report the first step with an
overflow and the overflowing front sizes.  DRAGG_LIB=... python tools/ovf_probe.py STEPS"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from dragg_amd.mpc import MPCBatch                                   # noqa: E402
from dragg_amd.community import synthetic_homes, synthetic_weather   # noqa: E402

STEPS = int(sys.argv[1])
N, HH, dt = 10000, 12, 4
H = HH * dt
homes = synthetic_homes(N, seed=12, days=4, dt=dt, horizon_hours=HH)
oat, ghi, tou = synthetic_weather(4, dt, 2 + STEPS // dt, seed=3, month=7)
b = MPCBatch(homes, oat, ghi, tou, 0, [0.0], int_mode="round", seed=12)
par = ((N * H * 336 * 2 + 255) // 256) * 256
for t in range(STEPS):
    b.step(t)
    torch.cuda.synchronize()
    x = b.workspace.view(torch.uint8)[par:par + N * 8 * H * 8].view(torch.float64).view(N, H, 8)[:, :, 7].cpu().numpy()
    m = x >= 1e7
    if m.any():
        hs, ks = np.nonzero(m)
        print(f"step {t}: {len(np.unique(hs))} homes overflow; first: " +
              ", ".join(f"home {h} stage {k} nn {x[h, k] - 1e7:.0f} prev {x[h, k - 1] if k else 0:.0f}" for h, k in list(zip(hs, ks))[:8]))
        break
else:
    print("no overflow")
