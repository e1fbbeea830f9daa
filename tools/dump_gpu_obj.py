#!/usr/bin/env python3
"""Solve every record of every golden fixture on the GPU (C ABI, solve_explicit) and save the
per-record status / objective / duties to gpurun_out/obj_<tag>_<scenario>.npz.

Diagnostic tool (GPU box): the files are compared offline against the proven optima
(tests/golden/proven_*.json.gz) without re-running the GPU."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from tests import fixtures as F
    from dragg_amd import _lib as L
    from dragg_amd.mpc import MPCBatch
    tag = sys.argv[1] if len(sys.argv) > 1 else "cur"
    mode = sys.argv[2] if len(sys.argv) > 2 else "round"
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    for name in F.scenarios():
        d = F.load(name)
        recs = d["records"]
        homes, ex = F.explicit_inputs(d, recs)
        b = MPCBatch(homes, int_mode=mode)
        fc, vals = F.prev_hash_arrays(recs, b.H, L.FC_KEYS, L.VAL_KEYS)
        b.fc.copy_(torch.tensor(fc))
        b.vals.copy_(torch.tensor(vals))
        b.solve_explicit(**ex)
        torch.cuda.synchronize()
        fcn = b.fc.cpu().numpy()
        np.savez_compressed(os.path.join(out, f"obj_{tag}_{name}.npz"), status=b.status.cpu().numpy(),
                            obj=b.obj.cpu().numpy(), fc=fcn, vals=b.vals.cpu().numpy(),
                            int_path=b.int_path.cpu().numpy())
        print(name, len(recs), "records", flush=True)


if __name__ == "__main__":
    main()
