"""Diagnostic (not product, not a test): run the wide DeepFM ITEM kernel of
whatever hhfm_amd is first on PYTHONPATH on fixed seeded inputs and save the
outputs, so builds of dfm_wide.hip at different (RT, NWV, knock-out) settings
can be compared bit for bit (a row's score never depends on its block).
  python scripts/diag/wide_probe.py OUT.npz"""
import sys

import numpy as np
import torch

from hhfm_amd import ops
from hhfm_amd.DFM import DeepFM

out = {}
for k, layers, B, grouped in [(64, [150] * 3, 777, False), (64, [150] * 3, 20000, True),
                              (256, [400] * 3, 3000, False), (256, [400] * 3, 82000, True)]:
    rng = np.random.default_rng(k + B)
    nu, ni, ctx = 957, 4082, (7, 2, 3)
    M = nu + ni + sum(ctx)
    m = DeepFM(nu, ni, M, 5, k, layers, None, 0.01, 0, 0.01, mlp_dtype=torch.bfloat16,
               table_dtype=torch.bfloat16)
    cols = [rng.integers(0, nu if grouped else M, B), rng.integers(nu, nu + ni, B)]
    off = nu + ni
    for c in ctx:
        cols.append(rng.integers(off, off + c, B) if grouped else rng.integers(0, M, B))
        off += c
    X = np.stack(cols, 1).astype(np.int32)
    Wt, bs, dims, Wpd, bpd = m._prepared()
    wb = m.weights["feature_bias"].reshape(-1)
    xd = torch.from_numpy(X).cuda()
    for name, plan in (("wide", 0), ("narrow", ops.PLAN_NARROW)):
        y = ops.dfm_forward(xd, m.table, wb, Wt, bs, dims, torch.bfloat16, Wpd, bpd,
                            proj="item", plan=plan).cpu().numpy()
        out[f"k{k}_B{B}_{name}"] = y
np.savez(sys.argv[1], **out)
print("saved", sys.argv[1], sorted(out))
