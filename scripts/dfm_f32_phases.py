#!/usr/bin/env python3
"""Diagnostic: the fp32-MLP DeepFM forward (projected layer 0; split-bf16
hidden layers, or exact fp32 with HHFM_DFM_F32_EXACT=1) at the C5 per-GPU
shape (F=5, k=256, 400-wide layers, Frappe vocabulary), by layer count
(2 = one hidden layer, 3 = two), rows grouped by user (default) or not
(HHFM_DFM_F32_GROUP=0).  Not part of the product; prints one JSON object."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hhfm_amd import ops  # noqa: E402
from hhfm_amd.DFM import DeepFM  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


dev = torch.device("cuda", 0)
nu, ni = 957, 4082
M = nu + ni + 12
B = int(os.environ.get("PH_ROWS", 1 << 21))
g = torch.Generator(device=dev)
g.manual_seed(4)
cols = [torch.randint(0, nu, (B,), generator=g, device=dev),
        torch.randint(nu, nu + ni, (B,), generator=g, device=dev)]
off = nu + ni
for c in (7, 2, 3):
    cols.append(torch.randint(off, off + c, (B,), generator=g, device=dev))
    off += c
X = torch.stack(cols, 1).to(torch.int32).contiguous()
res = {"rows": B}
for grp, waves in (("1", "8"), ("1", "4"), ("0", "8")):
    os.environ["HHFM_DFM_F32_GROUP"] = grp
    os.environ["HHFM_DFM_F32_WAVES"] = waves
    for layers in ([400, 400], [400, 400, 400]):
        m = DeepFM(nu, ni, M, 5, 256, layers, None, 0.01, 0, 0.0, device=dev)
        Wt, bs, dims, Wp, bp = m._prepared()
        out = torch.empty(B, device=dev)
        wb = m.weights["feature_bias"].reshape(-1)
        res[f"group{grp}_w{waves}_L{len(layers)}"] = timeit(
            lambda: ops.dfm_forward(X, m.table, wb, Wt, bs, dims, torch.float32, Wp, bp, out=out,
                                    proj=True))
print(json.dumps(res), flush=True)
