"""Diagnostic: DeepFM fused-kernel time by layer count (phase costs), C5
per-GPU shape (F=5, k=256, 400-wide layers), direct vs projected layer 0.
Not part of the product; prints one JSON object."""
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
if os.environ.get("PH_SORTSWAP"):   # experiment: rows grouped by user, item as field 0
    X = X[torch.argsort(X[:, 0], stable=True)][:, [1, 0, 2, 3, 4]].contiguous()
res = {}
for mdt in (torch.bfloat16,):
    for tdt in [torch.float32, torch.bfloat16][int(os.environ.get("PH_T0", 0)):]:
        for layers in [[400], [400, 400], [400, 400, 400]][int(os.environ.get("PH_L0", 0)):]:
            m = DeepFM(nu, ni, M, 5, 256, layers, None, 0.01, 0, 0.0, device=dev,
                       mlp_dtype=mdt, table_dtype=tdt)
            m.validate = False
            Wt, bs, dims, Wp, bp = m._prepared()
            out = torch.empty(B, device=dev)
            for pj in (False, True, "ctx", "item"):
                fn = lambda: ops.dfm_forward(X, m.table, m.weights["feature_bias"].reshape(-1),  # noqa
                                             Wt, bs, dims, mdt, Wp, bp, out=out, proj=pj)
                key = f"{'bf16' if mdt == torch.bfloat16 else 'f32'}mlp_{'tbf16' if tdt == torch.bfloat16 else 'tf32'}_L{len(layers)}_{ {False: 'direct', True: 'proj', 'ctx': 'ctx', 'item': 'item'}[pj] }"
                res[key] = round(timeit(fn), 4)
            del m
            torch.cuda.empty_cache()
print(json.dumps(res, indent=1))
