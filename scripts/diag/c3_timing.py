"""Diagnostic (with a HHFM_FUSED_TIMING=1 build first on PYTHONPATH): the
s_memtime phase marks of workgroup 0, wave 0 of the fused catalog kernel
(N = 1,024 items: one workgroup per 32 queries, so the marks land in the
first query's ids)."""
import json

import torch

from hhfm_amd import ops

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(2)
res = {}
for B in (32, 300, 3000):
    nu, ni, k = 957, 1024, 64
    M = nu + ni + 12
    E = (torch.randn(M, k, generator=g, device=dev) * 0.01).to(torch.bfloat16)
    cols = [torch.randint(0, nu, (B,), generator=g, device=dev),
            torch.randint(nu, nu + ni, (B,), generator=g, device=dev)]
    off = nu + ni
    for c in (7, 2, 3):
        cols.append(torch.randint(off, off + c, (B,), generator=g, device=dev))
        off += c
    A = torch.stack(cols, 1).to(torch.int32).contiguous()
    marks = []
    for rep in range(5):
        s, i = ops.catalog_topk(A, E, ops.MODE_HHFM, 20, nu, ni, 0, None, 0, (2, 5), (0, 0))
        marks.append(i[0, :11].tolist())
    res[f"B{B}"] = marks[-2:]
print(json.dumps(res))
