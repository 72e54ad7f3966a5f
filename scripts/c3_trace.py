"""Diagnostic: the C3 call (HHFM k=64 bf16 table, Frappe catalog, 3,000
queries, top-20) and the reference-shape 300-query call, 20 times each, for a
rocprofv3 kernel trace (scripts/c3_trace.sh).  Prints the event-timed medians."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hhfm_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(2)
nu, ni, k = 957, 4082, 64
M = nu + ni + 12
E = (torch.randn(M, k, generator=g, device=dev) * 0.01).to(torch.bfloat16)
res = {}
for B in (3000, 300):
    cols = [torch.randint(0, nu, (B,), generator=g, device=dev),
            torch.randint(nu, nu + ni, (B,), generator=g, device=dev)]
    off = nu + ni
    for c in (7, 2, 3):
        cols.append(torch.randint(off, off + c, (B,), generator=g, device=dev))
        off += c
    A = torch.stack(cols, 1).to(torch.int32).contiguous()
    fn = lambda: ops.catalog_topk(A, E, ops.MODE_HHFM, 20, nu, ni, 0, None, 0, (2, 5), (0, 0))  # noqa
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    res[f"B{B}_us"] = {"median": float(np.median(ts)) * 1e3, "min": float(np.min(ts)) * 1e3}
print(json.dumps(res))
