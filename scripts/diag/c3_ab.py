"""Diagnostic A/B at the C3 shape (HHFM k=64 bf16 table, Frappe 4,082 items,
top-20): median call time (HIP events, 50 back-to-back calls after warm-up)
of the fused kernel path at 3,000 and 300 queries, and whether its top-20
ids and scores equal the score-matrix path's (HHFM_PLAN_STORE)."""
import json
import os
import sys

import torch

sys.path.append(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
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

    def run(plan):
        return ops.catalog_topk(A, E, ops.MODE_HHFM, 20, nu, ni, 0, None, 0, (2, 5), (0, 0),
                                plan=plan)
    ref = run(ops.PLAN_STORE)
    out = run(ops.PLAN_FUSED)
    same = bool(torch.equal(ref[0], out[0]) and torch.equal(ref[1], out[1]))
    for _ in range(200):
        run(ops.PLAN_FUSED)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(50)]
    for e0, e1 in ev:
        e0.record()
        run(ops.PLAN_FUSED)
        e1.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    res[f"B{B}"] = {"fused_us_median": ts[25], "fused_us_min": ts[0], "identical_to_store": same}
print(json.dumps(res))
