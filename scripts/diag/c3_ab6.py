"""Diagnostic A/B at the C3 shape: event-timed back-to-back calls of the
fused plan at 300 and 3,000 queries (C-ABI directly: the GPU time per call)."""
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
nat = ops.native()
st = torch.cuda.current_stream().cuda_stream
res = {}
for B in (300, 3000):
    cols = [torch.randint(0, nu, (B,), generator=g, device=dev),
            torch.randint(nu, nu + ni, (B,), generator=g, device=dev)]
    off = nu + ni
    for c in (7, 2, 3):
        cols.append(torch.randint(off, off + c, (B,), generator=g, device=dev))
        off += c
    A = torch.stack(cols, 1).to(torch.int32).contiguous()
    ws = ops._catalog_workspace(dev, st, nat.catalog_topk_workspace(B, ni, k, 20))
    os_ = torch.empty(B, 20, dtype=torch.float32, device=dev)
    oi_ = torch.empty(B, 20, dtype=torch.int32, device=dev)

    def run(plan):
        nat.catalog_topk(A.data_ptr(), B, 5, ops.MODE_HHFM, 0, 2, 5, 0, 0, E.data_ptr(), M, k,
                         1, 0, nu, ni, 0, 20, os_.data_ptr(), oi_.data_ptr(), ws.data_ptr(),
                         ws.numel(), plan, 0, st)
    run(ops.PLAN_STORE)
    ref = (os_.clone(), oi_.clone())
    run(ops.PLAN_FUSED)
    same = bool(torch.equal(ref[0], os_) and torch.equal(ref[1], oi_))
    for _ in range(50):
        run(ops.PLAN_FUSED)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(200):
        run(ops.PLAN_FUSED)
    b.record()
    b.synchronize()
    res[f"B{B}"] = {"us": a.elapsed_time(b) / 200 * 1e3, "identical_to_store": same}
print(json.dumps(res))
