"""Diagnostic: where the C3 reference call's time goes on the host.
Host-timed back-to-back calls (as bench.py's reference_call_300_queries_us)
of: ops.catalog_topk at 300 / 3,000 queries (default plan, fused plan, STORE
plan); the same C-ABI call with every Python-side step hoisted out of the
loop (outputs, workspace and stream preallocated); one trivial launch
(topk_merge over one query) for the per-launch floor; and the Python pieces
(torch.empty, current_stream) alone.  Prints one JSON line."""
import json
import os
import sys
import time

import torch

sys.path.append(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hhfm_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(2)
nu, ni, k = 957, 4082, 64
M = nu + ni + 12
E = (torch.randn(M, k, generator=g, device=dev) * 0.01).to(torch.bfloat16)


def batch(B):
    cols = [torch.randint(0, nu, (B,), generator=g, device=dev),
            torch.randint(nu, nu + ni, (B,), generator=g, device=dev)]
    off = nu + ni
    for c in (7, 2, 3):
        cols.append(torch.randint(off, off + c, (B,), generator=g, device=dev))
        off += c
    return torch.stack(cols, 1).to(torch.int32).contiguous()


def host_us(fn, n=400):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def event_us(fn, n=200):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / n * 1e3


nat = ops.native()
st = torch.cuda.current_stream().cuda_stream
res = {}
for B in (300, 3000):
    A = batch(B)
    ws = ops._catalog_workspace(dev, st, nat.catalog_topk_workspace(B, ni, k, 20))
    os_ = torch.empty(B, 20, dtype=torch.float32, device=dev)
    oi_ = torch.empty(B, 20, dtype=torch.int32, device=dev)
    for name, plan in (("default", 0), ("fused", ops.PLAN_FUSED), ("store", ops.PLAN_STORE)):
        def full(plan=plan):
            return ops.catalog_topk(A, E, ops.MODE_HHFM, 20, nu, ni, 0, None, 0, (2, 5),
                                    (0, 0), plan=plan)

        def raw(plan=plan):
            nat.catalog_topk(A.data_ptr(), B, 5, ops.MODE_HHFM, 0, 2, 5, 0, 0, E.data_ptr(),
                             M, k, 1, 0, nu, ni, 0, 20, os_.data_ptr(), oi_.data_ptr(),
                             ws.data_ptr(), ws.numel(), plan, 0, st)
        res[f"B{B}_{name}"] = {"ops_host_us": host_us(full), "raw_host_us": host_us(raw),
                               "raw_event_us": event_us(raw)}
s1 = torch.zeros(1, 1, 20, device=dev)
i1 = torch.zeros(1, 1, 20, dtype=torch.int32, device=dev)
o1 = torch.empty(1, 20, device=dev)
p1 = torch.empty(1, 20, dtype=torch.int32, device=dev)
res["one_launch_host_us"] = host_us(
    lambda: nat.topk_merge(s1.data_ptr(), i1.data_ptr(), 1, 1, 20, o1.data_ptr(), p1.data_ptr(),
                           st))
res["one_launch_event_us"] = event_us(
    lambda: nat.topk_merge(s1.data_ptr(), i1.data_ptr(), 1, 1, 20, o1.data_ptr(), p1.data_ptr(),
                           st))
res["two_empty_host_us"] = host_us(
    lambda: (torch.empty(300, 20, device=dev), torch.empty(300, 20, dtype=torch.int32,
                                                            device=dev)))
res["current_stream_host_us"] = host_us(lambda: torch.cuda.current_stream(dev).cuda_stream)
print(json.dumps(res))
