"""Diagnostic: AFM A1 rows (F=5 k=64 A=64, 1 M rows, fp32 table) and A2
catalog (300 queries x 4,082 items) kernel times.  Not part of the product;
prints one JSON object."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hhfm_amd import ops  # noqa: E402
from hhfm_amd.AFM import AFM  # noqa: E402


def timeit(fn, reps=7):
    """Median device time per call, calls queued back to back (host set-up
    overlaps the previous call instead of being timed as idle device time)."""
    fn()
    torch.cuda.synchronize()
    t_end = time.perf_counter() + 0.2   # >= 200 ms of the same work first: clocks ramp
    while time.perf_counter() < t_end:
        fn()
        torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return round(ts[len(ts) // 2], 4)


dev = torch.device("cuda", 0)
nu, ni = 957, 4082
M = nu + ni + 12
B = 1 << 20
g = torch.Generator(device=dev)
g.manual_seed(5)
cols = [torch.randint(0, nu, (B,), generator=g, device=dev),
        torch.randint(nu, nu + ni, (B,), generator=g, device=dev)]
off = nu + ni
for c in (7, 2, 3):
    cols.append(torch.randint(off, off + c, (B,), generator=g, device=dev))
    off += c
X = torch.stack(cols, 1).to(torch.int32).contiguous()
m = AFM(nu, ni, M, 1, [64, 64], None, 0.1, 100.0, [1, 1], "AdagradOptimizer", 0.999, 5,
        device=dev)
m.validate = False
Wt, b, p_, P = m._att()
w = m.weights["feature_bias"].reshape(-1)
out = torch.empty(B, device=dev)
res = {"A1_rows_1M": timeit(lambda: ops.afm_forward(X, m.table, w, 0.0, Wt, b, p_, P, out=out)),
       "A2_cat_300": timeit(lambda: ops.afm_catalog_topk(X[:300], m.table, w, Wt, b, p_, P,
                                                         nu, ni, 20))}
print(json.dumps(res))
