"""Diagnostic: the fused small-catalog kernel (catalog_fused.h, default
plan) against the score-matrix path (HHFM_PLAN_STORE) at the C3 shapes —
identical top-K ids and scores, and event-timed calls queued back to back
after a warm-up.  Prints one JSON object."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".") if "PYTHONPATH" not in __import__("os").environ else None
from hhfm_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
res = {}


def timeit(fn, reps=50):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3   # us per call


g = torch.Generator(device=dev)
g.manual_seed(2)
for B in (3000, 300):
    for dt in (torch.bfloat16, torch.float32):
        for mode in (ops.MODE_HHFM, ops.MODE_FM):
            nu, ni, k = 957, 4082, 64
            M = nu + ni + 12
            E = (torch.randn(M, k, generator=g, device=dev) * 0.01).to(dt)
            w = torch.randn(M, generator=g, device=dev) * 0.01
            cols = [torch.randint(0, nu, (B,), generator=g, device=dev),
                    torch.randint(nu, nu + ni, (B,), generator=g, device=dev)]
            off = nu + ni
            for c in (7, 2, 3):
                cols.append(torch.randint(off, off + c, (B,), generator=g, device=dev))
                off += c
            A = torch.stack(cols, 1).to(torch.int32).contiguous()
            wm = w if mode == ops.MODE_FM else None

            def run(plan):
                return ops.catalog_topk(A, E, mode, 20, nu, ni, 0, wm, 0, (2, 5), (0, 0),
                                        plan=plan)
            s0, i0 = run(ops.PLAN_STORE)
            s1, i1 = run(ops.PLAN_FUSED)
            same = bool(torch.equal(i0, i1) and torch.equal(s0, s1))
            name = f"B{B}_{'bf16' if dt == torch.bfloat16 else 'f32'}_{'hhfm' if mode else 'fm'}"
            res[name] = {"identical": same, "fused_us": timeit(lambda: run(ops.PLAN_FUSED)),
                         "store_us": timeit(lambda: run(ops.PLAN_STORE))}
            if not same:
                res[name]["ndiff_idx"] = int((i0 != i1).sum())
print(json.dumps(res, indent=1))
