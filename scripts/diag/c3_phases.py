"""Diagnostic (with a -DHHFM_DIAG_BUILD -DHHFM_FUSED_TIMING=1 build first on
PYTHONPATH): the fused small-catalog kernel's per-phase cycles (wave 0 of
every workgroup, s_memtime) at the C3 shape (HHFM k=64 bf16, Frappe 4,082
items, top-20) for 300, 2,048 and 3,000 queries: mean over the workgroups of
one call, the merging workgroups' hand-off + merge separately."""
import ctypes
import json
import os

import numpy as np
import torch

from hhfm_amd import ops

lib = ctypes.CDLL(os.path.join(os.path.dirname(ops.__file__), "lib", "libhhfm.so"))
rd, clr = lib.hhfm_debug_fused_timing, lib.hhfm_debug_fused_timing_clear
NWG, NM = 16384, 24
buf = (ctypes.c_ulonglong * (NWG * NM))()
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(2)
nu, ni, k = 957, 4082, 64
M = nu + ni + 12
E = (torch.randn(M, k, generator=g, device=dev) * 0.01).to(torch.bfloat16)
names = ["ids", "rows_hq", "bar_q", "b_operand", "scores", "offers", "bar_t1", "thr_sort", "bar_t2", "filter", "atomic", "appends", "bar_s", "compact", "sort32", "emit", "drain", "bar_h1", "counter_add", "bar_h2", "merge"]
for B in (300, 2048, 3000):
    cols = [torch.randint(0, nu, (B,), generator=g, device=dev),
            torch.randint(nu, nu + ni, (B,), generator=g, device=dev)]
    off = nu + ni
    for c in (7, 2, 3):
        cols.append(torch.randint(off, off + c, (B,), generator=g, device=dev))
        off += c
    A = torch.stack(cols, 1).to(torch.int32).contiguous()

    def run():
        return ops.catalog_topk(A, E, ops.MODE_HHFM, 20, nu, ni, 0, None, 0, (2, 5), (0, 0),
                                plan=ops.PLAN_FUSED)
    for _ in range(30):
        run()
    torch.cuda.synchronize()
    clr()
    run()
    torch.cuda.synchronize()
    rd(buf)
    t = np.frombuffer(buf, dtype=np.uint64).reshape(NWG, NM).astype(np.float64)
    t = t[t[:, 23] == 1]
    mg = t[:, 22] == 1
    d = np.diff(t[:, :22], axis=1)           # 21 intervals between marks 0..21
    res = {"workgroups": int(len(t)), "merging": int(mg.sum()),
           "cycles_mean_nonmerging": {n: round(float(d[~mg, i].mean())) for i, n in enumerate(names)}
           if (~mg).any() else None,
           "cycles_mean_merging": {n: round(float(d[mg, i].mean())) for i, n in enumerate(names)}
           if mg.any() else None,
           "total_max": float((t[:, 21] - t[:, 0]).max()),
           "start_spread": float(t[:, 0].max() - t[:, 0].min())}
    print(json.dumps({f"B{B}": res}), flush=True)
