"""Diagnostic (with a -DHHFM_DIAG_BUILD -DHHFM_FUSED_TIMING=1 build first on PYTHONPATH): the
fused small-catalog kernel's per-phase cycles per wave (s_memtime sums over
every wave) at the C3 shape (HHFM k=64 bf16, Frappe 4,082 items, top-20) for
300 and 3,000 queries."""
import ctypes
import json
import os

import torch

from hhfm_amd import ops

lib = ctypes.CDLL(os.path.join(os.path.dirname(ops.__file__), "lib", "libhhfm.so"))
fn = lib.hhfm_debug_fused_timing
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(2)
nu, ni, k = 957, 4082, 64
M = nu + ni + 12
E = (torch.randn(M, k, generator=g, device=dev) * 0.01).to(torch.bfloat16)
buf = (ctypes.c_ulonglong * 8)()
names = ["query_phase", "scores", "threshold", "survivors", "range_sort"]
res = {}
for B in (300, 2048, 3000):
    cols = [torch.randint(0, nu, (B,), generator=g, device=dev),
            torch.randint(nu, nu + ni, (B,), generator=g, device=dev)]
    off = nu + ni
    for c in (7, 2, 3):
        cols.append(torch.randint(off, off + c, (B,), generator=g, device=dev))
        off += c
    A = torch.stack(cols, 1).to(torch.int32).contiguous()
    plan = ops.PLAN_FUSED

    def run():
        return ops.catalog_topk(A, E, ops.MODE_HHFM, 20, nu, ni, 0, None, 0, (2, 5), (0, 0),
                                plan=plan)
    for _ in range(30):
        run()
    torch.cuda.synchronize()
    fn(buf)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(20)]
    for e0, e1 in ev:
        e0.record()
        run()
        e1.record()
    torch.cuda.synchronize()
    fn(buf)
    t = list(buf)
    nw = max(t[5], 1)
    res[f"B{B}"] = {"cycles_per_wave": {n: t[i] / nw for i, n in enumerate(names)},
                    "waves_per_call": nw / 20, "merging_waves": t[6] / 20,
                    "merge_cycles_per_merging_wave": t[7] / max(t[6], 1),
                    "call_us_median": sorted(a.elapsed_time(b) for a, b in ev)[10] * 1e3}
    print(json.dumps({f"B{B}": res[f"B{B}"]}), flush=True)
