"""Diagnostic (with a HHFM_RING_TIMING=1 build first on PYTHONPATH): the
catalog_ring per-phase s_memtime sums at the C4 shard shape (HHFM k = 128,
1,024 queries x 1.25M items, top-20), fp32 and bf16 tables: cycles per
wave-tile in publish (vmcnt + barrier + staging issue), the MFMA chain up to
the ballots, and the selection; and the whole kernel per wave."""
import ctypes
import json
import os

import torch

from hhfm_amd import ops

lib = ctypes.CDLL(os.path.join(os.path.dirname(ops.__file__), "lib", "libhhfm.so"))
fn = lib.hhfm_debug_ring_timing
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
dev = torch.device("cuda", 0)
nu, N, k, B, K = 1 << 20, 1_250_000, 128, 1024, 20
g = torch.Generator(device=dev)
g.manual_seed(3)
E32 = torch.empty(nu + 12 + N, k, device=dev).normal_(0, 0.01, generator=g)
A = torch.stack([torch.randint(0, nu, (B,), generator=g, device=dev),
                 torch.zeros(B, dtype=torch.int64, device=dev),
                 nu + torch.randint(0, 7, (B,), generator=g, device=dev),
                 nu + 7 + torch.randint(0, 2, (B,), generator=g, device=dev),
                 nu + 9 + torch.randint(0, 3, (B,), generator=g, device=dev)],
                1).to(torch.int32).contiguous()
res = {}
buf = (ctypes.c_ulonglong * 8)()
for tname, E in (("fp32", E32), ("bf16", E32.to(torch.bfloat16))):
    def run():
        return ops.catalog_topk(A, E, ops.MODE_HHFM, K, nu + 12, N, 0, None, 0, (2, 5), (0, 0))
    for _ in range(20):
        run()
    torch.cuda.synchronize()
    assert fn(buf) == 0
    for _ in range(10):
        run()
    torch.cuda.synchronize()
    assert fn(buf) == 0
    t = list(buf)
    n = max(t[3], 1)
    res[tname] = {"publish_cyc_per_tile": t[0] / n, "mma_cyc_per_tile": t[1] / n,
                  "select_cyc_per_tile": t[2] / n, "wave_tiles": t[3] / 10,
                  "kernel_cyc_per_wave": t[4] / max(t[5], 1), "waves": t[5] / 10}
    print(json.dumps({tname: res[tname]}), flush=True)
print(json.dumps(res))
