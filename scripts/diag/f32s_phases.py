"""Diagnostic (a HHFM_F32S_TIMING=1 build first on PYTHONPATH): the C5 fp32
DeepFM kernel dfm_fused_f32s per-phase s_memtime sums per wave and block —
ids + plan loads, item gather issue + spans + staging, layer-0 adds, hidden
layers, epilogue — at the bench's C5 shape (F=5, k=256, 3x400, Frappe
vocabulary, rows grouped by user), 2 M rows."""
import ctypes
import json
import os

import torch

from hhfm_amd import ops
from hhfm_amd.DFM import DeepFM

lib = ctypes.CDLL(os.path.join(os.path.dirname(ops.__file__), "lib", "libhhfm.so"))
fn = lib.hhfm_debug_f32s_timing
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
dev = torch.device("cuda", 0)
rows = 2_000_000
nu, ni, ctx = 957, 4082, (7, 2, 3)
M = nu + ni + sum(ctx)
g = torch.Generator(device=dev)
g.manual_seed(4)
cols = [torch.randint(0, nu, (rows,), generator=g, device=dev),
        torch.randint(nu, nu + ni, (rows,), generator=g, device=dev)]
off = nu + ni
for c in ctx:
    cols.append(torch.randint(off, off + c, (rows,), generator=g, device=dev))
    off += c
X = torch.stack(cols, 1).to(torch.int32).contiguous()
m = DeepFM(nu, ni, M, 5, 256, [400, 400, 400], None, 0.01, 0, 0.0, device=dev,
           mlp_dtype=torch.float32, table_dtype=torch.float32)
Wt, bs, dims, Wp, bp = m._prepared()
out = torch.empty(rows, device=dev)
wb = m.weights["feature_bias"].reshape(-1)


def step():
    ops.dfm_forward(X, m.table, wb, Wt, bs, dims, torch.float32, Wp, bp, out=out)


buf = (ctypes.c_ulonglong * 8)()
for _ in range(3):
    step()
torch.cuda.synchronize()
assert fn(buf) == 0
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    step()
e1.record()
torch.cuda.synchronize()
assert fn(buf) == 0
n = buf[5]
names = ["ids_plan", "gather_spans_staging", "layer0_adds", "hidden_layers", "epilogue"]
res = {"rows": rows, "ms_per_pass": e0.elapsed_time(e1) / 5, "wave_blocks": n,
       "cycles_per_wave_block": {k: buf[i] / max(n, 1) for i, k in enumerate(names)}}
print(json.dumps(res))
