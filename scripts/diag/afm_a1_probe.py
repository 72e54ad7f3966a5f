#!/usr/bin/env python3
"""Diagnostic: why A1 times differ between scripts/afm_rows_ab.py and the
model-weight scripts (afm_phases.py, rowtable.py): the same 1 M Frappe rows
timed with the AFM model's weights and with random weights, interleaved."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from hhfm_amd import ops  # noqa: E402
from hhfm_amd.AFM import AFM  # noqa: E402

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
Wt, b, p_, P = m._att()
w = m.weights["feature_bias"].reshape(-1)
E = m.table
Er = (torch.randn(M, 64, generator=g, device=dev) * 0.01)
Wr = torch.randn(64, 64, generator=g, device=dev) * (2.0 / 128) ** 0.5
br = torch.randn(64, generator=g, device=dev) * (2.0 / 128) ** 0.5
pr = torch.randn(64, generator=g, device=dev)
out = torch.empty(B, device=dev)
cases = {"model": (E, Wt, b, p_), "rand_all": (Er, Wr, br, pr), "model_E_rand_att": (E, Wr, br, pr),
         "rand_E_model_att": (Er, Wt, b, p_)}
res = {n: [] for n in cases}
for _ in range(7):
    for n, (e, wt, bb, pp) in cases.items():
        ops.afm_forward(X, e, w, 0.0, wt, bb, pp, P, out=out)
        a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a0.record()
        ops.afm_forward(X, e, w, 0.0, wt, bb, pp, P, out=out)
        a1.record()
        a1.synchronize()
        res[n].append(a0.elapsed_time(a1))
print(json.dumps({n: sorted(v)[3] for n, v in res.items()}))
print(json.dumps({"E_model_absmax": float(E.abs().max()), "E_model_std": float(E.std()),
                  "b_model": [float(b.min()), float(b.max())], "p_model": [float(p_.min()), float(p_.max())],
                  "Wt_std": float(Wt.std())}))
