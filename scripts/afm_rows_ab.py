#!/usr/bin/env python3
"""A/B (diagnostic): AFM A1 (hhfm_afm_forward) at the row-table shape (1M
Frappe-shape rows, F = 5, k = A = 64, fp32 table): the pair-major kernel
(default plan) against the combo-packed afm_rows_fused (HHFM_PLAN_PER_FIELD)
and the exact-fp32 kernel, interleaved in one process; scores compared with
each other (max relative difference).  usage: python scripts/afm_rows_ab.py"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hhfm_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    res = {}
    for k, A, tdt in ((64, 64, torch.float32), (32, 32, torch.float32), (64, 64, torch.bfloat16)):
        nu, ni, ctx = 957, 4082, (7, 2, 3)
        M = nu + ni + sum(ctx)
        B = 1 << 20
        g = torch.Generator(device=dev)
        g.manual_seed(5)
        E = (torch.randn(M, k, generator=g, device=dev) * 0.01).to(tdt)
        w = torch.randn(M, generator=g, device=dev) * 0.01
        Wt = torch.randn(A, k, generator=g, device=dev) * (2.0 / (k + A)) ** 0.5
        b = torch.randn(A, generator=g, device=dev) * (2.0 / (k + A)) ** 0.5
        p = torch.randn(A, generator=g, device=dev)
        P = torch.ones(k, device=dev)
        cols = [torch.randint(0, nu, (B,), generator=g, device=dev),
                torch.randint(nu, nu + ni, (B,), generator=g, device=dev)]
        o = nu + ni
        for c in ctx:
            cols.append(torch.randint(o, o + c, (B,), generator=g, device=dev))
            o += c
        X = torch.stack(cols, 1).to(torch.int32).contiguous()
        plans = {"pairs": 0, "fused": ops.PLAN_PER_FIELD, "exact": ops.PLAN_EXACT_FP32}
        outs = {n: torch.empty(B, device=dev) for n in plans}
        for n, pl in plans.items():
            ops.afm_forward(X, E, w, 0.0, Wt, b, p, P, out=outs[n], plan=pl)
        torch.cuda.synchronize()
        ts = {n: [] for n in plans}
        for _ in range(rounds):
            for n, pl in plans.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.afm_forward(X, E, w, 0.0, Wt, b, p, P, out=outs[n], plan=pl)
                e1.record()
                e1.synchronize()
                ts[n].append(e0.elapsed_time(e1))
        ref = outs["exact"].double()
        tag = f"k{k}_A{A}_{'bf16' if tdt == torch.bfloat16 else 'f32'}"
        res[tag] = {n: {"median_ms": float(np.median(t)),
                        "max_abs_diff_vs_exact": float((outs[n].double() - ref).abs().max())}
                    for n, t in ts.items()}
        res[tag]["ref_abs_max"] = float(ref.abs().max())
        print(json.dumps({tag: res[tag]}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
