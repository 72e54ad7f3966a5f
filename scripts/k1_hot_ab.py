#!/usr/bin/env python3
"""A/B (diagnostic): K1 at configs[1] (FM k=64 fp32, 8M users + 8M items +
12 ctx ids, 2^25 rows) with and without the hot-tail staging (hot_begin =
n_user + n_item: the 12 context rows and their w staged in LDS per
workgroup), interleaved in ONE process so box-to-box variance cancels;
asserts identical bits.  usage: python scripts/k1_hot_ab.py [--rounds N]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hhfm_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=9)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    nu = ni = 1 << 23
    M = nu + ni + 12
    B = 1 << 25
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    E = torch.empty(M, 64, device=dev).normal_(0, 0.01, generator=g)
    w = torch.empty(M, device=dev).normal_(0, 0.01, generator=g)
    cols = [torch.randint(0, nu, (B,), generator=g, device=dev),
            torch.randint(nu, nu + ni, (B,), generator=g, device=dev)]
    o = nu + ni
    for c in (7, 2, 3):
        cols.append(torch.randint(o, o + c, (B,), generator=g, device=dev))
        o += c
    X = torch.stack(cols, 1).to(torch.int32).contiguous()
    del cols
    outs = {v: torch.empty(B, device=dev) for v in ("plain", "hot")}
    hot = {"plain": None, "hot": nu + ni}
    for v in outs:
        ops.fm_score_rows(X, E, w, 0.0, out=outs[v], hot_begin=hot[v])
    torch.cuda.synchronize()
    assert torch.equal(outs["plain"], outs["hot"]), "hot staging changed bits"
    ts = {v: [] for v in outs}
    for _ in range(a.rounds):
        for v in outs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.fm_score_rows(X, E, w, 0.0, out=outs[v], hot_begin=hot[v])
            e1.record()
            e1.synchronize()
            ts[v].append(e0.elapsed_time(e1))
    res = {v: {"median_ms": float(np.median(t)), "min_ms": float(np.min(t))}
           for v, t in ts.items()}
    res["same_bits"] = True
    res["hot_vs_plain"] = res["hot"]["median_ms"] / res["plain"]["median_ms"]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
