#!/usr/bin/env python3
"""Probe (diagnostic, not a product path): how much of K1's time at configs[1]
(FM k=64 fp32, 8M users + 8M items + 12 ctx, 2^25 rows) is the re-reading of
user rows that the batch references ~4 times each.  Times the shipped row
kernel over (a) the rows as given, (b) the same rows ordered by user id
(torch.sort, outside the timed region), (c) ordered by coarse user buckets,
and the torch sort / permute costs beside them.  Scores of (b) are checked
equal to (a) after un-permuting (every row's arithmetic is unchanged).
usage: python scripts/k1_bucket_probe.py [--reps N]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hhfm_amd import ops  # noqa: E402


def ms_of(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
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
    out = torch.empty(B, device=dev)
    res = {}
    res["given_ms"] = ms_of(lambda: ops.fm_score_rows(X, E, w, 0.0, out=out), a.reps)
    ref = out.clone()
    print(json.dumps(res), flush=True)
    for name, shift in (("user_exact", 0), ("user_b10", 10), ("user_b14", 14), ("user_b18", 18)):
        key = (X[:, 0] >> shift).long()
        ts = ms_of(lambda: torch.sort(key, stable=False), 3)
        _, perm = torch.sort(key, stable=False)
        Xs = X[perm].contiguous()
        tg = ms_of(lambda: X[perm], 3)
        outs = torch.empty(B, device=dev)
        res[name + "_ms"] = ms_of(lambda: ops.fm_score_rows(Xs, E, w, 0.0, out=outs), a.reps)
        back = torch.empty_like(outs)
        tsc = ms_of(lambda: back.index_copy_(0, perm, outs), 3)
        res[name + "_same_bits"] = bool(torch.equal(back, ref))
        res[name + "_torch_sort_ms"] = ts
        res[name + "_torch_gather_rows_ms"] = tg
        res[name + "_torch_scatter_out_ms"] = tsc
        print(json.dumps(res), flush=True)
        del Xs, perm, key
    print(json.dumps(res))


if __name__ == "__main__":
    main()
