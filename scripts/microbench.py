#!/usr/bin/env python3
"""Kernel microbenchmarks (one process, HIP events, medians):
  K1 fm_score_rows  : bench workload with / without w, fp32 / bf16 table
  H1 hybrid rows    : same shape, HHFM layout
  K2 catalog_topk   : C3 (HHFM k=64 bf16, Frappe catalog, B=3000 = the 10
                      evaluate_TopK batches) and a C4 shard (k=128, 1.25 M
                      items, B=1024, K=20), fp32 and bf16
Prints one JSON object."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from hhfm_amd import ops  # noqa: E402
from hhfm_amd._native import native  # noqa: E402

dev = torch.device("cuda", 0)
nat = native()
st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
only = os.environ.get("MB_ONLY", "")


def timeit(fn, reps=10, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts)), float(np.min(ts))


res = {}
if not only or "k1" in only:
    rows = 1 << 25
    idx, E, w, M = bench.make_batch(rows, 8 << 20, 8 << 20, 64, 1, dev)
    out = torch.empty(rows, dtype=torch.float32, device=dev)
    res["k1_f32_w"] = timeit(lambda: ops.fm_score_rows(idx, E, w, 0.0, out=out))
    res["k1_f32_now"] = timeit(lambda: ops.fm_score_rows(idx, E, None, 0.0, out=out))
    res["h1_f32"] = timeit(lambda: ops.hybrid_score_rows(idx, E, 0, 1, (2, 5), (0, 0), out=out))
    Eb = E.to(torch.bfloat16)
    del E
    res["k1_bf16_w"] = timeit(lambda: ops.fm_score_rows(idx, Eb, w, 0.0, out=out))
    res["h1_bf16"] = timeit(lambda: ops.hybrid_score_rows(idx, Eb, 0, 1, (2, 5), (0, 0), out=out))
    del Eb, idx, w, out
    torch.cuda.empty_cache()

if not only or "k2" in only:
    g = torch.Generator(device=dev)
    g.manual_seed(2)
    for name, nu, ni, k, B, dt in [("c3_hhfm_k64_bf16", 957, 4082, 64, 3000, torch.bfloat16),
                                   ("c3_hhfm_k64_f32", 957, 4082, 64, 3000, torch.float32),
                                   ("c4_shard_k128_f32", 1 << 20, 1_250_000, 128, 1024, torch.float32),
                                   ("c4_shard_k128_bf16", 1 << 20, 1_250_000, 128, 1024, torch.bfloat16)]:
        M = nu + ni + 12
        E = (torch.randn(M, k, generator=g, device=dev) * 0.01).to(dt)
        cols = [torch.randint(0, nu, (B,), generator=g, device=dev),
                torch.randint(nu, nu + ni, (B,), generator=g, device=dev)]
        off = nu + ni
        for c in (7, 2, 3):
            cols.append(torch.randint(off, off + c, (B,), generator=g, device=dev))
            off += c
        A = torch.stack(cols, 1).to(torch.int32).contiguous()
        fn = lambda: ops.catalog_topk(A, E, ops.MODE_HHFM, 20, nu, ni, 0, None, 0, (2, 5), (0, 0))  # noqa
        med, mn = timeit(fn, reps=10)
        flops = 2.0 * B * ni * k
        res[name] = {"median_ms": med, "min_ms": mn, "TFLOPs": flops / (med * 1e-3) / 1e12,
                     "pairs_per_s": B * ni / (med * 1e-3)}
        del E
        torch.cuda.empty_cache()
if "topk" in only:   # dense top-K alone (C3 score-matrix shape), diagnostic leg
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    for name, B, N in [("topk_dense_3000x4082", 3000, 4082), ("topk_dense_300x4082", 300, 4082),
                       ("topk_dense_60x4082", 60, 4082)]:
        S = torch.randn(B, N, generator=g, device=dev) * 0.01
        med, mn = timeit(lambda: ops.topk_dense(S, 20), reps=20)
        res[name] = {"median_ms": med, "min_ms": mn}
if not only or "dfm" in only:
    # C5 per-GPU shape (DFM k=256, 3x400 MLP, Frappe-field rows), 2 M rows per launch
    from hhfm_amd.DFM import DeepFM
    nu, ni = 957, 4082
    M = nu + ni + 12
    B = 1 << 21
    g = torch.Generator(device=dev)
    g.manual_seed(4)
    cols = [torch.randint(0, nu, (B,), generator=g, device=dev),
            torch.randint(nu, nu + ni, (B,), generator=g, device=dev)]
    off = nu + ni
    for c in (7, 2, 3):
        cols.append(torch.randint(off, off + c, (B,), generator=g, device=dev))
        off += c
    X = torch.stack(cols, 1).to(torch.int32).contiguous()
    flops_row = 2.0 * (5 * 256 * 400 + 2 * 400 * 400) + 2.0 * (5 + 256 + 400)
    legs = [(torch.bfloat16, torch.float32, "dfm_c5_bf16"),
            (torch.bfloat16, torch.bfloat16, "dfm_c5_bf16_tbf16"),
            (torch.float32, torch.float32, "dfm_c5_f32")]
    if os.environ.get("MB_DFM_LEGS"):
        legs = [x for x in legs if x[2] in os.environ["MB_DFM_LEGS"].split(",")]
    # MB_DFM_PROJ: "0" direct layer 0 only, "1" every field projected only,
    # "auto" the library's choice only (bf16 MLP: ITEM; fp32 MLP: every field);
    # default all three
    projs = {"0": [False], "1": [True], "auto": [None]}.get(os.environ.get("MB_DFM_PROJ", ""),
                                                             [False, True, None])
    for mdt, tdt, name in legs:
        m = DeepFM(nu, ni, M, 5, 256, [400, 400, 400], None, 0.01, 0, 0.0, device=dev,
                   mlp_dtype=mdt, table_dtype=tdt)
        m.validate = False
        Wt, bs, dims, Wp, bp = m._prepared()
        outs = {}
        for pj in projs:
            out = torch.empty(B, device=dev)
            fn = lambda: ops.dfm_forward(X, m.table, m.weights["feature_bias"].reshape(-1),  # noqa
                                         Wt, bs, dims, mdt, Wp, bp, out=out, proj=pj)
            med, mn = timeit(fn, reps=5)
            leg = name + {False: "", True: "_proj", None: "_auto"}[pj]
            res[leg] = {"median_ms": med, "rows_per_s": B / (med * 1e-3),
                        "TFLOPs_reference_flops": flops_row * B / (med * 1e-3) / 1e12}
            outs[pj] = out
        if False in outs:
            for pj, suf in ((True, "_proj"), (None, "_auto")):
                if pj in outs:
                    res[name + suf]["max_abs_diff_vs_direct"] = \
                        (outs[pj] - outs[False]).abs().max().item()
                    res[name + suf]["out_abs_max"] = outs[False].abs().max().item()
        del m, outs
        torch.cuda.empty_cache()

if not only or "afm" in only:
    from hhfm_amd.AFM import AFM
    nu, ni, k = 957, 4082, 64
    M = nu + ni + 12
    m = AFM(nu, ni, M, 1, [k, k], None, 0.1, 100.0, [1, 1], "AdagradOptimizer", 0.999, 5,
            device=dev)
    m.validate = False
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    B = 1 << 20
    cols = [torch.randint(0, nu, (B,), generator=g, device=dev),
            torch.randint(nu, nu + ni, (B,), generator=g, device=dev)]
    off = nu + ni
    for c in (7, 2, 3):
        cols.append(torch.randint(off, off + c, (B,), generator=g, device=dev))
        off += c
    X = torch.stack(cols, 1).to(torch.int32).contiguous()
    Wt, b, p_, P = m._att()
    out = torch.empty(B, device=dev)
    med, mn = timeit(lambda: ops.afm_forward(X, m.table, m.weights["feature_bias"].reshape(-1),
                                             0.0, Wt, b, p_, P, out=out), reps=5)
    res["afm_rows_k64"] = {"median_ms": med, "rows_per_s": B / (med * 1e-3),
                           "TFLOPs": 2.0 * 10 * k * k * B / (med * 1e-3) / 1e12}
    A = X[:300]
    med, mn = timeit(lambda: ops.afm_catalog_topk(A, m.table, m.weights["feature_bias"].reshape(-1),
                                                  Wt, b, p_, P, nu, ni, 20), reps=5)
    res["afm_topk_c300_k64"] = {"median_ms": med,
                                "TFLOPs": 2.0 * 300 * ni * 4 * k * k / (med * 1e-3) / 1e12}

print(json.dumps(res, indent=1))
