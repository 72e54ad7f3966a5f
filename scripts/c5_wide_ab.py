"""C5 bf16 leg (DeepFM F=5, k=256, 3x400, Frappe vocabulary, bf16 table and
MLP, ITEM plan) timed with the 192-row kernel (dfm_wide.hip) and with the
128-row one (HHFM_DFM_WIDE=0), alternating, plus the max difference between
the two on every row.  usage: python scripts/c5_wide_ab.py [rows] [reps]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    from hhfm_amd import ops
    from hhfm_amd.DFM import DeepFM
    dev = torch.device("cuda:0")
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
               mlp_dtype=torch.bfloat16, table_dtype=torch.bfloat16)
    Wt, bs, dims, Wp, bp = m._prepared()
    wb = m.weights["feature_bias"].reshape(-1)
    outs = {v: torch.empty(rows, device=dev) for v in ("wide", "old")}

    def step(v):
        os.environ["HHFM_DFM_WIDE"] = "1" if v == "wide" else "0"
        ops.dfm_forward(X, m.table, wb, Wt, bs, dims, torch.bfloat16, Wp, bp, out=outs[v])

    res = {}
    for v in ("wide", "old"):
        step(v)
    torch.cuda.synchronize()
    for rnd in range(2):
        for v in ("wide", "old"):
            ts = []
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                step(v)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            res.setdefault(v, []).append(min(ts))
            print(json.dumps({v: min(ts), "round": rnd}), flush=True)
    d = (outs["wide"] - outs["old"]).abs()
    mag = outs["old"].abs().max()
    print(json.dumps({"rows": rows, "ms_min": {v: min(t) for v, t in res.items()},
                      "max_abs_diff": float(d.max()), "max_abs_out": float(mag)}))


if __name__ == "__main__":
    main()
