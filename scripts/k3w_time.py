"""Diagnostic: time the C5 bf16 DeepFM forward (F=5, k=256, 3x400, Frappe
vocabulary, bf16 table and MLP, ITEM plan) with the library in hhfm_amd/lib;
used with scripts/build_variants.sh knock-out builds.  Prints one JSON line.
usage: python scripts/k3w_time.py [rows] [reps]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
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
    f32 = os.environ.get("K3W_F32") == "1"
    dt = torch.float32 if f32 else torch.bfloat16
    m = DeepFM(nu, ni, M, 5, 256, [400, 400, 400], None, 0.01, 0, 0.0, device=dev,
               mlp_dtype=dt, table_dtype=dt)
    m.validate = False
    Wt, bs, dims, Wp, bp = m._prepared()
    wb = m.weights["feature_bias"].reshape(-1)
    out = torch.empty(rows, device=dev)

    def step():
        ops.dfm_forward(X, m.table, wb, Wt, bs, dims, dt, Wp, bp, out=out)

    step()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        step()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    print(json.dumps({"rows": rows, "f32": f32, "ms_min": ts[0], "ms_med": ts[len(ts) // 2],
                      "out_sum": float(out.double().sum())}))


if __name__ == "__main__":
    main()
